#!/bin/bash
# A/B of the tail issue priority (RT_TAIL_PRIO=1) on every BASELINE config + final_scene, same box,
# alternating, 2 rounds each; frames hashed by the pixel-parity test afterwards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export VARIANTS="off|RT_TAIL_PRIO=0;on|RT_TAIL_PRIO=1" ROUNDS=2
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_tail_prio_s20.jsonl || exit $?
BENCH_ARGS="--scene 0 --spp 512 --bounces 16 --steps 5 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_tail_prio_s0.jsonl || exit $?
BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_tail_prio_s1.jsonl || exit $?
BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_tail_prio_s17.jsonl || exit $?
BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_tail_prio_s3.jsonl || exit $?
RT_TAIL_PRIO=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "baseline or catalog or verified or mixed" > gpurun_out/pytest_tail_prio.txt 2>&1 || { echo "pytest rc=$?"; tail -20 gpurun_out/pytest_tail_prio.txt; exit 1; }
tail -2 gpurun_out/pytest_tail_prio.txt
echo done
