#!/bin/bash
# r06: every kernel argument used in the render loop re-read where used (except around the mixed walk) vs the camera /
# pickup re-reads only (RT_KARGS_LOOP_HOLD): the whole GPU suite on the new default, then same-box A/Bs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/kloop_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/kloop_pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/kloop_pytest_gpu.txt | head; exit $rc; }
V="loop|RT_AB=0;pickup|RT_JIT_OPTS=-DRT_KARGS_LOOP_HOLD"
VARIANTS=$V ROUNDS=3 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kloop_scene0.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kloop_cornell.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kloop_perlin.jsonl || exit 1
VARIANTS=$V ROUNDS=3 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kloop_10k.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kloop_4k.jsonl || exit 1
