#!/bin/bash
# r06: kernarg reloads now the default; the held form (RT_KARGS_HOLD) against it on the configs not yet compared, then
# the whole GPU suite on the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
V="reload|RT_AB=0;hold|RT_JIT_OPTS=-DRT_KARGS_HOLD"
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_4k.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_final.jsonl || exit 1
VARIANTS=$V ROUNDS=3 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs2_10k.jsonl || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/kargs_pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/kargs_pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/kargs_pytest_gpu.txt | head; exit $rc; }
