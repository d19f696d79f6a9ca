#!/bin/bash
# r06: camera / tile-pickup kernel arguments re-read from the kernarg segment where used (RT_KARGS_RELOAD) instead of
# held in SGPRs across the render loop (scene 0: SGPR spills 27 -> 7, v_readlane / v_writelane 195 -> 57 static):
# the GPU parity suite with it compiled in, then same-box A/Bs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
RT_JIT_OPTS=-DRT_KARGS_RELOAD timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/kargs_tests.txt 2>&1
rc=$?; tail -2 $O/kargs_tests.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/kargs_tests.txt | head; exit $rc; }
V="def|RT_AB=0;kargs|RT_JIT_OPTS=-DRT_KARGS_RELOAD"
VARIANTS=$V ROUNDS=3 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_scene0.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_cornell.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_perlin.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_10k.jsonl || exit 1
