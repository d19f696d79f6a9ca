#!/bin/bash
# r06: the mixed walk's own kernel arguments (tree bases, pause knobs, proof / fallback words) read where used vs held
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
RT_JIT_OPTS= timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k mixed --timeout 300 --timeout-method thread > $O/kargs_mix_tests.txt 2>&1
rc=$?; tail -2 $O/kargs_mix_tests.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/kargs_mix_tests.txt | head; exit $rc; }
VARIANTS="mixk|RT_AB=0;hold|RT_JIT_OPTS=-DRT_KARGS_MIX_HOLD" ROUNDS=3 LIM=300 \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kargs_mix_final.jsonl || exit 1
