#!/bin/bash
# r06: the mixed walk at 4 waves / SIMD without spills (slab offsets recomputed per macro step, a 16-VGPR raise) vs the
# first build at 3 (RT_JIT_RAISE=0): the mixed parity tests, the raise in the debug log, then a same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q -k "mixed or final" --timeout 300 --timeout-method thread > $O/mixraise_tests.txt 2>&1
rc=$?; tail -2 $O/mixraise_tests.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/mixraise_tests.txt | head; exit $rc; }
RT_DEBUG=1 timeout -k 10 300 python3 bench.py --scene 3 --width 800 --height 800 --spp 8 --bounces 40 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --pipelined-steps 0 > $O/mixraise_debug.json 2> $O/mixraise_debug.err || { tail -5 $O/mixraise_debug.err; exit 1; }
grep -i "raise\|rt_mixed" $O/mixraise_debug.err | head -5
VARIANTS="raise|RT_AB=0;noraise|RT_JIT_RAISE=0" ROUNDS=3 LIM=300 \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_mixed_raise.jsonl || exit 1
