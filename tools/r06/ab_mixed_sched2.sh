#!/bin/bash
# r06: max-ilp now the mixed walk's default: the mixed parity tests, then default vs the compiler's default strategy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -m gpu -x -q -k "mixed or final" --timeout 300 --timeout-method thread > $O/mixsched_tests.txt 2>&1
rc=$?; tail -2 $O/mixsched_tests.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/mixsched_tests.txt | head; exit $rc; }
VARIANTS="ilp|RT_AB=0;def|RT_MIXED_SCHED=0" ROUNDS=3 LIM=300 \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 4 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_mixed_sched2.jsonl || exit 1
