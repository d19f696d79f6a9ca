#!/bin/bash
# r06: kind-scheduled trips of the mixed walk (RT_MIX_KIND, one step class per trip): the mixed parity tests with it
# compiled in, then a same-box A/B on final_scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
RT_JIT_OPTS=-DRT_MIX_KIND=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k mixed \
  --timeout 300 --timeout-method thread > $O/mix_kind_tests.txt 2>&1
rc=$?; tail -2 $O/mix_kind_tests.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/mix_kind_tests.txt | head; exit $rc; }
VARIANTS="def|RT_AB=0;kind|RT_JIT_OPTS=-DRT_MIX_KIND=1" ROUNDS=3 LIM=300 \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" \
  bash tools/gpu_ab_env.sh $O/ab_mix_kind_final.jsonl || exit 1
