#!/bin/bash
# mixed walk: chain pairs in one trip + quad inside tests skipped above the bound — parity, then A/B
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pyt_mix7 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed" &&
step ab_pair 1000 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_MIX_PAIR=0" "RT_JIT_OPTS=-DRT_MIX_OLD_DISPATCH" "" "RT_MIX_PAIR=0" "RT_JIT_OPTS=-DRT_MIX_OLD_DISPATCH" "" "RT_MIX_PAIR=0"
