#!/bin/bash
# mixed walk: next reference record prefetched a trip ahead — parity, then A/B (alternating)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pyt_mix4 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed" &&
step ab_pf 900 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_MIX_PREFETCH=1" "" "RT_MIX_PREFETCH=1" "" "RT_MIX_PREFETCH=1"
