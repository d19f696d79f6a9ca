#!/bin/bash
# final_scene with mixed hot waves: pause thresholds of the mixed walk (frame hashes)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step ab_defer2 1150 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_DEFER_TRACE=8" "RT_DEFER_TRACE=32" "RT_DEFER_TRACE=64" "RT_TRACE_MIN=4" "RT_TRACE_MIN=32" "RT_DEFER_TRACE=32,RT_TRACE_MIN=32" "RT_MIX_PAUSE=0" ""
