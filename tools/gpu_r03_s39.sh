#!/bin/bash
# final_scene wave trace with mixed hot waves; diag trip counters
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step wt_mix 300 python3 tools/wave_trace.py --scene 3 --width 800 --height 800 --spp 16 --bounces 40 &&
step diag_mix 300 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "RT_JIT_OPTS=-DRT_MIX_DIAG"
