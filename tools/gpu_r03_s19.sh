#!/bin/bash
# final_scene diagnostics: mixed-walk trip/lane counters (RT_MIX_DIAG build) and the wave trace
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step mixdiag 400 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_JIT_OPTS=-DRT_MIX_DIAG" &&
step wtrace3 300 python3 tools/wave_trace.py --scene 3 --width 800 --height 800 --spp 16 --bounces 40
