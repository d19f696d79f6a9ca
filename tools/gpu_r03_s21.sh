#!/bin/bash
# residency of a 168-VGPR kernel at 3 blocks/CU (wave start stamps), and its frame time
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step wt_b3 300 python3 tools/wave_trace.py --scene 3 --width 800 --height 800 --spp 16 --bounces 40 --env RT_BLOCKS_PER_CU=3 &&
step ab_b3 900 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_BLOCKS_PER_CU=3" "RT_TRACE_MIN=4" "RT_BLOCKS_PER_CU=3,RT_TRACE_MIN=4" "" "RT_BLOCKS_PER_CU=3"
