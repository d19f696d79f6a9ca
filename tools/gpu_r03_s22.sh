#!/bin/bash
# 168-VGPR mixed kernel: 2 blocks/CU (granule 16) vs 3 (granule 8), alternating
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step ab_gran 900 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_VGPR_GRANULE=8" "" "RT_VGPR_GRANULE=8" "RT_VGPR_GRANULE=8,RT_MIX_PAUSE=0"
