#!/bin/bash
# mixed hot waves at the bench's spp 64 on final_scene (frame hashes)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step ab_pmix64b 1150 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 64 "" "RT_PRIO_MIX=0" "RT_PRIO_LANES=24" "RT_PRIO_LANES=48" "RT_PRIO_TILES=1024" "RT_PRIO_TILES=5000" "RT_PRIO_LANES=16,RT_PRIO_TILES=1250" ""
