#!/bin/bash
# final_scene schedule: probe density and split hot tiles (spp 16 and the bench's spp 64)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step ab_sched16 900 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_PROBE=32" "RT_PROBE=64" "RT_PRIO_LANES=64" "RT_PRIO_LANES=8,RT_PRIO_TILES=64" "RT_PRIO_LANES=16,RT_PRIO_TILES=256" "" &&
step ab_sched64 900 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 64 "" "RT_PROBE=64" "RT_PRIO_LANES=64" "RT_PRIO_LANES=16,RT_PRIO_TILES=256" ""
