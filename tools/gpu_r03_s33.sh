#!/bin/bash
# RT_PRIO_MIX sweep: final_scene (spp 16 and the bench's spp 64)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step ab_pmix2 1100 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=2048" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=4096" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=10000" "RT_PRIO_MIX=1,RT_PRIO_LANES=32,RT_PRIO_TILES=2048" "RT_PRIO_MIX=1,RT_PRIO_LANES=2,RT_PRIO_TILES=1024" "RT_PRIO_MIX=1,RT_PRIO_LANES=16,RT_PRIO_TILES=2048" "" &&
step ab_pmix64 1100 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 64 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=1024" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=2048" "RT_PRIO_MIX=1,RT_PRIO_LANES=16,RT_PRIO_TILES=2048"
