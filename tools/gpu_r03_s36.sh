#!/bin/bash
# RT_PRIO_MIX on the other BASELINE scenes (frame hashes: every schedule gives the same frame)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step ab_pmix_s20 900 python3 tools/mixed_diag.py --scene 20 --width 1920 --height 1080 --spp 64 --bounces 16 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=32,RT_PRIO_TILES=8100" "RT_PRIO_MIX=1,RT_PRIO_LANES=16,RT_PRIO_TILES=8100" "" &&
step ab_pmix_s1 900 python3 tools/mixed_diag.py --scene 1 --width 1920 --height 1080 --spp 64 --bounces 50 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=32,RT_PRIO_TILES=8100" "" &&
step ab_pmix_s0 900 python3 tools/mixed_diag.py --scene 0 --width 1920 --height 1080 --spp 128 --bounces 16 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=32,RT_PRIO_TILES=8100" "" &&
step ab_pmix_s17 900 python3 tools/mixed_diag.py --scene 17 --width 1920 --height 1080 --spp 128 --bounces 50 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=32,RT_PRIO_TILES=8100" "" &&
step c6_final2 400 python3 bench.py --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1 --no-e2e
