#!/bin/bash
# RT_PRIO_MIX after the exhaustion fix: parity (incl. every tile costly), then a sweep with frame hashes
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pyt_mix9 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed or cooperative_noise" &&
step ab_pmix3 1100 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_PRIO_MIX=0" "RT_PRIO_TILES=1024" "RT_PRIO_TILES=4096" "RT_PRIO_TILES=10000" "RT_PRIO_LANES=4" "RT_PRIO_LANES=16" "" "RT_PRIO_MIX=0" &&
step ab_pmix_s20 900 python3 tools/mixed_diag.py --scene 20 --width 1920 --height 1080 --spp 64 --bounces 16 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=8100" "RT_PRIO_MIX=1,RT_PRIO_LANES=16,RT_PRIO_TILES=4000" "" &&
step ab_pmix_s1 900 python3 tools/mixed_diag.py --scene 1 --width 1920 --height 1080 --spp 64 --bounces 50 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=8100" "" &&
step ab_pmix_s0 900 python3 tools/mixed_diag.py --scene 0 --width 1920 --height 1080 --spp 128 --bounces 16 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=8100" "" &&
step ab_pmix_s17 900 python3 tools/mixed_diag.py --scene 17 --width 1920 --height 1080 --spp 128 --bounces 50 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=8100" ""
