#!/bin/bash
# final_scene: costliest tiles' pixels capped per wave with ordinary tiles filling the other lanes (RT_PRIO_MIX)
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pyt_mix8 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed or cooperative_noise" &&
step ab_pmix 1100 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_PRIO_MIX=1,RT_PRIO_LANES=4,RT_PRIO_TILES=64" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=256" "RT_PRIO_MIX=1,RT_PRIO_LANES=16,RT_PRIO_TILES=1024" "RT_PRIO_MIX=1,RT_PRIO_LANES=8,RT_PRIO_TILES=1024" "RT_PRIO_MIX=1,RT_PRIO_LANES=4,RT_PRIO_TILES=256" ""
