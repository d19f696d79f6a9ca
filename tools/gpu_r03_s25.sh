#!/bin/bash
# lazy sphere u,v (material-flagged) A/B on final_scene, alternating
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pyt_mix3 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed or earth or image" &&
step ab_lazyuv 900 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_LAZY_UV=0" "" "RT_LAZY_UV=0" ""
