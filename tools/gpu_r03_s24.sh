#!/bin/bash
# mixed walk: lazy sphere u,v + deferral of leaf / macro steps behind BVH steps — parity, then A/B
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pyt_mix2 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "mixed or earth or image or uv or sphere" &&
step ab_defer 1000 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_MIX_DEFER_LEAF=8" "RT_MIX_DEFER_LEAF=16" "RT_MIX_DEFER_LEAF=64" "RT_MIX_DEFER_MACRO=16" "RT_MIX_DEFER_LEAF=16,RT_MIX_DEFER_MACRO=16" "RT_MIX_DEFER_LEAF=64,RT_MIX_DEFER_MACRO=64" ""
