#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_MIXED=0" "RT_MIX_DYN_MIN=1000000" "" "RT_MIXED=0" > gpurun_out/mixed_diag.jsonl 2> gpurun_out/mixed_diag.err
rc=$?; cat gpurun_out/mixed_diag.jsonl; tail -5 gpurun_out/mixed_diag.err; exit $rc
