#!/bin/bash
# r05 s17: scene-20 mismatch at 1 spp and shallow depths (frames saved for the analysis on the CPU side)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s17
for c in "1 16" "1 2" "1 1" "16 2" "16 1"; do
  set -- $c
  timeout -k 10 120 python3 tools/r05/dbg20.py --spp $1 --bounces $2 --save gpurun_out/s17/spp$1_d$2 "def|" "notail|RT_JIT_OPTS=-DRT_NO_TAIL_CODE" \
    > gpurun_out/s17/spp$1_d$2.log 2>&1 || { echo "spp $1 d $2 failed"; exit 1; }
  echo "== spp $1 d $2"; grep -v amdgpu.ids gpurun_out/s17/spp$1_d$2.log
done
