#!/bin/bash
# r05 s18: scene-20 mismatch vs spp and depth (frames saved)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s18
for c in "2 16" "4 16" "16 4" "16 8" "2 3"; do
  set -- $c
  timeout -k 10 120 python3 tools/r05/dbg20.py --spp $1 --bounces $2 --save gpurun_out/s18/spp$1_d$2 "def|" "notail|RT_JIT_OPTS=-DRT_NO_TAIL_CODE" \
    > gpurun_out/s18/spp$1_d$2.log 2>&1 || { echo "spp $1 d $2 failed"; exit 1; }
  echo "== spp $1 d $2"; grep -v amdgpu.ids gpurun_out/s18/spp$1_d$2.log
done
