#!/bin/bash
# r05 s19: scene-20 mismatch — the failing 6-wave kernel with its SGPR spills in scratch instead of VGPR lanes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/r05/dbg20.py --spp 2 "def|" "w6|RT_ACCEL_WAVES=6" \
  "sgprmem|RT_ACCEL_WAVES=6 RT_JIT_OPTS=-mllvm+-amdgpu-spill-sgpr-to-vgpr=0" > gpurun_out/s19.log 2>&1; echo "rc=$?"
grep -v amdgpu.ids gpurun_out/s19.log
