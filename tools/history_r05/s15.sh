#!/bin/bash
# r05 s15: scene-20 mismatch, one pixel's colour-stack pushes and unwinds (RT_DBG_PX printf hooks) in the failing 6-wave
# build and the exact allocator-budget build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/r05/dbg20.py "def|" > gpurun_out/s15_def.log 2>&1; echo "def rc=$?"
grep -v amdgpu.ids gpurun_out/s15_def.log
timeout -k 10 200 python3 tools/r05/dbg20.py "dbg6|RT_JIT_OPTS=-DRT_DBG_PX=131102" > gpurun_out/s15_dbg6.log 2>&1; echo "dbg6 rc=$?"
timeout -k 10 200 python3 tools/r05/dbg20.py "dbg0|RT_JIT_OPTS=-DRT_DBG_PX=131102 RT_ACCEL_WAVES=0" > gpurun_out/s15_dbg0.log 2>&1; echo "dbg0 rc=$?"
grep -h "differing" gpurun_out/s15_dbg6.log gpurun_out/s15_dbg0.log
grep -c dbg gpurun_out/s15_dbg6.log gpurun_out/s15_dbg0.log
