#!/bin/bash
# r05 s14: scene-20 parity probe after s13's mismatch (test_tail_issue_priority_agrees[*-20-64-36-16]): the current
# library under several variants, and the last library whose full GPU suite passed (0c0b10e, ablib/librt_hip_r05s10.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/r05/dbg20.py "def|" "noprim|RT_ACCEL_PRIM=0" "sched1|RT_SCHED=1" "w0|RT_ACCEL_WAVES=0" \
  "rc16|RT_RC_LDS_LEVELS=16" "lane|RT_ACCEL=0" "nojitc|RT_JIT_CACHE_DIR=0" > gpurun_out/s14_new.log 2>&1; echo "new rc=$?"
cat gpurun_out/s14_new.log | grep -v amdgpu.ids
RT_HIP_LIB=$PWD/ablib/librt_hip_r05s10.so timeout -k 10 300 python3 tools/r05/dbg20.py "def|" "noprim|RT_ACCEL_PRIM=0" \
  > gpurun_out/s14_old.log 2>&1; echo "old rc=$?"
cat gpurun_out/s14_old.log | grep -v amdgpu.ids
