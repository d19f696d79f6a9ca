#!/bin/bash
# r05 s5: which per-lane state carried across rounds does the v16 6-wave 4-wide mismatch need?  v16 at 6 waves on the
# two failing worlds with rejection deferral off (no pending lanes: random_test and the hit never wait a round), with
# walk pausing off (no paused walk state), both off, and v16 with only the kernel-entry span atomic replaced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s5_steps.log
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 -u tools/r05/w4_diag.py --seeds 1 4 --waves 6 --no-trace --reps 2 --out gpurun_out/w4s5_$label > gpurun_out/w4s5_$label.log 2>&1
  local rc=$?
  echo "$label rc=$rc" >> gpurun_out/s5_steps.log
  [ $rc -ne 0 ] && { tail -5 gpurun_out/w4s5_$label.log; exit $rc; }
  return 0
}
L16=$PWD/ablib/librt_hip_r04v16.so
run base RT_HIP_LIB=$L16
run nodefer RT_HIP_LIB=$L16 RT_DEFER_LANES=0
run nopause RT_HIP_LIB=$L16 RT_DEFER_TRACE=0
run neither RT_HIP_LIB=$L16 RT_DEFER_LANES=0 RT_DEFER_TRACE=0
run span RT_HIP_LIB=$PWD/ablib/librt_hip_r04v16_span.so
for f in gpurun_out/w4s5_*.log; do echo "== $f"; grep -v amdgpu.ids $f; done
