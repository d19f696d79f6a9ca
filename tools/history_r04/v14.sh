#!/bin/bash
# r04 v14: the float 4-wide walk's random-world mismatch (r04 v10: test_wide_random_sphere_worlds_verified_walk
# [0-0], [3-0]) under variants — lists forced on, allocator's register budget, the other widths — then the 10k
# A/B of the list path (tools/r04/v13.sh).  -> profiles/r04_v14_wide_diag.txt, r04_ab_v13_10k.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T='tests/test_gpu_parity.py::test_wide_random_sphere_worlds_verified_walk'
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 300 python3 -u -m pytest "$T[0-0]" "$T[3-0]" "$T[0-1]" -q --timeout 120 --timeout-method thread > gpurun_out/wd_$label.log 2>&1
  local rc=$?
  echo "$label rc=$rc $(tail -1 gpurun_out/wd_$label.log)" | tee -a gpurun_out/wide_diag.txt
  [ $rc -gt 1 ] && exit $rc
  return 0
}
: > gpurun_out/wide_diag.txt
run default X=1
run lists_on RT_ACCEL_PRIM=1
run waves0 RT_ACCEL_WAVES=0
run waves5 RT_ACCEL_WAVES=5
run no_lds RT_ACCEL_LDS_NODES=0
bash tools/r04/v13.sh || exit $?
echo done
