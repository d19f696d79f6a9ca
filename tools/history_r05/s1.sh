#!/bin/bash
# r05 s1: 4-wide 6-wave mismatch diagnosis (tools/r05/w4_diag.py) + a default bench line on this box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/w4
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
: > gpurun_out/steps.log
step w4_diag 400 python3 -u tools/r05/w4_diag.py --out gpurun_out/w4
step seedtab 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "stream_ordered or context_reuse or golden_frames or random_sphere_worlds_verified"
step bench 400 python3 bench.py --no-cpu-baseline
tail -n 30 gpurun_out/w4_diag.log
tail -n 4 gpurun_out/seedtab.log
tail -n 2 gpurun_out/bench.log
