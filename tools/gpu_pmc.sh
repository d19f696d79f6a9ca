#!/bin/bash
# PMC session (custom counter sets).  Each GPU step has its own limit; stop on fault/abort/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
if [ "${RUN_TESTS:-0}" = 1 ]; then
  step pytest_gpu 600 python3 -m pytest tests -q -m gpu -x
fi
if [ "${LIST:-0}" = 1 ]; then
  export TMPDIR=/tmp
  step counters_list 120 rocprofv3 -L
fi
step pmc 900 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc2" --sets "$PMC_SETS" $PMC_ARGS
tail -n 40 gpurun_out/pmc.log
