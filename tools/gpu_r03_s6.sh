#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -40 "gpurun_out/$name.log" >&2; exit $rc; fi
}
step pytest_mixed 300 python3 -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread -k "mixed"
step mixed_diag 600 python3 tools/mixed_diag.py --scene 3 --size 800 --spp 16 "" "RT_MIXED=0" "" "RT_MIX_DYN_MIN=1000000"
cat gpurun_out/mixed_diag.log | cut -c1-300
