#!/bin/bash
# mixed-walk tests + PMC of rt_mixed_render on final_scene
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
step pytest_mixed 300 python3 -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread -k "mixed or texture"
step pmc_s3_mixed 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s3_mixed" --scene 3 --width 800 --height 800 --spp 16 --bounces 40
tail -3 gpurun_out/pytest_mixed.log
