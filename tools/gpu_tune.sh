#!/bin/bash
# GPU session: pytest -m gpu then traversal A/B (tools/tune.py) on a few scenes.  Each GPU step runs
# under its own time limit; a fault/abort/timeout (rc not 0/1) stops the script before further GPU work.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 600 python3 -m pytest tests -q -m gpu -x
fi
for sc in ${TUNE_SCENES:-0 1 17}; do
  step "tune_s$sc" 180 python3 tools/tune.py --scene "$sc" --spp "${TUNE_SPP:-32}" \
    --configs "${TUNE_CONFIGS:-RT_TRAVERSAL=0,RT_TRAVERSAL=1,RT_TRAVERSAL=2}" --rounds 3
done
tail -n 4 gpurun_out/*.log
