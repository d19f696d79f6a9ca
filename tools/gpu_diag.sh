#!/bin/bash
# GPU diagnostics session: wave timeline + knob A/B.  Each GPU step has its own time limit; a
# fault/abort/timeout (rc not 0/1) stops the script before any further GPU work.
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
for sc in ${DIAG_SCENES:-0 1}; do
  step wt_s${sc} 180 python3 tools/wave_trace.py --scene $sc --spp ${DIAG_SPP:-512}
  [ "${DIAG_ROWMAJOR:-0}" = 1 ] && step wt_s${sc}_rowmajor 180 python3 tools/wave_trace.py --scene $sc --spp ${DIAG_SPP:-512} --env RT_SCHED=1
done
if [ -n "$DIAG_TUNE" ]; then
  step tune_knobs 300 python3 tools/tune.py --scene ${DIAG_TUNE_SCENE:-0} --spp 128 --rounds 3 --configs "$DIAG_TUNE"
fi
tail -n 30 gpurun_out/wt_*.log gpurun_out/tune_knobs.log 2>/dev/null
