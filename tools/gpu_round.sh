#!/bin/bash
# One GPU session: pytest -m gpu, smoke, bench, rocprofv3 kernel-trace stats.  Each GPU step has its
# own time limit; a fault/abort/timeout (rc not 0/1) stops the script before any further GPU work.
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
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" != 1 ]; then
  step pytest_gpu 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread ${PYTEST_ARGS:-}
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 900 python3 bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --pipelined-steps 0 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-}
fi
if [ "${PMC:-0}" = 1 ]; then
  step pmc 1000 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc" ${PMC_ARGS:---scene 0 --spp 512}
fi
tail -n 3 gpurun_out/*.log
