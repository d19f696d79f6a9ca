#!/bin/bash
# r06: GPU suite + smoke + default bench on one box (each step under its own limit; the first failure stops)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${TAG:-check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" $O/pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt | tail -5; exit 1; }
tail -1 $O/smoke.txt
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
