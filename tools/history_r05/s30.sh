#!/bin/bash
# r05 s30: full GPU suite on the tree with the 5-level deep unwind batch, then the scene-0 schedule sweep (s28)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/s30_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/s30_pytest_gpu.log; grep FAILED gpurun_out/s30_pytest_gpu.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/r05/s28.sh
