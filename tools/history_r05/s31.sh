#!/bin/bash
# r05 s31: the relaxed pool test, then the scene-0 schedule sweep (s28)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -v -k "colour_stack_pool" --timeout 120 --timeout-method thread > gpurun_out/s31_pool.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/s31_pool.log
[ $rc -eq 0 ] || exit $rc
bash tools/r05/s28.sh
