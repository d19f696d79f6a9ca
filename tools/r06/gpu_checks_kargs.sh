#!/bin/bash
# r06: the device-check builds (RT_CHECKS=1) with the kernarg re-read check: the GPU kernel tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/checks_kargs.txt 2>&1
rc=$?; tail -2 gpurun_out/r06/checks_kargs.txt; exit $rc
