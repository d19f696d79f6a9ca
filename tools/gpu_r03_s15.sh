#!/bin/bash
# Round-3 session 15: wave traces (tail-round phases) of the 10k scene, scene 0 and Cornell.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/wave_trace.py --scene 20 --spp 256 --bounces 16 > gpurun_out/wave_s20.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/wave_trace.py --scene 0 --spp 512 --bounces 16 > gpurun_out/wave_s0.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/wave_trace.py --scene 1 --spp 1024 --bounces 50 > gpurun_out/wave_s1.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/wave_s20.log | head -22
