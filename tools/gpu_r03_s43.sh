#!/bin/bash
# Re-created container, final round-3 tree: pytest -m gpu, smoke, default bench, rocprof stats, then
# wave traces of scene 0 and the 10k scene (where the single frame's tail is).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PROFILE=1 bash tools/gpu_round.sh || exit $?
timeout -k 10 300 python3 tools/wave_trace.py --scene 0 --spp 512 > gpurun_out/wave_trace_scene0.txt 2>&1 || { echo "wt0 rc=$?"; exit 1; }
timeout -k 10 400 python3 tools/wave_trace.py --scene 20 --spp 256 > gpurun_out/wave_trace_scene20.txt 2>&1 || { echo "wt20 rc=$?"; exit 1; }
echo done
