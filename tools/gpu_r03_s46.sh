#!/bin/bash
# Final round-3 tree (tail priority for the mixed walk): pytest -m gpu, smoke, default bench + rocprof stats,
# then every BASELINE config + final_scene through bench.py and rocprof kernel stats of each config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PROFILE=1 bash tools/gpu_round.sh || exit $?
bash tools/gpu_r03_s42.sh || exit $?
echo done
