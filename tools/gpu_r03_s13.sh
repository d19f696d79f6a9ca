#!/bin/bash
# Round-3 session 13: every BASELINE config + final_scene through bench.py on the current tree (CPU
# baseline legs, end to end), then the PMC of the Perlin render kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WITH_FINAL=1 timeout -k 10 1000 bash tools/gpu_configs.sh || exit $?
timeout -k 10 200 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s17" --scene 17 --spp 1024 --bounces 50 --ppm > gpurun_out/pmc_s17.log 2>&1 || exit $?
echo done
