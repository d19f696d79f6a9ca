#!/bin/bash
# Round-3 final tree, part B: every BASELINE config + final_scene through bench.py, and rocprof kernel
# stats of every config's isolated frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WITH_FINAL=1 timeout -k 10 900 bash tools/gpu_configs.sh > gpurun_out/configs_run.log 2>&1 || { echo "configs rc=$?" >&2; tail -20 gpurun_out/configs_run.log >&2; exit 1; }
timeout -k 10 500 bash tools/gpu_prof_configs.sh > gpurun_out/prof_cfg.log 2>&1 || { echo "prof_cfg failed" >&2; tail -20 gpurun_out/prof_cfg.log >&2; exit 1; }
echo done
