#!/bin/bash
# r04 v12 (final tree): every BASELINE config + final_scene through bench.py on one box (tools/gpu_configs.sh) and
# the rocprofv3 kernel-trace summaries of their frames (tools/gpu_prof_configs.sh).
# -> profiles/r04_v12_configs.jsonl, r04_v12_kernel_stats_c*.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
WITH_FINAL=1 bash tools/gpu_configs.sh || exit $?
bash tools/gpu_prof_configs.sh || exit $?
echo done
