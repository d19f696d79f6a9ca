#!/bin/bash
# r05 final 2 (final tree): the rocprofv3 kernel-trace summary of the bench's single-frame command, every BASELINE config
# through bench.py (+ final_scene), then the render kernel's HBM traffic of each (FETCH_SIZE x2 + WRITE_SIZE, separate
# passes) for profiles/hbm_traffic.json (tools/r04/apply_traffic.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/f2_prof" -o run -- python3 bench.py \
  --pipelined-steps 0 --no-cpu-baseline --no-e2e > gpurun_out/f2_rocprof_bench.log 2>&1 || { echo "rocprof failed"; exit 1; }
WITH_FINAL=1 bash tools/gpu_configs.sh || exit $?
bash tools/gpu_traffic_configs.sh || exit $?
echo done
