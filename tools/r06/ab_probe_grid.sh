#!/bin/bash
# r06: the schedule probe launched on a fraction of the render grid (RT_PROBE_GRID): schedule time vs frame time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
VARIANTS="g1|RT_AB=0;g2|RT_PROBE_GRID=2;g4|RT_PROBE_GRID=4" ROUNDS=3 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/r06/ab_probe_grid.jsonl || exit 1
