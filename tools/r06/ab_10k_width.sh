#!/bin/bash
# r06: the verified sphere walk's tree width under LLVM 22 (10k config): 2-wide (default) vs 4-wide, float and quantised
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06
mkdir -p $O
VARIANTS="w2|RT_AB=0;w4|RT_ACCEL_WIDTH=4;w4q|RT_ACCEL_WIDTH=4 RT_ACCEL_QUANT=1" ROUNDS=2 LIM=300 \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_10k_width.jsonl || exit 1
