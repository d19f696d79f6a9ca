#!/bin/bash
# r06: one residency step up for the data-driven walks at the price of a few spilled VGPRs (LLVM 22):
# the mixed walk at 4 waves (128 VGPRs, 9 spilled) on final_scene, the verified sphere walk at 7 (72, 6 spilled) on 10k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06
mkdir -p $O
VARIANTS="def|RT_AB=0;w4|RT_JIT_WAVES=4" ROUNDS=2 LIM=300 BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" \
  bash tools/gpu_ab_env.sh $O/ab_waves_final.jsonl || exit 1
VARIANTS="def|RT_AB=0;w7|RT_ACCEL_WAVES=7" ROUNDS=2 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh $O/ab_waves_10k.jsonl || exit 1
