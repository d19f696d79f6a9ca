#!/bin/bash
# r04 final 8: residency sweep on the final tree, same box, two rounds.
#   scene 0 (static kernel, 80 VGPRs / 6 waves by default): forced 7 and 8 waves.
#   10k spheres (verified walk): 4 / 6 waves vs the default, and the 4-wide walk.
# -> profiles/r04_ab_f8_{scene0,10k}.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 VARIANTS="def|RT_AB=0;w7|RT_JIT_WAVES=7;w8|RT_JIT_WAVES=8" BENCH_ARGS="--steps 5 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_f8_scene0.jsonl || exit $?
ROUNDS=2 VARIANTS="def|RT_AB=0;a4|RT_ACCEL_WAVES=4;a6|RT_ACCEL_WAVES=6;wide|RT_ACCEL_WIDTH=4" \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_f8_10k.jsonl || exit $?
echo done
