#!/bin/bash
# r04 final 6: final_scene after restricting the carried viewport point to the static kernels, vs the round's
# first build, same box, two rounds. -> profiles/r04_ab_f6_final.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/ablib/librt_hip_r04base.so
R=2 ROUNDS=2 VARIANTS="new|RT_AB_NEW=1;base|RT_HIP_LIB=$B" \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_f6_final.jsonl || exit $?
echo done
