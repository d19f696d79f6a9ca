#!/bin/bash
# r04 v18: the scene-0 single-frame regression (r04 v17: 41.4 ms vs 33.7 for the v7 build): commit 0ff3638 (the first
# with the per-wave span-start atomic), the v7 build, the first round-4 build and the current tree (start stamp from
# block 0 only), same box.  -> profiles/r04_ab_v18_scene0_bisect.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/ablib
ROUNDS=2 VARIANTS="new|RT_AB_NEW=1;v7|RT_HIP_LIB=$L/librt_hip_r04v7.so;c0ff3638|RT_HIP_LIB=$L/librt_hip_0ff3638.so;base|RT_HIP_LIB=$L/librt_hip_r04base.so" \
  BENCH_ARGS="--steps 4 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_v18_scene0_bisect.jsonl || exit $?
echo done
