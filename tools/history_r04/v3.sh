#!/bin/bash
# r04 v3: RNG seeding fused into the render kernel's tile pickup, lazy hit record of the verified walk, per-sample
# pixel point, 4-wide verified walk (RT_ACCEL_WIDTH=4): full -m gpu suite, then same-box A/B against the build of
# the first round-4 commit (ablib/librt_hip_r04base.so) on the headline, Cornell and the 10k config.
# -> profiles/r04_v3_pytest_gpu.txt, r04_ab_v3_*.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -1 gpurun_out/pytest_gpu.log
B=$PWD/ablib/librt_hip_r04base.so
ROUNDS=2 VARIANTS="base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" BENCH_ARGS="--steps 6 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_v3_scene0.jsonl || exit $?
ROUNDS=2 VARIANTS="base|RT_HIP_LIB=$B;new|RT_AB_NEW=1;w4v5|RT_ACCEL_WIDTH=4 RT_ACCEL_WAVES=5;w4v6|RT_ACCEL_WIDTH=4 RT_ACCEL_WAVES=6" \
  BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_v3_10k.jsonl || exit $?
ROUNDS=1 VARIANTS="base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_v3_cornell.jsonl || exit $?
echo done
