#!/bin/bash
# r04 v2: 4-wide verified sphere walk (RT_ACCEL_WIDTH=4): parity tests, then a same-box A/B on BASELINE config 4
# (10k spheres, 1080p, spp 256, d16) against the 2-wide walk, at several waves-per-SIMD requests.
# -> profiles/r04_ab_accel_wide.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -v -m gpu -k "wide or verified_sphere or random_sphere" --timeout 180 \
  --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 || { echo pytest rc=$?; tail -30 gpurun_out/pytest_wide.log; exit 1; }
tail -1 gpurun_out/pytest_wide.log
ROUNDS=2 VARIANTS="w2|RT_ACCEL_WIDTH=2;w4|RT_ACCEL_WIDTH=4;w4v5|RT_ACCEL_WIDTH=4 RT_ACCEL_WAVES=5;w4v6|RT_ACCEL_WIDTH=4 RT_ACCEL_WAVES=6;w4v4|RT_ACCEL_WIDTH=4 RT_ACCEL_WAVES=4" \
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_accel_wide.jsonl || exit $?
echo done
