#!/bin/bash
# r04 v5: RNG seeding by one column-table jump per pixel (phase bases + per-tile-column nibble tables) and the
# quantised 4-wide tree, residency raise by a VGPR cap at the hardware granule (final_scene's mixed walk 169 -> 160): full -m gpu suite, then same-box A/Bs against the first round-4 build
# (ablib/librt_hip_r04base.so): scene 0, Cornell d50, final_scene; 10k: 2-wide (default) vs quantised / float 4-wide.
# -> profiles/r04_v5_pytest_gpu.txt, r04_ab_v5_*.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
    || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
B=$PWD/ablib/librt_hip_r04base.so
ab() { local name=$1; shift; ROUNDS=${R:-2} VARIANTS="$1" BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/ab_v5_$name.jsonl || exit $?; }
ab scene0 "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--steps 6 --warmup 1"
ab 10k "w2|RT_AB_NEW=1;w4q5|RT_ACCEL_WIDTH=4 RT_ACCEL_WAVES=5;w4q6|RT_ACCEL_WIDTH=4;w4f5|RT_ACCEL_WIDTH=4 RT_ACCEL_QUANT=0 RT_ACCEL_WAVES=5" "--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
R=1 ab cornell "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1"
ab final "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1;noraise|RT_JIT_RAISE=0" "--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1"
echo done
