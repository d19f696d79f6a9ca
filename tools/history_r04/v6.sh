#!/bin/bash
# r04 v6: primary-ray candidate lists of the verified sphere walk (device/prim_lists.h) and the per-sample pixel
# point without a division: full -m gpu suite, then same-box A/Bs against the first round-4 build
# (ablib/librt_hip_r04base.so): scene 0; 10k (lists on / off); final_scene.
# -> profiles/r04_v6_pytest_gpu.txt, r04_ab_v6_*.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
    || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
B=$PWD/ablib/librt_hip_r04base.so
ab() { local name=$1; shift; ROUNDS=${R:-2} VARIANTS="$1" BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/ab_v6_$name.jsonl || exit $?; }
ab 10k "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1;noprim|RT_ACCEL_PRIM=0" "--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
ab scene0 "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--steps 6 --warmup 1"
R=1 ab final "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1"
echo done
