#!/bin/bash
# r04 v19: the viewport point carried from the pixel's pickup (kernels other than the verified sphere walk) vs
# recomputed per sample (ablib/librt_hip_ae039e0.so) vs the first round-4 build: scene 0 and Cornell, same box.
# -> profiles/r04_ab_v19_{scene0,cornell}.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "golden or static or byte or seed or oracle" --timeout 180 --timeout-method thread > gpurun_out/pytest_v19.log 2>&1 \
  || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_v19.log | head; exit 1; }
tail -1 gpurun_out/pytest_v19.log
L=$PWD/ablib
ab() { local name=$1; shift; ROUNDS=${R:-2} VARIANTS="$1" BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/ab_v19_$name.jsonl || exit $?; }
ab scene0 "pp|RT_AB_NEW=1;nopp|RT_HIP_LIB=$L/librt_hip_ae039e0.so;base|RT_HIP_LIB=$L/librt_hip_r04base.so" "--steps 6 --warmup 1"
R=1 ab cornell "pp|RT_AB_NEW=1;nopp|RT_HIP_LIB=$L/librt_hip_ae039e0.so;base|RT_HIP_LIB=$L/librt_hip_r04base.so" "--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1"
echo done
