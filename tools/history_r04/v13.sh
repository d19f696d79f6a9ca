#!/bin/bash
# r04 v13: 10k scene — is the camera-ray list path worth its code?  Same box, 3 rounds: lists on (default), the
# kernel compiled without the list path (RT_JIT_OPTS=-DRT_PRIM_LISTS=0), lists off at run time, the first round-4
# build.  -> profiles/r04_ab_v13_10k.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/ablib/librt_hip_r04base.so
ROUNDS=3 VARIANTS="new|RT_AB_NEW=1;nocode|RT_JIT_OPTS=-DRT_PRIM_LISTS=0;noprim|RT_ACCEL_PRIM=0;base|RT_HIP_LIB=$B" \
  BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_v13_10k.jsonl || exit $?
echo done
