#!/bin/bash
# r04 final 5: the d50 configs and final_scene, final tree vs the round's first build, same box, one round each.
# -> profiles/r04_ab_f5_{cornell,perlin,final}.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/ablib/librt_hip_r04base.so
ab() { local name=$1; shift; ROUNDS=${R:-1} VARIANTS="$1" BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/ab_f5_$name.jsonl || exit $?; }
ab cornell "new|RT_AB_NEW=1;base|RT_HIP_LIB=$B" "--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1"
ab perlin "new|RT_AB_NEW=1;base|RT_HIP_LIB=$B" "--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1"
ab final "new|RT_AB_NEW=1;base|RT_HIP_LIB=$B" "--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1"
echo done
