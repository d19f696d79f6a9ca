#!/bin/bash
# r04 v17: scene 0 single-frame regression check after the LDS RNG slots (r04 f1: render 37.4 ms in rocprof):
# same-box A/B of the current tree, ablib/librt_hip_r04v7.so (HBM slots) and the first round-4 build, 2 rounds, and
# the RT_DEBUG launch line of the current tree.  -> profiles/r04_ab_v17_scene0.jsonl, r04_v17_debug_scene0.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RT_DEBUG=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/v17_debug.json 2> gpurun_out/v17_debug.err || { echo debug rc=$?; tail gpurun_out/v17_debug.err; exit 1; }
grep -E "launch|occupancy|raise" gpurun_out/v17_debug.err | sort | uniq -c | head -12
B=$PWD/ablib/librt_hip_r04base.so
V7=$PWD/ablib/librt_hip_r04v7.so
ROUNDS=2 VARIANTS="new|RT_AB_NEW=1;v7|RT_HIP_LIB=$V7;base|RT_HIP_LIB=$B" BENCH_ARGS="--steps 6 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_v17_scene0.jsonl || exit $?
echo done
