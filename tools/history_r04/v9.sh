#!/bin/bash
# r04 v9: 10k scene — same-box A/B of the inline-entry list loop (current tree), the index-entry list loop
# (ablib/librt_hip_r04v7.so = commit 50c0e60), lists off, and the first round-4 build, 3 rounds; then the per-wave
# phase timeline (RT_WAVE_TRACE, tools/wave_trace.py) of one frame with the lists on and off.
# -> profiles/r04_ab_v9_10k.jsonl, r04_v9_wave_trace_10k_{prim,noprim}.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B=$PWD/ablib/librt_hip_r04base.so
V7=$PWD/ablib/librt_hip_r04v7.so
ROUNDS=3 VARIANTS="new|RT_AB_NEW=1;v7|RT_HIP_LIB=$V7;noprim|RT_ACCEL_PRIM=0;base|RT_HIP_LIB=$B" \
  BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_v9_10k.jsonl || exit $?
timeout -k 10 300 python3 tools/wave_trace.py --scene 20 --spp 64 > gpurun_out/wt_10k_prim.txt 2>&1 || { echo wt rc=$?; tail gpurun_out/wt_10k_prim.txt; exit 1; }
timeout -k 10 300 python3 tools/wave_trace.py --scene 20 --spp 64 --env RT_ACCEL_PRIM=0 > gpurun_out/wt_10k_noprim.txt 2>&1 || { echo wt rc=$?; tail gpurun_out/wt_10k_noprim.txt; exit 1; }
grep -E "phase cycles|render" gpurun_out/wt_10k_prim.txt gpurun_out/wt_10k_noprim.txt
echo done
