#!/bin/bash
# r04 v15: 10k scene — waves per SIMD of the 2-wide verified walk (6 default: 80 VGPRs with spills; 5: ~96 VGPRs),
# same box, 3 rounds.  -> profiles/r04_ab_v15_10k_waves.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=3 VARIANTS="w6|RT_AB_NEW=1;w5|RT_ACCEL_WAVES=5" \
  BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_v15_10k_waves.jsonl || exit $?
echo done
