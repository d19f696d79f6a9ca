#!/bin/bash
# r04 final 9: Perlin d50 colour-stack levels kept in LDS (RT_RC_LDS_LEVELS = the minimum), same box, two rounds.
# -> profiles/r04_ab_f9_perlin.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 VARIANTS="def|RT_AB=0;l24|RT_RC_LDS_LEVELS=24;l32|RT_RC_LDS_LEVELS=32;l50|RT_RC_LDS_LEVELS=50" \
  BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/ab_f9_perlin.jsonl || exit $?
echo done
