#!/bin/bash
# r06: more alternating rounds of the mixed walk at 4 waves (raise) vs 3 (RT_JIT_RAISE=0), 4 frames per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
VARIANTS="raise|RT_AB=0;noraise|RT_JIT_RAISE=0" ROUNDS=5 LIM=300 \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 4 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_mixed_raise2.jsonl || exit 1
