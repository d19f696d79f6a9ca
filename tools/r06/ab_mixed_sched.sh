#!/bin/bash
# r06: the mixed walk's machine scheduler under LLVM 22 (RT_MIXED_SCHED): default vs max-ilp vs max-memory-clause
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
VARIANTS="def|RT_AB=0;ilp|RT_MIXED_SCHED=max-ilp;mmc|RT_MIXED_SCHED=max-memory-clause" ROUNDS=3 LIM=300 \
  BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 4 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_mixed_sched.jsonl || exit 1
