#!/bin/bash
# r06: tail pieces on the final tree's 10k frame (the last ids of the longest-first order handed out in pieces)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
VARIANTS="def|RT_AB=0;t8|RT_TAIL_CHUNK=8 RT_TAIL_GEN=1;t4|RT_TAIL_CHUNK=4 RT_TAIL_GEN=2" ROUNDS=3 LIM=300 \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_10k_tail.jsonl || exit 1
