#!/bin/bash
# r06: scene-0 static kernel under LLVM 22 — residency requests and scheduler strategies, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
V="def|RT_AB=0;w7|RT_JIT_WAVES=7;w8|RT_JIT_WAVES=8;iilp|RT_STATIC_SCHED=iterative-ilp;mmc|RT_STATIC_SCHED=max-memory-clause;dflt|RT_STATIC_SCHED=0"
VARIANTS="$V" ROUNDS=${ROUNDS:-2} LIM=300 BENCH_ARGS="--steps 5 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_scene0_knobs.jsonl || exit 1
