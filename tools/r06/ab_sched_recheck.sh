#!/bin/bash
# r06: scheduler strategies re-checked after the kernel-argument re-reads: the Perlin (noise) kernel and the 10k walk
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
VARIANTS="def|RT_AB=0;ilp|RT_STATIC_SCHED=max-ilp;mmc|RT_STATIC_SCHED=max-memory-clause;iilp|RT_STATIC_SCHED=iterative-ilp" ROUNDS=2 LIM=300 \
  BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_sched_perlin.jsonl || exit 1
VARIANTS="def|RT_AB=0;dflt|RT_ACCEL_SCHED=0;mmc|RT_ACCEL_SCHED=max-memory-clause" ROUNDS=2 LIM=300 \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_sched_10k.jsonl || exit 1
