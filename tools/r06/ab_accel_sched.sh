#!/bin/bash
# r06: the verified sphere walk's scheduler after the kernel-argument re-reads: max-ilp (default) vs the compiler's
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
VARIANTS="ilp|RT_AB=0;dflt|RT_ACCEL_SCHED=0" ROUNDS=4 LIM=300 \
  BENCH_ARGS="--scene 20 --spp 256 --steps 4 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_accel_sched.jsonl || exit 1
VARIANTS="ilp|RT_AB=0;dflt|RT_ACCEL_SCHED=0" ROUNDS=2 LIM=300 \
  BENCH_ARGS="--scene 2 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_accel_sched_scene2.jsonl || exit 1
