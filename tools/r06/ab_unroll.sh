#!/bin/bash
# r06: LLVM 22 run-time kernels with the loop unroller limited to pragma-forced loops (-fno-unroll-loops) and the static
# kernels' max-ilp scheduler, against LLVM 22 default and torch's LLVM 20, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
V="l22|RT_JIT_COMPILER=rocm;l22nu|RT_JIT_COMPILER=rocm RT_JIT_OPTS=-fno-unroll-loops;l22nuilp|RT_JIT_COMPILER=rocm RT_JIT_OPTS=-fno-unroll-loops RT_STATIC_SCHED=max-ilp;l20|RT_JIT_COMPILER=process"
run() { VARIANTS="$V" ROUNDS=${3:-2} LIM=${LIM:-300} BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_unroll_$1.jsonl || exit 1; }
run scene0 "--steps 5 --warmup 1" 3
run 10k "--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
run cornell "--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1"
run perlin "--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1"
