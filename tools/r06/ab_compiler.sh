#!/bin/bash
# r06: run-time kernels compiled by /opt/rocm's hipRTC (ROCm 7.2, AMD clang 22, dlmopen: the new default) vs the hipRTC the
# process resolved (torch's bundled ROCm 7.0.2, AMD clang 20: every Python process before r06), every BASELINE config +
# final_scene, alternating on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
V="llvm22|RT_JIT_COMPILER=rocm;llvm20|RT_JIT_COMPILER=process"
run() { VARIANTS="$V" ROUNDS=${ROUNDS:-2} LIM=${LIM:-300} BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/r06/ab_compiler_$1.jsonl || exit 1; }
run scene0 "--steps 5 --warmup 1"
run cornell "--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1"
run perlin "--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1"
run 10k "--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
run final "--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1"
run 4k "--width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1"
