#!/bin/bash
# r06: clang's SLP vectoriser (packed f32 pairs) on the scene-specialised kernels under LLVM 22, scene 0 and Cornell
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06
mkdir -p $O
V="def|RT_AB=0;slp|RT_JIT_SLP=1"
VARIANTS=$V ROUNDS=3 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_slp_scene0.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_slp_cornell.jsonl || exit 1
