#!/bin/bash
# r06: row-major vs tile-major frame output under LLVM 22, single frame and two frames in flight (the pipelined leg is
# where the untile kernel waits behind the next frame's render kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
V="row|RT_TILED_OUT=0;tiled|RT_TILED_OUT=1"
VARIANTS=$V ROUNDS=3 PIPE=10 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_rowmajor_scene0.jsonl || exit 1
VARIANTS=$V ROUNDS=3 PIPE=3 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_rowmajor_10k.jsonl || exit 1
VARIANTS=$V ROUNDS=2 PIPE=3 LIM=300 BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_rowmajor_cornell.jsonl || exit 1
VARIANTS=$V ROUNDS=2 PIPE=3 LIM=300 BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_rowmajor_perlin.jsonl || exit 1
