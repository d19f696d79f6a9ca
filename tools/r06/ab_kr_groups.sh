#!/bin/bash
# r06: groups of the render loop's argument uses re-read where used (shading / colour stack), scene 0 and Perlin
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
V="def|RT_AB=0;shade|RT_JIT_OPTS=-DRT_KR_SHADE;rc|RT_JIT_OPTS=-DRT_KR_RC;both|RT_JIT_OPTS=-DRT_KR_SR"
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kr_scene0.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_kr_perlin.jsonl || exit 1
