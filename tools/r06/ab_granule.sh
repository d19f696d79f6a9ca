#!/bin/bash
# r06: residency from the occupancy table's 8-VGPR granule (7 blocks / CU at 70 VGPRs) vs the measured 16 (6 blocks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
RT_DEBUG=1 RT_VGPR_GRANULE=8 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --pipelined-steps 0 > $O/granule_debug.json 2> $O/granule_debug.err || { tail -5 $O/granule_debug.err; exit 1; }
grep "occupancy" $O/granule_debug.err | head -3
V="g16|RT_AB=0;g8|RT_VGPR_GRANULE=8"
VARIANTS=$V ROUNDS=3 LIM=300 BENCH_ARGS="--steps 10 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_granule_scene0.jsonl || exit 1
VARIANTS=$V ROUNDS=2 LIM=300 BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh $O/ab_granule_cornell.jsonl || exit 1
