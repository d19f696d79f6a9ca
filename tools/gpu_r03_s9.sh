#!/bin/bash
# Round-3 session 9: 10k-scene A/B, second set (same box, alternating, 3 rounds): breadth-first order with
# 0 / 64 / 128 LDS-staged top nodes, the early next-node fetch at 5 waves, and both together.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export VARIANTS="bfs|;lds64|RT_ACCEL_LDS_NODES=64;lds128|RT_ACCEL_LDS_NODES=128;early_w5|RT_JIT_OPTS=-DRT_ACCEL_EARLY_NEXT=1 RT_JIT_WAVES=5;lds64_early_w5|RT_ACCEL_LDS_NODES=64 RT_JIT_OPTS=-DRT_ACCEL_EARLY_NEXT=1 RT_JIT_WAVES=5"
export BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" ROUNDS=3
timeout -k 10 900 bash tools/gpu_ab_env.sh gpurun_out/ab2_s20.jsonl
timeout -k 10 300 python3 tools/wave_trace.py --scene 17 --spp 1024 --bounces 50 > gpurun_out/wave_s17.log 2>&1
