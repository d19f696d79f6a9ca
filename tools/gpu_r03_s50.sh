#!/bin/bash
# Same-box A/B: forced residency for the scene-specialised (static) kernels on the final tree —
# Cornell 86 VGPRs (5 waves) -> 6, Perlin 149 (3) -> 4, scene 0 72 (6) -> 8; alternating, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=2 VARIANTS="auto|RT_AB_BASE=1;w6|RT_JIT_WAVES=6" \
BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_waves_s1.jsonl || exit $?
ROUNDS=2 VARIANTS="auto|RT_AB_BASE=1;w4|RT_JIT_WAVES=4" \
BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_waves_s17.jsonl || exit $?
ROUNDS=2 VARIANTS="auto|RT_AB_BASE=1;w8|RT_JIT_WAVES=8" \
BENCH_ARGS="--scene 0 --spp 512 --bounces 16 --steps 6 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_waves_s0.jsonl || exit $?
echo done
