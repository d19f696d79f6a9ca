#!/bin/bash
# Same-box A/B of the schedule probe's density (RT_PROBE paths per 8x8 tile; auto = min(64, max(8, spp/4)))
# on scene 0 (headline) and the 10k scene, alternating, 3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export ROUNDS=3
VARIANTS="auto|RT_AB_BASE=1;p8|RT_PROBE=8;p16|RT_PROBE=16;p32|RT_PROBE=32" \
BENCH_ARGS="--scene 0 --spp 512 --bounces 16 --steps 8 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_probe_s0.jsonl || exit $?
VARIANTS="auto|RT_AB_BASE=1;p16|RT_PROBE=16;p32|RT_PROBE=32" \
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_probe_s20.jsonl || exit $?
echo done
