#!/bin/bash
# Same-box A/B: register budget one occupancy step up where the kernel sits just above a boundary
# (10k accel kernel 82 VGPRs -> 80 = 6 waves; mixed kernel 98 -> 96 = 5 waves), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RT_DEBUG=1 timeout -k 10 120 python3 bench.py --scene 1 --spp 16 --bounces 50 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s1.txt
RT_DEBUG=1 timeout -k 10 120 python3 bench.py --scene 17 --spp 16 --bounces 50 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s17.txt
RT_DEBUG=1 RT_JIT_WAVES=6 timeout -k 10 120 python3 bench.py --scene 20 --spp 16 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s20_w6.txt
ROUNDS=3 VARIANTS="auto|RT_AB_BASE=1;w6|RT_JIT_WAVES=6" \
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_waves_s20.jsonl || exit $?
RT_DEBUG=1 RT_JIT_WAVES=5 timeout -k 10 120 python3 bench.py --scene 3 --width 800 --height 800 --spp 4 --bounces 40 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s3_w5.txt
ROUNDS=3 VARIANTS="auto|RT_AB_BASE=1;w5|RT_JIT_WAVES=5" \
BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_waves_s3.jsonl || exit $?
echo done
