#!/bin/bash
# Same-box A/B of the residency cap (RT_BLOCKS_PER_CU: fewer resident waves = more pixels per lane, shorter
# relative tail, less latency hiding) on the final tree, alternating, 2-3 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ROUNDS=3 VARIANTS="auto|RT_AB_BASE=1;b4|RT_BLOCKS_PER_CU=4" \
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_bpc_s20.jsonl || exit $?
ROUNDS=3 VARIANTS="auto|RT_AB_BASE=1;b5|RT_BLOCKS_PER_CU=5" \
BENCH_ARGS="--scene 0 --spp 512 --bounces 16 --steps 8 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_bpc_s0.jsonl || exit $?
ROUNDS=2 VARIANTS="auto|RT_AB_BASE=1;b2|RT_BLOCKS_PER_CU=2" \
BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_bpc_s3.jsonl || exit $?
RT_DEBUG=1 timeout -k 10 120 python3 bench.py --scene 20 --spp 16 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s20.txt
RT_DEBUG=1 timeout -k 10 120 python3 bench.py --scene 0 --spp 16 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s0.txt
RT_DEBUG=1 timeout -k 10 120 python3 bench.py --scene 3 --width 800 --height 800 --spp 4 --bounces 40 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_s3.txt
echo done
