#!/bin/bash
# Verified sphere walk at 6 waves/SIMD by default (rt_jit.cpp accel_waves): occupancy lines, pytest -m gpu,
# the 10k config through bench.py (CPU sample bit-exact) + rocprof stats, A/B against RT_ACCEL_WAVES=0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RT_DEBUG=1 timeout -k 10 120 python3 bench.py --scene 20 --spp 16 --steps 1 --warmup 0 --pipelined-steps 0 --no-cpu-baseline --no-e2e > /dev/null 2> gpurun_out/occ_w6_s20.txt || { echo occ rc=$?; exit 1; }
grep -h 'occupancy\|launch:' gpurun_out/occ_w6_s20.txt
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest rc=$?; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1 > gpurun_out/cfg_c4.log 2> gpurun_out/cfg_c4.err || { echo c4 rc=$?; tail gpurun_out/cfg_c4.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_c4" -o run -- python3 bench.py --scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1 --pipelined-steps 0 --no-cpu-baseline --no-e2e > gpurun_out/prof_c4.log 2>&1 || { echo prof rc=$?; exit 1; }
ROUNDS=2 VARIANTS="w6|RT_AB_BASE=1;alloc|RT_ACCEL_WAVES=0" \
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_accelw_s20.jsonl || exit $?
ROUNDS=2 VARIANTS="w6|RT_AB_BASE=1;alloc|RT_ACCEL_WAVES=0;w5|RT_ACCEL_WAVES=5" \
BENCH_ARGS="--scene 2 --spp 256 --bounces 16 --steps 3 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_accelw_s2.jsonl || exit $?
echo done
