#!/bin/bash
# r04 v8: list entries with the sphere inline (one load chain per entry, the next entry prefetched): the GPU
# tests of the verified walk and the list path, one RT_DEBUG frame (list statistics), then same-box A/Bs:
# 10k (lists on / off, base), scene 2 (lists on / off).
# -> profiles/r04_v8_*.txt, r04_ab_v8_*.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -v -m gpu -k "primary or verified or wide or accel or seed or byte" \
  --timeout 180 --timeout-method thread > gpurun_out/pytest_v8.log 2>&1 \
  || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_v8.log | head -20; tail -5 gpurun_out/pytest_v8.log; exit 1; }
tail -1 gpurun_out/pytest_v8.log
RT_DEBUG=1 timeout -k 10 300 python3 bench.py --scene 20 --spp 16 --bounces 16 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
  > gpurun_out/v8_debug.json 2> gpurun_out/v8_debug.err || { echo debug rc=$?; tail -20 gpurun_out/v8_debug.err; exit 1; }
grep -E "primary lists|launch" gpurun_out/v8_debug.err | head -8
B=$PWD/ablib/librt_hip_r04base.so
ab() { local name=$1; shift; ROUNDS=${R:-2} VARIANTS="$1" BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/ab_v8_$name.jsonl || exit $?; }
ab 10k "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1;noprim|RT_ACCEL_PRIM=0" "--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
R=1 ab scene2 "new|RT_AB_NEW=1;noprim|RT_ACCEL_PRIM=0" "--scene 2 --spp 256 --bounces 16 --steps 3 --warmup 1"
echo done
