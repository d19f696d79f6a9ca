#!/bin/bash
# Round-3 session 16: verified sphere walk with the packed pause state (parity), then the 10k scene at
# 5 vs forced 6 waves per SIMD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread -k "verified or accel or sphere_world" > gpurun_out/pytest_accel.log 2>&1 || { tail -30 gpurun_out/pytest_accel.log; exit 1; }
tail -2 gpurun_out/pytest_accel.log
export ROUNDS=3 VARIANTS="w5|;w6|RT_JIT_WAVES=6" BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
timeout -k 10 600 bash tools/gpu_ab_env.sh gpurun_out/ab_w6_s20.jsonl || exit $?
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab_w6_s20.jsonl'): j=json.loads(l); d[j['label']].append(j['ms_per_step'])
print(dict(d))"
