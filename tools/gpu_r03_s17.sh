#!/bin/bash
# Round-3 session 17: cooperative finish of the verified sphere walk (compile-time RT_COOP_WALK):
# parity with it forced on (every walk of a wave with <= 8 tracing lanes, from step 1), then the 10k A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RT_JIT_OPTS=-DRT_COOP_WALK=1 RT_COOP_WALK=8 RT_COOP_MIN=1 timeout -k 10 400 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread -k "verified or accel or sphere_world" > gpurun_out/pytest_coop.log 2>&1 || { tail -30 gpurun_out/pytest_coop.log; exit 1; }
tail -2 gpurun_out/pytest_coop.log
export ROUNDS=2 VARIANTS="base|;c2m8|RT_JIT_OPTS=-DRT_COOP_WALK=1 RT_COOP_WALK=2 RT_COOP_MIN=8;c4m8|RT_JIT_OPTS=-DRT_COOP_WALK=1 RT_COOP_WALK=4 RT_COOP_MIN=8;c2m32|RT_JIT_OPTS=-DRT_COOP_WALK=1 RT_COOP_WALK=2 RT_COOP_MIN=32;c0|RT_JIT_OPTS=-DRT_COOP_WALK=1 RT_COOP_WALK=0" BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
timeout -k 10 700 bash tools/gpu_ab_env.sh gpurun_out/ab_coop_s20.jsonl || exit $?
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab_coop_s20.jsonl'): j=json.loads(l); d[j['label']].append(j['ms_per_step'])
print(dict(d))"
