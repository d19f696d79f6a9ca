#!/bin/bash
# r05 s41: 10k walk pause knobs on the final tree (same box, 2 rounds): RT_DEFER_TRACE (lanes still walking when the
# round's walk pauses), RT_TRACE_MIN (steps before it may), RT_ACCEL_PRIM off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;dt8|RT_DEFER_TRACE=8;dt32|RT_DEFER_TRACE=32;tm8|RT_TRACE_MIN=8;tm32|RT_TRACE_MIN=32;dt0|RT_DEFER_TRACE=0" \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" timeout -k 10 1100 bash tools/gpu_ab_env.sh gpurun_out/ab_s41_10k_pause.jsonl \
  > gpurun_out/s41.log 2>&1; echo "rc=$?"
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/ab_s41_10k_pause.jsonl"):
    d = json.loads(l); r[d["label"]].append(d["kernel_ms"]["render_median"])
for k, v in r.items(): print(k, v)
PY
