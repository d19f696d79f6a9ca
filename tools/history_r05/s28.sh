#!/bin/bash
# r05 s28: scene-0 schedule knobs on the final tree (same box, 2 rounds): probe paths per tile, costliest-tile priority
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 LIM=200 VARIANTS="def|RT_AB=0;pr16|RT_PROBE=16;pr32|RT_PROBE=32;pt0|RT_PRIO_TILES=0;pt1024|RT_PRIO_TILES=1024;dl8|RT_DEFER_LANES=8" \
  BENCH_ARGS="--steps 5 --warmup 1" timeout -k 10 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s28_scene0_sched.jsonl > gpurun_out/s28.log 2>&1
echo "rc=$?"
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/ab_s28_scene0_sched.jsonl"):
    d = json.loads(l); r[d["label"]].append((d["ms_per_step"], d["kernel_ms"]["render_median"], d["kernel_ms"]["schedule_median"]))
for k, v in r.items(): print(k, v)
PY
