#!/bin/bash
# r05 s43: scene-0 rejection-sampling knobs on the final tree (same box, 2 rounds): lanes left when the round's rejection
# stops (RT_DEFER_LANES, default 4) and a cap on tries per round (RT_MAX_TRIES, default none)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 LIM=200 VARIANTS="def|RT_AB=0;dl2|RT_DEFER_LANES=2;dl6|RT_DEFER_LANES=6;dl12|RT_DEFER_LANES=12;mt4|RT_MAX_TRIES=4;mt8|RT_MAX_TRIES=8" \
  BENCH_ARGS="--steps 5 --warmup 1" timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s43_scene0_rej.jsonl > gpurun_out/s43.log 2>&1
echo "rc=$?"
python3 - <<'PY'
import json, collections
r = collections.defaultdict(list)
for l in open("gpurun_out/ab_s43_scene0_rej.jsonl"):
    d = json.loads(l); r[d["label"]].append(d["kernel_ms"]["render_median"])
for k, v in r.items(): print(k, v)
PY
