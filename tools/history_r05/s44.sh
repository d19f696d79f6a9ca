#!/bin/bash
# r05 s44: rejection tries per round (RT_MAX_TRIES) — scene 0 (3 rounds, 6/8/12 tries) and the other configs (8 tries)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_s44.jsonl
run() { local r=$1 v=$2; shift 2; ROUNDS=$r LIM=300 VARIANTS="$v" BENCH_ARGS="$*" timeout -k 10 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s44.jsonl >> gpurun_out/s44.log 2>&1 || { echo "ab failed: $*"; exit 1; }; }
run 3 "def|RT_AB=0;mt6|RT_MAX_TRIES=6;mt8|RT_MAX_TRIES=8;mt12|RT_MAX_TRIES=12" --steps 5 --warmup 1
run 2 "def|RT_AB=0;mt8|RT_MAX_TRIES=8" --scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1
run 2 "def|RT_AB=0;mt8|RT_MAX_TRIES=8" --scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1
run 2 "def|RT_AB=0;mt8|RT_MAX_TRIES=8" --scene 20 --spp 256 --steps 3 --warmup 1
run 1 "def|RT_AB=0;mt8|RT_MAX_TRIES=8" --scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s44.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], d["traversal"], round(d["value"], 1), d["kernel_ms"]["render_median"])
PY
