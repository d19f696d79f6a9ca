#!/bin/bash
# r05 s47: tile-major output (now the default) vs row-major stores, same box: Perlin d50 and Cornell d50 (the f2 box ran
# Perlin 20 % slower than the earlier sweep), scene 0 once more
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s47_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s47_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="row|RT_TILED_OUT=0;tiled|RT_TILED_OUT=1"
ROUNDS=3 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 5 --warmup 1" \
  step s47_ab_perlin 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s47_perlin_tiled.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" \
  step s47_ab_cornell 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s47_cornell_tiled.jsonl
ROUNDS=3 LIM=200 VARIANTS="$V" BENCH_ARGS="--steps 5 --warmup 1" \
  step s47_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s47_scene0_tiled.jsonl
python3 - <<'PY'
import json
for f in ("perlin", "cornell", "scene0"):
    for l in open(f"gpurun_out/ab_s47_{f}_tiled.jsonl"):
        d = json.loads(l); print(f, d["label"], d["round"], d["ms_per_step"], d["kernel_ms"]["render_median"])
PY
