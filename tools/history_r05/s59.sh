#!/bin/bash
# r05 s59: the verified walk's pause knobs after its max-ilp build (RT_DEFER_TRACE lanes / RT_TRACE_MIN steps; default
# 16 / 16): 10k config, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s59_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s59_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="d16m16|;d8m16|RT_DEFER_TRACE=8;d24m16|RT_DEFER_TRACE=24;d16m32|RT_TRACE_MIN=32"
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s59_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s59_10k_defer.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s59_10k_defer.jsonl"):
    d = json.loads(l); k = d["kernel_ms"]
    print(d["label"], d["round"], d["ms_per_step"], k["render_median"])
PY
