#!/bin/bash
# r05 s54: the run-time kernels' machine-scheduler strategy (RT_JIT_SCHED): default vs max-ilp vs max-memory-clause,
# same box: scene 0, Perlin, 10k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s54_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s54_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="def|;ilp|RT_JIT_SCHED=max-ilp;mem|RT_JIT_SCHED=max-memory-clause"
ROUNDS=3 LIM=200 VARIANTS="$V" BENCH_ARGS="--steps 6 --warmup 1" step s54_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s54_scene0_sched.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" step s54_ab_perlin 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s54_perlin_sched.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s54_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s54_10k_sched.jsonl
python3 - <<'PY'
import json
for f in ("scene0", "perlin", "10k"):
    for l in open(f"gpurun_out/ab_s54_{f}_sched.jsonl"):
        d = json.loads(l); k = d["kernel_ms"]
        print(f, d["label"], d["round"], d["ms_per_step"], k["render_median"])
PY
