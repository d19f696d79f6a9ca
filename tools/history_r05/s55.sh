#!/bin/bash
# r05 s55: the verified sphere walk built with the max-ilp scheduler (RT_ACCEL_SCHED default): whole GPU suite, then
# same-box A/Bs against the default strategy (RT_ACCEL_SCHED=0): 10k config, scene 2 (bouncing spheres)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s55_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s55_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; grep -E "FAILED|Error" "gpurun_out/$name.log" | head; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s55_pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -n 1 gpurun_out/s55_pytest_gpu.log
V="ilp|;def|RT_ACCEL_SCHED=0"
ROUNDS=3 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s55_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s55_10k_sched.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 2 --spp 256 --steps 3 --warmup 1" step s55_ab_scene2 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s55_scene2_sched.jsonl
python3 - <<'PY'
import json
for f in ("10k", "scene2"):
    for l in open(f"gpurun_out/ab_s55_{f}_sched.jsonl"):
        d = json.loads(l); k = d["kernel_ms"]
        print(f, d["label"], d["round"], d["ms_per_step"], k["render_median"], d["traversal"])
PY
