#!/bin/bash
# r05 s57: scene-specialised kernels without noise textures built with the max-ilp scheduler (RT_STATIC_SCHED default):
# whole GPU suite, then same-box A/Bs against the default strategy (RT_STATIC_SCHED=0): scene 0, Cornell
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s57_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s57_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; grep -E "FAILED|Error" "gpurun_out/$name.log" | head; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s57_pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -n 1 gpurun_out/s57_pytest_gpu.log
V="ilp|;def|RT_STATIC_SCHED=0"
ROUNDS=3 LIM=300 VARIANTS="$V" BENCH_ARGS="--steps 6 --warmup 1" step s57_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s57_scene0_sched.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1" step s57_ab_cornell 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s57_cornell_sched.jsonl
python3 - <<'PY'
import json
for f in ("scene0", "cornell"):
    for l in open(f"gpurun_out/ab_s57_{f}_sched.jsonl"):
        d = json.loads(l); k = d["kernel_ms"]
        print(f, d["label"], d["round"], d["ms_per_step"], k["render_median"], d["traversal"])
PY
