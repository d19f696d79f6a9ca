#!/bin/bash
# r05 s56: machine-scheduler strategy of the other run-time kernels (RT_JIT_SCHED, every kernel of the process): the
# mixed walk (final_scene), the Cornell and 4K static kernels; default vs max-ilp vs max-memory-clause
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s56_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s56_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="def|;ilp|RT_JIT_SCHED=max-ilp;mem|RT_JIT_SCHED=max-memory-clause"
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" step s56_ab_final 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s56_final_sched.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1" step s56_ab_cornell 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s56_cornell_sched.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1" step s56_ab_4k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s56_4k_sched.jsonl
python3 - <<'PY'
import json
for f in ("final", "cornell", "4k"):
    for l in open(f"gpurun_out/ab_s56_{f}_sched.jsonl"):
        d = json.loads(l); k = d["kernel_ms"]
        print(f, d["label"], d["round"], d["ms_per_step"], k["render_median"], d["traversal"])
PY
