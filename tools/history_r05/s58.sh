#!/bin/bash
# r05 s58: the verified sphere walk's scheduler and residency once more: max-ilp (default) vs iterative-minreg vs max-ilp
# at 5 waves per SIMD (RT_ACCEL_WAVES=5), 10k config, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s58_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s58_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="ilp|;minreg|RT_ACCEL_SCHED=iterative-minreg;ilp5|RT_ACCEL_WAVES=5"
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s58_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s58_10k_sched.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s58_10k_sched.jsonl"):
    d = json.loads(l); k = d["kernel_ms"]
    print(d["label"], d["round"], d["ms_per_step"], k["render_median"])
PY
