#!/bin/bash
# r05 s53: schedule probe density (RT_PROBE paths per tile; default clamp(spp/4, 8, 64) = 64 here): scene 0 and 10k,
# same box, step time (probe + order + render + untile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s53_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s53_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="p64|RT_PROBE=64;p32|RT_PROBE=32;p16|RT_PROBE=16"
ROUNDS=3 LIM=200 VARIANTS="$V" BENCH_ARGS="--steps 8 --warmup 1" step s53_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s53_scene0_probe.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s53_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s53_10k_probe.jsonl
python3 - <<'PY'
import json
for f in ("scene0", "10k"):
    for l in open(f"gpurun_out/ab_s53_{f}_probe.jsonl"):
        d = json.loads(l); k = d["kernel_ms"]
        print(f, d["label"], d["round"], d["ms_per_step"], k["render_median"], k["schedule_median"])
PY
