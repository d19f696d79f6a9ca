#!/bin/bash
# r05 s33: the final tree against round 4's final library (ablib/librt_hip_r04final.so) on one box, every config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_s33_vs_r04.jsonl
L=$PWD/ablib/librt_hip_r04final.so
run() {  # rounds, bench args
  local r=$1; shift
  ROUNDS=$r LIM=300 VARIANTS="r05|RT_AB=0;r04|RT_HIP_LIB=$L" BENCH_ARGS="$*" timeout -k 10 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s33_vs_r04.jsonl \
    >> gpurun_out/s33.log 2>&1 || { echo "failed: $*"; exit 1; }
}
run 2 --steps 5 --warmup 1
run 2 --scene 20 --spp 256 --steps 3 --warmup 1
run 1 --scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1
run 1 --scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1
run 1 --scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1
run 1 --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s33_vs_r04.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], d["traversal"], round(d["value"], 1), d["kernel_ms"]["render_median"])
PY
