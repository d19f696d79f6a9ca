#!/bin/bash
# r05 s34: 10k config, same box, 3 rounds: the final tree (5 waves), its 6-wave build, round 4's final library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/ablib/librt_hip_r04final.so
ROUNDS=3 LIM=300 VARIANTS="w5|RT_AB=0;w6|RT_ACCEL_WAVES=6;r04|RT_HIP_LIB=$L" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s34_10k.jsonl > gpurun_out/s34.log 2>&1; echo "rc=$?"
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s34_10k.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], round(d["value"], 1), d["kernel_ms"]["render_median"], d["kernel_ms"]["render_mean"])
PY
