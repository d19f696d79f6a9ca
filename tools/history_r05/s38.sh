#!/bin/bash
# r05 s38: full GPU suite with colour levels ahead of staged SAH nodes; 10k A/B against 64 staged nodes (2 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/s38_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/s38_pytest_gpu.log; grep FAILED gpurun_out/s38_pytest_gpu.log | head
[ $rc -eq 0 ] || exit $rc
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;n64|RT_ACCEL_LDS_NODES=64" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  timeout -k 10 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s38_10k.jsonl > gpurun_out/s38_ab.log 2>&1; echo "ab rc=$?"
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s38_10k.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], round(d["value"], 1), d["kernel_ms"]["render_median"])
PY
