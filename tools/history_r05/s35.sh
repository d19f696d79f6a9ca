#!/bin/bash
# r05 s35: the 2-wide walk at 6 waves without VGPR spills (sum parked, ballot tail priority, scalar root): scratch of the
# hipRTC build, scene-20 parity probes, the full GPU suite, then the 10k A/B against 5 waves and round 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RT_DEBUG=1 timeout -k 10 300 python3 tools/r05/dbg20.py --spp 2 "def|" > gpurun_out/s35_dbg2.log 2>&1 || { echo dbg failed; exit 1; }
RT_DEBUG=1 timeout -k 10 300 python3 tools/r05/dbg20.py --spp 16 "def|" > gpurun_out/s35_dbg16.log 2>&1 || { echo dbg failed; exit 1; }
grep -h "waves_per_eu\|differing\|jit occupancy" gpurun_out/s35_dbg*.log | sort | uniq
if grep -q "differing px [1-9]" gpurun_out/s35_dbg*.log; then echo "mismatch: stop"; exit 1; fi
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/s35_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/s35_pytest_gpu.log; grep FAILED gpurun_out/s35_pytest_gpu.log | head
[ $rc -eq 0 ] || exit $rc
L=$PWD/ablib/librt_hip_r04final.so
ROUNDS=3 LIM=300 VARIANTS="w6|RT_AB=0;w5|RT_ACCEL_WAVES=5;r04|RT_HIP_LIB=$L" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s35_10k.jsonl > gpurun_out/s35_ab.log 2>&1; echo "ab rc=$?"
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s35_10k.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], round(d["value"], 1), d["kernel_ms"]["render_median"], d["kernel_ms"]["render_mean"])
PY
