#!/bin/bash
# r05 s45: the mixed walk with its noise octaves rolled (147 VGPRs, 3 waves without spills): mixed-walk parity tests,
# final_scene A/B against the unrolled build (RT_MIX_NOISE_UNROLL=7), 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RT_DEBUG=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -k "mixed or final" > gpurun_out/s45_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/s45_tests.log | tail -1; grep -h "jit occupancy" gpurun_out/s45_tests.log | sort | uniq -c | head -5
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 LIM=300 VARIANTS="rolled|RT_AB=0;unrolled|RT_MIX_NOISE_UNROLL=7" BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" \
  timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s45_final.jsonl > gpurun_out/s45_ab.log 2>&1; echo "ab rc=$?"
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s45_final.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], round(d["value"], 2), d["kernel_ms"]["render_median"])
PY
