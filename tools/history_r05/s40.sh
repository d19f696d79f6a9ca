#!/bin/bash
# r05 s40: tile pickup values read with v_readlane (default) vs the round-4 shuffle (RT_PICKUP_SHFL): parity subset,
# same-box A/Bs on scene 0, Perlin, Cornell and 10k
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab_s40.jsonl
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or tile_schedules or tail or verified_sphere or fused_ppm or mixed_walk" > gpurun_out/s40_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 1 gpurun_out/s40_tests.log; [ $rc -eq 0 ] || exit $rc
V="rl|RT_AB=0;shfl|RT_JIT_OPTS=-DRT_PICKUP_SHFL"
run() { local r=$1; shift; ROUNDS=$r LIM=300 VARIANTS="$V" BENCH_ARGS="$*" timeout -k 10 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s40.jsonl >> gpurun_out/s40.log 2>&1 || { echo "ab failed: $*"; exit 1; }; }
run 3 --steps 5 --warmup 1
run 2 --scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1
run 2 --scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1
run 2 --scene 20 --spp 256 --steps 3 --warmup 1
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s40.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], d["traversal"], round(d["value"], 1), d["kernel_ms"]["render_median"])
PY
