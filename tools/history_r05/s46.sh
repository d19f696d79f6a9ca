#!/bin/bash
# r05 s46: tile-major output with the band untile kernel: parity; scene-0 PMC (render + untile); A/Bs scene 0, 10k, 4K

cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s46_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s46_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; grep -E "FAILED|Error" "gpurun_out/$name.log" | head; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s46_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "tiled_output or fused_ppm"
tail -n 2 gpurun_out/s46_tests.log
R="TCC_EA0_RDREQ,TCC_EA0_RDREQ_32B,TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;FETCH_SIZE;WRITE_SIZE"
RT_TILED_OUT=1 step s46_pmc_s0_tiled 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s46_pmc_s0_tiled" --sets "$R" --scene 0 --spp 128 --ppm
step s46_pmc_s0_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s46_pmc_s0_def" --sets "$R" --scene 0 --spp 128 --ppm
ROUNDS=3 LIM=200 VARIANTS="def|RT_TILED_OUT=0;tiled|RT_TILED_OUT=1" BENCH_ARGS="--steps 5 --warmup 1" \
  step s46_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s46_scene0_tiled.jsonl
ROUNDS=2 LIM=300 VARIANTS="def|RT_TILED_OUT=0;tiled|RT_TILED_OUT=1" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s46_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s46_10k_tiled.jsonl
ROUNDS=2 LIM=300 VARIANTS="def|RT_TILED_OUT=0;tiled|RT_TILED_OUT=1" BENCH_ARGS="--width 3840 --height 2160 --spp 2048 --bounces 50 --steps 3 --warmup 1" \
  step s46_ab_4k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s46_4k_tiled.jsonl
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/s46_pmc_s0_*/summary.json")):
    m = json.load(open(f))["merged"]
    for k, v in m.items():
        if "render" in k or "untile" in k:
            print(f.split("/")[1], k[:30], {a: round(b) for a, b in v.items()})
for f in ("gpurun_out/ab_s46_scene0_tiled.jsonl", "gpurun_out/ab_s46_10k_tiled.jsonl", "gpurun_out/ab_s46_4k_tiled.jsonl"):
    for l in open(f):
        d = json.loads(l); print(f[-20:], d["label"], d["round"], d["ms_per_step"], d["kernel_ms"]["render_median"])
PY
