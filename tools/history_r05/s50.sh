#!/bin/bash
# (RT_PRIM_PAD was an A/B knob of that build; it changed nothing and was removed again: DESIGN §5e)
# r05 s50: primary-ray lists padded apart (RT_PRIM_PAD words between tiles' lists; they were 4 KB apart): list parity
# tests, 10k PMC at spp 32 (pad 0 / 32 / 96), 10k full-config A/B pad 0 vs 32
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s50_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s50_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; grep -E "FAILED|Error" "gpurun_out/$name.log" | head; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s50_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "primary_candidate or full_spp_config_rows"
tail -n 2 gpurun_out/s50_tests.log
R="TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;FETCH_SIZE;WRITE_SIZE"
RT_PRIM_PAD=0 step s50_pmc_p0 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s50_pmc_p0" --sets "$R" --scene 20 --spp 32 --ppm
step s50_pmc_p32 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s50_pmc_p32" --sets "$R" --scene 20 --spp 32 --ppm
RT_PRIM_PAD=96 step s50_pmc_p96 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s50_pmc_p96" --sets "$R" --scene 20 --spp 32 --ppm
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/s50_pmc_*/summary.json")):
    m = json.load(open(f))["merged"]
    for k, v in m.items():
        if "render" in k:
            print(f.split("/")[1], k[:28], {a: round(b) for a, b in v.items()}, "MB", round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) / 1e3, 1))
PY
ROUNDS=3 LIM=300 VARIANTS="p0|RT_PRIM_PAD=0;p32|RT_PRIM_PAD=32" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s50_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s50_10k_prim_pad.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s50_10k_prim_pad.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], d["ms_per_step"], d["kernel_ms"]["render_median"])
PY
