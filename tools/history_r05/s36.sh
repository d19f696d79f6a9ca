#!/bin/bash
# r05 s36: 10k config — LDS levels left by the parked sum: default, the deep-level pool (8 chunks), 32 staged SAH nodes;
# same-box A/B (2 rounds) and render-kernel traffic at the full config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s36_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s36_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s36_pool_tests 300 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "colour_stack_pool and 20"
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;pool8|RT_RC_POOL=8;n32|RT_ACCEL_LDS_NODES=32" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s36_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s36_10k.jsonl
P="FETCH_SIZE;WRITE_SIZE"
export RT_DEBUG=1
step s36_pmc_def 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s36_pmc_def" --sets "$P" --scene 20 --spp 256 --ppm
RT_RC_POOL=8 step s36_pmc_pool8 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s36_pmc_pool8" --sets "$P" --scene 20 --spp 256 --ppm
RT_ACCEL_LDS_NODES=32 step s36_pmc_n32 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s36_pmc_n32" --sets "$P" --scene 20 --spp 256 --ppm
grep -h "launch:" gpurun_out/s36_pmc_*/pass0.log | sort | uniq -c
python3 - <<'PY'
import json, glob
for l in open("gpurun_out/ab_s36_10k.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], round(d["value"], 1), d["kernel_ms"]["render_median"])
for f in sorted(glob.glob("gpurun_out/s36_pmc_*/summary.json")):
    m = json.load(open(f))["derived"]
    for k, v in m.items():
        if "render" in k: print(f.split("/")[1], round(v["hbm_bytes_fetch_x2_plus_write"] / 1e6, 1), "MB")
PY
