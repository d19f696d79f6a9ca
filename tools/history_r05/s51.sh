#!/bin/bash
# r05 s51: 8-B primary-ray list entries (SAH prim index + axial bound; the sphere's words from the tree's prims):
# parity (list tests, verified-walk tests, full-spp rows), 10k PMC at spp 32 and at the full config, 10k A/B against
# the previous library (32-B entries with the sphere inline, ablib/librt_hip_r05_prelist.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s51_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s51_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; grep -E "FAILED|Error" "gpurun_out/$name.log" | head; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s51_tests 500 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "primary_candidate or full_spp_config_rows or sphere_world or verified or accel or scene20 or random_10k"
tail -n 2 gpurun_out/s51_tests.log
R="TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;FETCH_SIZE;WRITE_SIZE"
step s51_pmc_new 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s51_pmc_new" --sets "$R" --scene 20 --spp 32 --ppm
RT_HIP_LIB=$PWD/ablib/librt_hip_r05_prelist.so step s51_pmc_old 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s51_pmc_old" --sets "$R" --scene 20 --spp 32 --ppm
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/s51_pmc_*/summary.json")):
    m = json.load(open(f))["merged"]
    for k, v in m.items():
        if "render" in k or "prim_list" in k:
            print(f.split("/")[1], k[:28], {a: round(b) for a, b in v.items()}, "MB", round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) / 1e3, 1))
PY
ROUNDS=3 LIM=300 VARIANTS="old|RT_HIP_LIB=$PWD/ablib/librt_hip_r05_prelist.so;new|" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s51_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s51_10k_compact_lists.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/ab_s51_10k_compact_lists.jsonl"):
    d = json.loads(l); print(d["label"], d["round"], d["ms_per_step"], d["kernel_ms"]["render_median"])
PY
