#!/bin/bash
# r05 s49: where the 10k render kernel's ~100 MB of memory writes come from (the frame is 25 MB): PMC at spp 32 with the
# default (tile-major, primary-ray lists), row-major stores, no lists
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s49_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s49_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
R="TCC_EA0_RDREQ,TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;FETCH_SIZE;WRITE_SIZE"
step s49_def 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s49_def" --sets "$R" --scene 20 --spp 32 --ppm
RT_TILED_OUT=0 step s49_row 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s49_row" --sets "$R" --scene 20 --spp 32 --ppm
RT_ACCEL_PRIM=0 step s49_nolist 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s49_nolist" --sets "$R" --scene 20 --spp 32 --ppm
RT_ACCEL_PRIM=0 step s49_nolist_spp128 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s49_nolist_spp128" --sets "$R" --scene 20 --spp 128 --ppm
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/s49_*/summary.json")):
    m = json.load(open(f))["merged"]
    for k, v in m.items():
        if any(x in k for x in ("render", "untile", "prim_list", "probe")):
            print(f.split("/")[1], k[:28], {a: round(b) for a, b in v.items()})
PY
