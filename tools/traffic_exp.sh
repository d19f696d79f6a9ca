#!/bin/bash
# HBM traffic attribution (FETCH_SIZE / WRITE_SIZE in separate rocprofv3 passes per variant):
#   bash tools/traffic_exp.sh   -> gpurun_out/traffic/<name>/summary.json + traffic.txt
# Each step has its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/traffic
run() {  # name, env assignments..., -- workload args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic/$name" --sets "FETCH_SIZE;WRITE_SIZE" "$@" \
    > "gpurun_out/traffic/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/traffic/steps.log
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/traffic/$name.log"; exit $rc; }
  python3 - "$name" <<'PY' | tee -a gpurun_out/traffic/traffic.txt
import json, sys
d = json.load(open(f"gpurun_out/traffic/{sys.argv[1]}/summary.json"))
for k, v in d["merged"].items():
    if "render" in k or "probe" in k or "seed" in k:
        print(f"{sys.argv[1]:34s} {k[:40]:40s} fetch {2 * v.get('FETCH_SIZE', 0) * 1024 / 1e6:9.1f} MB  write {v.get('WRITE_SIZE', 0) * 1024 / 1e6:9.1f} MB")
PY
}
run s0_spp64 X=1 -- --scene 0 --spp 64
run s0_spp256 X=1 -- --scene 0 --spp 256
run s0_spp64_lds16 RT_RC_LDS_LEVELS=16 -- --scene 0 --spp 64
run s0_spp64_ppm X=1 -- --scene 0 --spp 64 --ppm
run s0_spp64_rowmajor RT_SCHED=1 -- --scene 0 --spp 64
run s20_spp16 X=1 -- --scene 20 --spp 16
run s20_spp64 X=1 -- --scene 20 --spp 64
run s20_spp16_lds16 RT_RC_LDS_LEVELS=16 -- --scene 20 --spp 16
