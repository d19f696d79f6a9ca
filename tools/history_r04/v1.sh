#!/bin/bash
# r04 v1: pytest -m gpu, smoke, default bench, PMC (incl. FETCH/WRITE) of the shipped scene-0 static kernel and of
# the shipped 6-wave verified-sphere kernel on the 10k scene.  -> profiles/r04_v1_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...   (stop on fault / abort / timeout: rc not 0)
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
step pytest_gpu 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
tail -2 gpurun_out/pytest_gpu.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
tail -c 3000 gpurun_out/bench.log
step pmc_s0 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s0" --scene 0 --spp 128 --ppm
step pmc_s20 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s20" --scene 20 --spp 32 --ppm
echo done
