#!/bin/bash
# Round-3 session 7: full -m gpu suite (image decoders, earth JPEG), default bench, rocprof kernel stats of
# the default bench command, final-tree PMC of the 10k-scene kernel (rt_accel_render), step traffic of
# the default config.  Each step has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -40 "gpurun_out/$name.log" >&2; exit $rc; fi
}
step pytest_gpu 600 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread
step bench 400 python3 bench.py
step prof_default 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_default" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e
step traffic_s0 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_s0" --sets "FETCH_SIZE;WRITE_SIZE" --scene 0 --spp 512 --bounces 16 --ppm
step pmc_s20 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s20" --scene 20 --spp 256 --bounces 16 --ppm
tail -1 gpurun_out/bench.log | cut -c1-600
