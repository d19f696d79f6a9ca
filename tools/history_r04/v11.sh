#!/bin/bash
# r04 v11 (final tree): smoke, the default bench line, the rocprofv3 kernel-trace summary of the same command's
# frames, PMC (instruction mix, lane utilisation, waits, FETCH/WRITE) of the shipped scene-0 static kernel, the
# 10k verified-walk kernel and final_scene's mixed-walk kernel.
# -> profiles/r04_v11_bench.json, r04_v11_kernel_stats.csv, r04_v11_pmc_{scene0,scene20_10k,scene3_final}/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...   (stop on any failure)
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then tail -40 "gpurun_out/$name.log"; exit $rc; fi
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
tail -c 1500 gpurun_out/bench.log
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --pipelined-steps 0 --no-cpu-baseline --no-e2e
step pmc_s0 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s0" --scene 0 --spp 128 --ppm
step pmc_s20 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s20" --scene 20 --spp 32 --ppm
step pmc_s3 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s3" --scene 3 --width 800 --height 800 --spp 8 --bounces 40 --ppm
echo done
