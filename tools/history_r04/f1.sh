#!/bin/bash
# r04 final 1: full -m gpu suite, smoke, the default bench line, the rocprofv3 kernel-trace summary of the same
# command's frames, then the FETCH / WRITE traffic of every BASELINE config + final_scene (profiles/hbm_traffic.json).
# -> profiles/r04_f1_pytest_gpu.txt, r04_f1_bench.json, r04_f1_kernel_stats.csv, r04_f1_traffic/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic_cfg
step() {  # name, limit, command...   (stop on any failure)
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "gpurun_out/$name.log" | head -20; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
step pytest_gpu 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
tail -1 gpurun_out/pytest_gpu.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
tail -c 600 gpurun_out/bench.log
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --pipelined-steps 0 --no-cpu-baseline --no-e2e
: > gpurun_out/traffic_cfg/kernels.txt
for cfg in "0 1920 1080 512 16" "20 1920 1080 256 16" "1 1920 1080 1024 50" "17 1920 1080 1024 50" "0 3840 2160 2048 50" "3 800 800 64 40"; do
  set -- $cfg
  name=$(python3 -c "import sys; sys.path.insert(0, '.'); import cuda_raytracing_amd as rt; print(f'scene$1_{rt.scene_name($1)}_$2x$3_spp$4_d$5')")
  step "traffic_$1_$2" 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_cfg/$name" --sets "FETCH_SIZE;WRITE_SIZE" \
    --scene "$1" --width "$2" --height "$3" --spp "$4" --bounces "$5" --ppm
  echo "$name $(python3 -c "import json; m=json.load(open('gpurun_out/traffic_cfg/$name/summary.json'))['merged']; print([k for k in m if k.endswith('_render')][0])")" >> gpurun_out/traffic_cfg/kernels.txt
done
cat gpurun_out/traffic_cfg/kernels.txt
echo done
