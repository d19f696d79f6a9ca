#!/bin/bash
# HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 --pmc passes) of the render kernel for every
# BASELINE config at its full one-GPU size, through the bench path (context + fused PPM bytes), written
# into profiles/hbm_traffic.json (bench.py roofline.traffic) afterwards, on this side:
#   bash tools/gpu_traffic_configs.sh          -> gpurun_out/traffic_cfg/<workload>/summary.json
#   python3 tools/traffic_from_pmc.py gpurun_out/traffic_cfg/<workload>/summary.json <workload> <kernel>
# Each step has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/traffic_cfg
run() {  # scene width height spp bounces
  local name
  name=$(python3 -c "import sys; sys.path.insert(0, '.'); import cuda_raytracing_amd as rt; print(f'scene$1_{rt.scene_name($1)}_$2x$3_spp$4_d$5')")
  timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_cfg/$name" --sets "FETCH_SIZE;WRITE_SIZE" \
    --scene "$1" --width "$2" --height "$3" --spp "$4" --bounces "$5" --ppm > "gpurun_out/traffic_cfg/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/traffic_cfg/steps.log
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/traffic_cfg/$name.log"; exit $rc; }
  local kernel
  kernel=$(python3 -c "import json,sys; m=json.load(open('gpurun_out/traffic_cfg/$name/summary.json'))['merged']; print([k for k in m if k.endswith('_render')][0])")
  echo "$name $kernel" >> gpurun_out/traffic_cfg/kernels.txt
}
run 0 1920 1080 512 16
run 1 1920 1080 1024 50
run 17 1920 1080 1024 50
run 20 1920 1080 256 16
run 0 3840 2160 2048 50
run 3 800 800 64 40
