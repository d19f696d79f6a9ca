#!/bin/bash
# r04 v10: full -m gpu suite (slot entries by id & 63, span start stamped at once), then HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes) of every BASELINE config and final_scene
# on the round-4 tree (tools/gpu_traffic_configs.sh; + final_scene) -> profiles/r04_v10_traffic/, hbm_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_traffic_configs.sh || exit $?
name=scene3_$(python3 -c "import sys; sys.path.insert(0, '.'); import cuda_raytracing_amd as rt; print(rt.scene_name(3))")_800x800_spp64_d40
timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_cfg/$name" --sets "FETCH_SIZE;WRITE_SIZE" \
  --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --ppm > "gpurun_out/traffic_cfg/$name.log" 2>&1 || { echo final rc=$?; tail -20 "gpurun_out/traffic_cfg/$name.log"; exit 1; }
echo "$name $(python3 -c "import json; m=json.load(open('gpurun_out/traffic_cfg/$name/summary.json'))['merged']; print([k for k in m if k.endswith('_render')][0])")" >> gpurun_out/traffic_cfg/kernels.txt
cat gpurun_out/traffic_cfg/kernels.txt
echo done
