#!/bin/bash
# r04 v16: the per-wave RNG slots in LDS (were an HBM buffer: 41 MB written and read back per 1080p frame, r04 v10
# traffic): full -m gpu suite, same-box A/Bs against the first round-4 build, and the FETCH / WRITE traffic of
# scene 0 and the 10k scene.  -> profiles/r04_v16_pytest_gpu.txt, r04_ab_v16_*.jsonl, r04_v16_traffic/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic_cfg
timeout -k 10 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
  || { echo pytest rc=$?; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
B=$PWD/ablib/librt_hip_r04base.so
ab() { local name=$1; shift; ROUNDS=${R:-2} VARIANTS="$1" BENCH_ARGS="$2" bash tools/gpu_ab_env.sh gpurun_out/ab_v16_$name.jsonl || exit $?; }
ab scene0 "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--steps 6 --warmup 1"
ab 10k "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1"
R=1 ab cornell "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1"
R=1 ab perlin "base|RT_HIP_LIB=$B;new|RT_AB_NEW=1" "--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1"
: > gpurun_out/traffic_cfg/kernels.txt
for cfg in "0 1920 1080 512 16" "20 1920 1080 256 16"; do
  set -- $cfg
  name=$(python3 -c "import sys; sys.path.insert(0, '.'); import cuda_raytracing_amd as rt; print(f'scene$1_{rt.scene_name($1)}_$2x$3_spp$4_d$5')")
  timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_cfg/$name" --sets "FETCH_SIZE;WRITE_SIZE" \
    --scene "$1" --width "$2" --height "$3" --spp "$4" --bounces "$5" --ppm > "gpurun_out/traffic_cfg/$name.log" 2>&1 || { echo traffic rc=$?; exit 1; }
  echo "$name $(python3 -c "import json; m=json.load(open('gpurun_out/traffic_cfg/$name/summary.json'))['merged']; print([k for k in m if k.endswith('_render')][0])")" >> gpurun_out/traffic_cfg/kernels.txt
done
cat gpurun_out/traffic_cfg/kernels.txt
echo done
