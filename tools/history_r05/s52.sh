#!/bin/bash
# r05 s52: after the 8-B list entries: the whole GPU suite, then the 10k config's render traffic at full size
# (FETCH_SIZE x2 + WRITE_SIZE, for profiles/hbm_traffic.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/traffic_cfg
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s52_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/s52_pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/s52_pytest_gpu.log
name=scene20_random_10k_1920x1080_spp256_d16
timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_cfg/$name" --sets "FETCH_SIZE;WRITE_SIZE" \
  --scene 20 --width 1920 --height 1080 --spp 256 --bounces 16 --ppm > "gpurun_out/traffic_cfg/$name.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo done
