#!/bin/bash
# Round-3 session 8: verified sphere walk with breadth-first node order (default now) against the
# oracle, then the 10k-scene A/B of node order / LDS-staged top nodes / early next-node fetch, then the
# HBM traffic (render kernel and whole step) of every BASELINE config.  First failure stops the script.
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
step pytest_accel 400 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread -k "verified or accel or sphere_world"
export VARIANTS="dfs|RT_ACCEL_BFS=0;bfs|;bfs_lds64|RT_ACCEL_LDS_NODES=64;bfs_lds256|RT_ACCEL_LDS_NODES=256;early|RT_JIT_OPTS=-DRT_ACCEL_EARLY_NEXT=1;early_w5|RT_JIT_OPTS=-DRT_ACCEL_EARLY_NEXT=1 RT_JIT_WAVES=5"
export BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" ROUNDS=2
step ab_s20 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s20.jsonl
step wave_s17 300 python3 tools/wave_trace.py --scene 17 --spp 1024 --bounces 50
step traffic_cfg 900 bash tools/gpu_traffic_configs.sh
cat gpurun_out/ab_s20.jsonl | cut -c1-200
