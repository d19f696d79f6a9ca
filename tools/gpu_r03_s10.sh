#!/bin/bash
# Round-3 session 10: sparse hot waves (RT_PRIO_LANES) and LDS-64 default: parity first, then the
# Perlin (scene 17) A/B of lanes per hot wave x costliest tiles, and a 10k check of the new defaults.
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
step pytest_sel 400 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread -k "cooperative_noise or verified or accel or random_scenes"
export VARIANTS="base|;l4t16|RT_PRIO_LANES=4 RT_PRIO_TILES=16;l4t64|RT_PRIO_LANES=4 RT_PRIO_TILES=64;l8t64|RT_PRIO_LANES=8 RT_PRIO_TILES=64;l2t16|RT_PRIO_LANES=2 RT_PRIO_TILES=16;l1t8|RT_PRIO_LANES=1 RT_PRIO_TILES=8;l8t256|RT_PRIO_LANES=8 RT_PRIO_TILES=256"
export BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" ROUNDS=2
step ab_s17 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s17_sparse.jsonl
export VARIANTS="lds64|;lds0|RT_ACCEL_LDS_NODES=0"
export BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" ROUNDS=2
step ab_s20 600 bash tools/gpu_ab_env.sh gpurun_out/ab3_s20.jsonl
cut -c1-150 gpurun_out/ab_s17_sparse.jsonl gpurun_out/ab3_s20.jsonl
