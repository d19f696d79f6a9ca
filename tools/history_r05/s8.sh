#!/bin/bash
# r05 s8: tile shape vs frame time (scene 0: 8x8, 16x4, 32x2, 64x1; Cornell and 10k: 8x8 vs 32x2), and the 10k render
# kernel's remaining writes (FETCH/WRITE at spp 8 and 32; the code object dumped for an ISA check).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s8_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s8_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
ROUNDS=2 VARIANTS="t8|RT_TILE_W=8;t16|RT_TILE_W=16;t32|RT_TILE_W=32;t64|RT_TILE_W=64" BENCH_ARGS="--steps 5 --warmup 1" \
  step s8_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s8_scene0.jsonl
ROUNDS=1 VARIANTS="t8|RT_TILE_W=8;t32|RT_TILE_W=32" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s8_ab_cornell 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s8_cornell.jsonl
mkdir -p gpurun_out/s8_dump10k
RT_JIT_DUMP=$PWD/gpurun_out/s8_dump10k RT_JIT_CACHE_DIR=0 RT_DEBUG=1 step s8_dump10k 200 python3 tools/pmc_workload.py --scene 20 --spp 4 --ppm
step s8_pmc10k_spp8 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s8_pmc10k_spp8" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 8 --ppm
cut -c1-190 gpurun_out/ab_s8_scene0.jsonl gpurun_out/ab_s8_cornell.jsonl
