#!/bin/bash
# r05 s3: coalesced tile writes (RT_TILE_W / RT_STAGE_SLOTS) — every GPU test with 32x2 tiles and 4 staging slots,
# same-box A/B of the tile shape and staging on scene 0 and the 10k scene, L2/EA request counters of scene 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s3_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s3_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
RT_DEBUG=1 RT_TILE_W=32 RT_STAGE_SLOTS=4 step s3_debug 120 python3 tools/pmc_workload.py --scene 0 --spp 16 --ppm
RT_TILE_W=32 RT_STAGE_SLOTS=4 step s3_pytest_t32s4 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
ROUNDS=2 VARIANTS="def|RT_AB=0;t32|RT_TILE_W=32;t32s4|RT_TILE_W=32 RT_STAGE_SLOTS=4;t8s4|RT_STAGE_SLOTS=4" \
  BENCH_ARGS="--steps 5 --warmup 1" step s3_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s3_scene0.jsonl
ROUNDS=2 VARIANTS="def|RT_AB=0;t32s4|RT_TILE_W=32 RT_STAGE_SLOTS=4" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s3_ab_10k 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s3_10k.jsonl
SETS="TCC_EA0_RDREQ,TCC_EA0_RDREQ_32B,TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;TCC_HIT,TCC_MISS,TCC_READ,TCC_WRITE;FETCH_SIZE;WRITE_SIZE"
step s3_pmc_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s3_pmc_def" --sets "$SETS" --scene 0 --spp 128 --ppm
RT_TILE_W=32 RT_STAGE_SLOTS=4 step s3_pmc_t32s4 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s3_pmc_t32s4" --sets "$SETS" --scene 0 --spp 128 --ppm
RT_TILE_W=32 step s3_pmc_t32 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s3_pmc_t32" --sets "$SETS" --scene 0 --spp 128 --ppm
tail -n 3 gpurun_out/s3_pytest_t32s4.log
cat gpurun_out/ab_s3_scene0.jsonl gpurun_out/ab_s3_10k.jsonl | cut -c1-200
