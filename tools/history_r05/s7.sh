#!/bin/bash
# r05 s7: every GPU test on the default settings (hit flag as a word, random_test parked in the LDS stack of the
# verified walk, two-level seeding column tables); scene-0 A/B separating the staging code's static cost (compiled in,
# no slots: RT_STAGE_SLOTS=-1) from its run-time cost; the 10k config against the round-4 final build (time and
# FETCH/WRITE: the spill writes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s7_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s7_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step s7_pytest 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
ROUNDS=2 VARIANTS="def|RT_AB=0;t32|RT_TILE_W=32;t32sc|RT_TILE_W=32 RT_STAGE_SLOTS=-1;t32s4|RT_TILE_W=32 RT_STAGE_SLOTS=4;t8sc|RT_STAGE_SLOTS=-1;t8s4|RT_STAGE_SLOTS=4" \
  BENCH_ARGS="--steps 5 --warmup 1" step s7_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s7_scene0.jsonl
ROUNDS=2 VARIANTS="def|RT_AB=0;r04f|RT_HIP_LIB=$PWD/ablib/librt_hip_r04final.so" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s7_ab_10k 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s7_10k.jsonl
step s7_pmc10k_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s7_pmc10k_def" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
RT_HIP_LIB=$PWD/ablib/librt_hip_r04final.so step s7_pmc10k_r04f 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s7_pmc10k_r04f" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
SETS="TCC_EA0_RDREQ,TCC_EA0_RDREQ_32B,TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;FETCH_SIZE;WRITE_SIZE"
step s7_pmc_s0_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s7_pmc_s0_def" --sets "$SETS" --scene 0 --spp 128 --ppm
tail -n 3 gpurun_out/s7_pytest.log
cut -c1-190 gpurun_out/ab_s7_scene0.jsonl gpurun_out/ab_s7_10k.jsonl
