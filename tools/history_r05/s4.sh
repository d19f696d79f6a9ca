#!/bin/bash
# r05 s4: (1) every GPU test with 32x2 tiles + 4 staging slots (lean staging, tile-width seeding tables);
# (2) the 4-wide 6-wave mismatch: round-4 final tree vs this tree (16 seeds), v16 with its launch layout printed and
# with an explicit colour-stack size (no LDS-only kernel); (3) scene-0 A/B of tile shape / staging.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s4_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s4_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
RT_TILE_W=32 RT_STAGE_SLOTS=4 step s4_pytest_t32s4 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
SEEDS="0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15"
RT_HIP_LIB=$PWD/ablib/librt_hip_r04final.so step w4_r04final 300 python3 -u tools/r05/w4_diag.py --seeds $SEEDS --waves 6 --no-trace --reps 2 --out gpurun_out/w4_r04final
step w4_r05b 300 python3 -u tools/r05/w4_diag.py --seeds $SEEDS --waves 6 --no-trace --reps 2 --out gpurun_out/w4_r05b
RT_DEBUG=1 RT_HIP_LIB=$PWD/ablib/librt_hip_r04v16.so step w4_v16_debug 200 python3 -u tools/r05/w4_diag.py --seeds 1 4 0 --waves 6 5 --no-trace --reps 1 --out gpurun_out/w4_v16d
RT_RC_LDS_LEVELS=12 RT_HIP_LIB=$PWD/ablib/librt_hip_r04v16.so step w4_v16_rc12 200 python3 -u tools/r05/w4_diag.py --seeds 1 4 --waves 6 --no-trace --reps 2 --out gpurun_out/w4_v16rc
ROUNDS=2 VARIANTS="def|RT_AB=0;t32|RT_TILE_W=32;t32s2|RT_TILE_W=32 RT_STAGE_SLOTS=2;t32s4|RT_TILE_W=32 RT_STAGE_SLOTS=4" \
  BENCH_ARGS="--steps 5 --warmup 1" step s4_ab_scene0 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s4_scene0.jsonl
tail -n 3 gpurun_out/s4_pytest_t32s4.log
for f in gpurun_out/w4_r04final.log gpurun_out/w4_r05b.log gpurun_out/w4_v16_rc12.log; do echo "== $f"; grep -v "amdgpu.ids\|\[\]" $f; done
grep "launch\|seed" gpurun_out/w4_v16_debug.log
cut -c1-200 gpurun_out/ab_s4_scene0.jsonl
