#!/bin/bash
# r05 s10: output staging flushed at tile pickup (no per-round check): every GPU test with 8x8 tiles + 4 slots; kernel
# register counts (RT_DEBUG) of the staged kernels; 10k and scene-0 A/B; the 10k render kernel's writes with staging;
# instruction counts of the scene-0 kernel with and without staging.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s10_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s10_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
RT_STAGE_SLOTS=4 step s10_pytest_s4 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
for v in "def|" "t8s4|RT_STAGE_SLOTS=4" "t32s4|RT_TILE_W=32 RT_STAGE_SLOTS=4"; do
  l=${v%%|*}; e=${v#*|}
  env RT_DEBUG=1 $e timeout -k 10 120 python3 tools/pmc_workload.py --scene 0 --spp 16 --ppm > gpurun_out/s10_dbg_s0_$l.log 2>&1 || exit $?
  env RT_DEBUG=1 $e timeout -k 10 120 python3 tools/pmc_workload.py --scene 20 --spp 4 --ppm > gpurun_out/s10_dbg_10k_$l.log 2>&1 || exit $?
done
ROUNDS=2 VARIANTS="def|RT_AB=0;t8s4|RT_STAGE_SLOTS=4;t32s4|RT_TILE_W=32 RT_STAGE_SLOTS=4" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s10_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s10_10k.jsonl
ROUNDS=2 VARIANTS="def|RT_AB=0;t8s4|RT_STAGE_SLOTS=4" BENCH_ARGS="--steps 5 --warmup 1" step s10_ab_scene0 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s10_scene0.jsonl
RT_STAGE_SLOTS=4 step s10_pmc10k_t8s4 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s10_pmc10k_t8s4" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
RT_TILE_W=32 RT_STAGE_SLOTS=4 step s10_pmc10k_t32s4 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s10_pmc10k_t32s4" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
P0="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
step s10_pmc_s0_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s10_pmc_s0_def" --sets "$P0" --scene 0 --spp 64 --ppm
RT_STAGE_SLOTS=4 step s10_pmc_s0_t8s4 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s10_pmc_s0_t8s4" --sets "$P0" --scene 0 --spp 64 --ppm
tail -n 3 gpurun_out/s10_pytest_s4.log
grep -h "NUM_REGS\|launch" gpurun_out/s10_dbg_*.log | sort | uniq | head -20
cut -c1-190 gpurun_out/ab_s10_10k.jsonl gpurun_out/ab_s10_scene0.jsonl
