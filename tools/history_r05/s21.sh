#!/bin/bash
# r05 s21: 10k config A/B of the accel kernel's builds (the tail-piece code now compiled only on request): default (6 waves,
# SGPR spills in VGPR lanes), 6 waves with SGPR spills in scratch, 5 waves, the allocator's budget; parity of each first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spp in 2 16; do
  timeout -k 10 300 python3 tools/r05/dbg20.py --spp $spp "def|" "sgprmem|RT_ACCEL_WAVES=6 RT_JIT_SGPR_MEM=1" "w5|RT_ACCEL_WAVES=5" \
    "w0|RT_ACCEL_WAVES=0" > gpurun_out/s21_dbg_spp$spp.log 2>&1 || { echo "dbg failed"; exit 1; }
  echo "== spp $spp"; grep -v amdgpu.ids gpurun_out/s21_dbg_spp$spp.log
  if grep -q "differing px [1-9]" gpurun_out/s21_dbg_spp$spp.log; then echo "mismatch: no A/B"; exit 1; fi
done
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;sgprmem|RT_ACCEL_WAVES=6 RT_JIT_SGPR_MEM=1;w5|RT_ACCEL_WAVES=5;w0|RT_ACCEL_WAVES=0" \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s21_10k.jsonl \
  > gpurun_out/s21_ab.log 2>&1; echo "ab rc=$?"
cut -c1-160 gpurun_out/ab_s21_10k.jsonl
