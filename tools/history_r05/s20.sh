#!/bin/bash
# r05 s20: the scene-20 mismatch's mitigations — parity of each on the failing small frames, then the 10k config A/B:
# default (6 waves, SGPR spills in VGPR lanes), 6 waves with SGPR spills in scratch, 5 waves, the allocator's budget, and
# the 6-wave build without the tail-piece code
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spp in 2 16; do
  timeout -k 10 300 python3 tools/r05/dbg20.py --spp $spp "def|" "sgprmem|RT_ACCEL_WAVES=6 RT_JIT_SGPR_MEM=1" "w5|RT_ACCEL_WAVES=5" \
    "w0|RT_ACCEL_WAVES=0" "notail|RT_JIT_OPTS=-DRT_NO_TAIL_CODE" > gpurun_out/s20_dbg_spp$spp.log 2>&1 || { echo "dbg failed"; exit 1; }
  echo "== spp $spp"; grep -v amdgpu.ids gpurun_out/s20_dbg_spp$spp.log
done
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;sgprmem|RT_ACCEL_WAVES=6 RT_JIT_SGPR_MEM=1;w5|RT_ACCEL_WAVES=5;w0|RT_ACCEL_WAVES=0;notail|RT_JIT_OPTS=-DRT_NO_TAIL_CODE" \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s20_10k.jsonl \
  > gpurun_out/s20_ab.log 2>&1; echo "ab rc=$?"
cut -c1-160 gpurun_out/ab_s20_10k.jsonl
