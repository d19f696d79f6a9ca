#!/bin/bash
# r05 s2: is the round-4 4-wide 6-wave mismatch the HBM RNG-slot hand-off?  The same diagnosis on the build of
# 922baa8 (slots in HBM, the r04_v14 tree), of a7a8f92 (the next commit: the same code with the slots in LDS), of
# 922baa8 with the slot loads at agent scope (bypassing the CU's vector L1), and on this tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s2_steps.log
run() {  # label, lib
  local label=$1 lib=$2
  RT_HIP_LIB=$lib timeout -k 10 300 python3 -u tools/r05/w4_diag.py --seeds 0 1 2 3 4 5 6 7 --no-trace --reps 3 \
      --out gpurun_out/w4_$label > gpurun_out/w4_$label.log 2>&1
  local rc=$?
  echo "$label rc=$rc" >> gpurun_out/s2_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $label (rc=$rc)"; tail -5 gpurun_out/w4_$label.log; exit $rc; fi
}
run v14_hbm_slots "$PWD/ablib/librt_hip_r04v14.so"
run v16_lds_slots "$PWD/ablib/librt_hip_r04v16.so"
run v14_agent_loads "$PWD/ablib/librt_hip_r04v14_agentload.so"
run r05 "$PWD/cuda_raytracing_amd/lib/librt_hip.so"
for f in gpurun_out/w4_*.log; do echo "== $f"; grep -v amdgpu.ids "$f"; done
