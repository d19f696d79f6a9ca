#!/bin/bash
# r05 s11: the staging valid-mask fix (partial-tile guard test + fused PPM with and without staging); the 10k render
# kernel's HBM traffic with every colour-stack level in LDS (RT_RC_LDS_LEVELS=16), at the allocator's register
# budget (no spills), without primary-ray lists, and at spp 128, against the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s11_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s11_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step s11_staged_tests 300 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "staged_tile_writes or fused_ppm"
RT_STAGE_SLOTS=4 step s11_staged_fused_s4 300 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "fused_ppm"
RT_DEBUG=1 step s11_pmc10k_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s11_pmc10k_def" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
RT_RC_LDS_LEVELS=16 RT_DEBUG=1 step s11_pmc10k_rc16 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s11_pmc10k_rc16" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
RT_ACCEL_WAVES=0 RT_DEBUG=1 step s11_pmc10k_w0 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s11_pmc10k_w0" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
RT_ACCEL_PRIM=0 RT_DEBUG=1 step s11_pmc10k_noprim 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s11_pmc10k_noprim" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 32 --ppm
RT_DEBUG=1 step s11_pmc10k_def_spp128 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s11_pmc10k_def_spp128" --sets "FETCH_SIZE;WRITE_SIZE" --scene 20 --spp 128 --ppm
tail -n 3 gpurun_out/s11_staged_tests.log gpurun_out/s11_staged_fused_s4.log
grep -h "launch" gpurun_out/s11_pmc10k_*/pass0.log | sort | uniq | head -10
