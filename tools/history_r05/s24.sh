#!/bin/bash
# r05 s24: HBM traffic of the 10k render kernel (spill-free 5-wave build): default, every colour level in LDS, no
# primary-ray lists, spp 128; then the deep-level pool (RT_RC_POOL): parity tests, Perlin d50 traffic and A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s24_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s24_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
P="FETCH_SIZE;WRITE_SIZE"
RT_DEBUG=1 step s24_pmc10k_def 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s24_pmc10k_def" --sets "$P" --scene 20 --spp 32 --ppm
RT_DEBUG=1 RT_RC_LDS_LEVELS=16 step s24_pmc10k_rc16 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s24_pmc10k_rc16" --sets "$P" --scene 20 --spp 32 --ppm
RT_DEBUG=1 RT_ACCEL_PRIM=0 step s24_pmc10k_noprim 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s24_pmc10k_noprim" --sets "$P" --scene 20 --spp 32 --ppm
RT_DEBUG=1 step s24_pmc10k_spp128 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s24_pmc10k_spp128" --sets "$P" --scene 20 --spp 128 --ppm
step s24_pool_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "colour_stack_pool"
tail -n 2 gpurun_out/s24_pool_tests.log
for v in "def|RT_RC_POOL=0" "p16|RT_RC_POOL=16"; do
  l=${v%%|*}; e=${v#*|}
  env RT_DEBUG=1 $e step s24_pmc_perlin_$l 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s24_pmc_perlin_$l" --sets "$P" \
    --scene 17 --spp 1024 --bounces 50 --ppm
done
ROUNDS=2 LIM=300 VARIANTS="def|RT_RC_POOL=0;p16|RT_RC_POOL=16;p32|RT_RC_POOL=32" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s24_ab_perlin 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s24_perlin.jsonl
grep -h "launch:" gpurun_out/s24_pmc*/pass0.log | sort | uniq -c | head
cut -c1-160 gpurun_out/ab_s24_perlin.jsonl
