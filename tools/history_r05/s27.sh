#!/bin/bash
# r05 s27: the deep-level pool with the lanes' chunk indices in LDS (Perlin kernel back at 128 VGPRs): parity tests,
# Perlin d50 A/B (3 rounds) and render-kernel traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s27_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s27_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s27_pool_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "colour_stack or deep_unwind or byte_colour"
tail -n 2 gpurun_out/s27_pool_tests.log
ROUNDS=3 LIM=300 VARIANTS="def|RT_RC_POOL=0;p16|RT_RC_POOL=16;p8|RT_RC_POOL=8" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s27_ab_perlin 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s27_perlin_pool.jsonl
P="FETCH_SIZE;WRITE_SIZE"
export RT_DEBUG=1
RT_RC_POOL=16 step s27_pmc_perlin_p16 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s27_pmc_perlin_p16" --sets "$P" --scene 17 --spp 1024 --bounces 50 --ppm
RT_RC_POOL=8 step s27_pmc_perlin_p8 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s27_pmc_perlin_p8" --sets "$P" --scene 17 --spp 1024 --bounces 50 --ppm
grep -h "launch:" gpurun_out/s27_pmc*/pass0.log | sort | uniq -c | head
cut -c1-160 gpurun_out/ab_s27_perlin_pool.jsonl
