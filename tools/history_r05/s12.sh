#!/bin/bash
# r05 s12: the deep-level colour-stack pool (RT_RC_POOL): its parity tests; the Perlin d50 config (BASELINE config 3)
# and the 4K scene-0 d50 config's render-kernel HBM traffic with and without it; a same-box Perlin A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s12_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s12_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step s12_pool_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "colour_stack_pool or colour_stack_hbm or deep_unwind"
for v in "def|RT_RC_POOL=0" "p16|RT_RC_POOL=16" "p32|RT_RC_POOL=32"; do
  l=${v%%|*}; e=${v#*|}
  env RT_DEBUG=1 $e timeout -k 10 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s12_pmc_perlin_$l" --sets "FETCH_SIZE;WRITE_SIZE" \
    --scene 17 --spp 1024 --bounces 50 --ppm > gpurun_out/s12_pmc_perlin_$l.log 2>&1 || exit $?
done
ROUNDS=2 VARIANTS="def|RT_RC_POOL=0;p16|RT_RC_POOL=16;p32|RT_RC_POOL=32" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s12_ab_perlin 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s12_perlin.jsonl
for v in "def|RT_RC_POOL=0" "p16|RT_RC_POOL=16"; do
  l=${v%%|*}; e=${v#*|}
  env RT_DEBUG=1 $e timeout -k 10 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s12_pmc_4k_$l" --sets "FETCH_SIZE;WRITE_SIZE" \
    --scene 0 --width 3840 --height 2160 --spp 256 --bounces 50 --ppm > gpurun_out/s12_pmc_4k_$l.log 2>&1 || exit $?
done
tail -n 3 gpurun_out/s12_pool_tests.log
grep -h "launch" gpurun_out/s12_pmc_*/pass0.log | sort | uniq | head -10
cut -c1-200 gpurun_out/ab_s12_perlin.jsonl
