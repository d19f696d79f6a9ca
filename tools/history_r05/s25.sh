#!/bin/bash
# r05 s25: 10k config with and without primary-ray candidate lists on the 5-wave walk (same box, 3 rounds); Perlin d50
# render-kernel traffic with and without the deep-level pool
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s25_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s25_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
ROUNDS=3 LIM=300 VARIANTS="prim|RT_ACCEL_PRIM=1;noprim|RT_ACCEL_PRIM=0" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  step s25_ab_10k_prim 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s25_10k_prim.jsonl
P="FETCH_SIZE;WRITE_SIZE"
export RT_DEBUG=1
RT_RC_POOL=0 step s25_pmc_perlin_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s25_pmc_perlin_def" --sets "$P" --scene 17 --spp 1024 --bounces 50 --ppm
RT_RC_POOL=16 step s25_pmc_perlin_p16 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s25_pmc_perlin_p16" --sets "$P" --scene 17 --spp 1024 --bounces 50 --ppm
grep -h "launch:" gpurun_out/s25_pmc*/pass0.log | sort | uniq -c | head
cut -c1-160 gpurun_out/ab_s25_10k_prim.jsonl
