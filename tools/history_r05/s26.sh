#!/bin/bash
# r05 s26: the deep-level pool on the other deep config (scene 0, 4K, d50: traffic + A/B) and Perlin again (3 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s26_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s26_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
ROUNDS=2 LIM=300 VARIANTS="def|RT_RC_POOL=0;p16|RT_RC_POOL=16" BENCH_ARGS="--scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1" \
  step s26_ab_4k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s26_4k_pool.jsonl
ROUNDS=3 LIM=300 VARIANTS="def|RT_RC_POOL=0;p16|RT_RC_POOL=16" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s26_ab_perlin 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s26_perlin_pool.jsonl
P="FETCH_SIZE;WRITE_SIZE"
export RT_DEBUG=1
RT_RC_POOL=0 step s26_pmc_4k_def 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s26_pmc_4k_def" --sets "$P" --scene 0 --width 3840 --height 2160 --spp 256 --bounces 50 --ppm
RT_RC_POOL=16 step s26_pmc_4k_p16 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s26_pmc_4k_p16" --sets "$P" --scene 0 --width 3840 --height 2160 --spp 256 --bounces 50 --ppm
grep -h "launch:" gpurun_out/s26_pmc*/pass0.log | sort | uniq -c | head
cut -c1-160 gpurun_out/ab_s26_4k_pool.jsonl gpurun_out/ab_s26_perlin_pool.jsonl
