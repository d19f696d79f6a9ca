#!/bin/bash
# r05 s9: per-XCD tile queues (RT_XCD_CLASSES=1): every GPU test with them on, same-box A/B on scene 0 / Cornell /
# 10k, L2-to-memory request counters of scene 0 with them (each 128-B frame line written through one XCD's L2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s9_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s9_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
RT_DEBUG=1 RT_XCD_CLASSES=1 step s9_debug 120 python3 tools/pmc_workload.py --scene 0 --spp 16 --ppm
RT_XCD_CLASSES=1 step s9_pytest_cls 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
ROUNDS=2 VARIANTS="def|RT_AB=0;cls|RT_XCD_CLASSES=1" BENCH_ARGS="--steps 5 --warmup 1" step s9_ab_scene0 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s9_scene0.jsonl
SETS="TCC_EA0_RDREQ,TCC_EA0_RDREQ_32B,TCC_EA0_WRREQ,TCC_EA0_WRREQ_64B;FETCH_SIZE;WRITE_SIZE"
RT_XCD_CLASSES=1 step s9_pmc_s0_cls 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s9_pmc_s0_cls" --sets "$SETS" --scene 0 --spp 128 --ppm
RT_XCD_CLASSES=1 step s9_pmc_s0_cls512 400 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/s9_pmc_s0_cls512" --sets "$SETS" --scene 0 --spp 512 --ppm
ROUNDS=1 VARIANTS="def|RT_AB=0;cls|RT_XCD_CLASSES=1" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1" step s9_ab_cornell 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s9_cornell.jsonl
ROUNDS=1 VARIANTS="def|RT_AB=0;cls|RT_XCD_CLASSES=1" BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s9_ab_10k 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s9_10k.jsonl
tail -n 3 gpurun_out/s9_pytest_cls.log
grep "queues\|launch" gpurun_out/s9_debug.log | head -3
cut -c1-190 gpurun_out/ab_s9_scene0.jsonl gpurun_out/ab_s9_cornell.jsonl gpurun_out/ab_s9_10k.jsonl
