#!/bin/bash
# r05 s22: spill-free register budgets by default (accel walk at 5 waves, residency raise only without scratch): the full
# GPU suite, then same-box A/Bs against round 4's budgets (RT_ACCEL_WAVES=6 is NOT run at the 10k config: it faulted)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s22_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step s22_pytest_gpu 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
tail -n 3 gpurun_out/s22_pytest_gpu.log
grep FAILED gpurun_out/s22_pytest_gpu.log | head
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;r4|RT_JIT_RAISE_SCRATCH=16" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s22_ab_cornell 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s22_cornell.jsonl
ROUNDS=2 LIM=300 VARIANTS="def|RT_AB=0;r4|RT_JIT_RAISE_SCRATCH=16" BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" \
  step s22_ab_final 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s22_final.jsonl
cut -c1-160 gpurun_out/ab_s22_cornell.jsonl gpurun_out/ab_s22_final.jsonl
