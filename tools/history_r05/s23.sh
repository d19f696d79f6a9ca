#!/bin/bash
# r05 s23: tail pieces on the spill-free kernels — parity tests, then same-box A/Bs (10k, scene 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s23_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s23_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
step s23_tail_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "tail_pieces or tail_issue"
tail -n 2 gpurun_out/s23_tail_tests.log
ROUNDS=3 LIM=300 VARIANTS="def|RT_TAIL_CHUNK=0;t8|RT_TAIL_CHUNK=8;t4g2|RT_TAIL_CHUNK=4 RT_TAIL_GEN=2" \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s23_ab_10k 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_s23_10k.jsonl
cut -c1-160 gpurun_out/ab_s23_10k.jsonl
