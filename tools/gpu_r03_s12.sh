#!/bin/bash
# Round-3 session 12: full -m gpu suite on the tree with sparse hot waves by default (noise scenes),
# then final_scene (noise + mixed walk) with and without them.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -40 "gpurun_out/$name.log" >&2; exit $rc; fi
}
step pytest_gpu 700 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread
export ROUNDS=2
VARIANTS="sparse|;nosparse|RT_PRIO_LANES=64" BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1" \
  step ab_s3 600 bash tools/gpu_ab_env.sh gpurun_out/ab_sparse_s3.jsonl
step wave_s17 300 python3 tools/wave_trace.py --scene 17 --spp 1024 --bounces 50
tail -2 gpurun_out/pytest_gpu.log
cut -c1-160 gpurun_out/ab_sparse_s3.jsonl
