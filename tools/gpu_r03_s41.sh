#!/bin/bash
# Round-3 final tree, part A: full -m gpu suite, default bench, rocprof kernel stats of the default bench
# command, 2-rank gloo rehearsal with the gather self-check.
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
step bench 400 python3 bench.py
step prof_default 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_default" -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e
step gloo2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --spp 64 --dist-backend gloo --no-e2e --pipelined-steps 0
tail -1 gpurun_out/bench.log | cut -c1-300
