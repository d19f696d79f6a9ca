#!/bin/bash
# Round-3 session 2: pytest -m gpu (colour-stack spill tests), default bench (all-core CPU baseline),
# scene-0 traffic PMC (seed / probe / render), 2-rank gloo rehearsal of the N>1 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -30 "gpurun_out/$name.log" >&2; exit $rc; fi
}
step pytest_gpu 600 python3 -u -m pytest tests -v -m gpu -x --timeout 180 --timeout-method thread
step bench 400 python3 bench.py
step traffic_s0 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_s0" --sets "FETCH_SIZE;WRITE_SIZE" --scene 0 --spp 512 --bounces 16 --ppm
step gloo2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --spp 64 --dist-backend gloo --no-e2e --pipelined-steps 0
tail -2 gpurun_out/bench.log gpurun_out/gloo2.log
