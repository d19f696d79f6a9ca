#!/bin/bash
# bench with single-frame steps queued back to back on one stream; two-rank gloo rehearsal
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step bench_q1 400 python3 bench.py --no-cpu-baseline --no-e2e &&
step bench_q2 400 python3 bench.py --no-cpu-baseline --no-e2e &&
step gloo2q 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --spp 64 --dist-backend gloo --no-e2e --pipelined-steps 0 --no-cpu-baseline
