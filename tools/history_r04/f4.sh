#!/bin/bash
# r04 final 4: the N > 1 bench path rehearsed with two ranks sharing the box's one MI355X (gloo collectives: the
# RCCL path needs one GPU per rank), scene 0 at a reduced spp, and the 10k config with the frame split two ways.
# -> profiles/r04_f4_gloo2_*.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --dist-backend gloo --spp 64 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/gloo2_scene0.json 2> gpurun_out/gloo2_scene0.err \
  || { echo rc=$?; tail -20 gpurun_out/gloo2_scene0.err; exit 1; }
tail -c 800 gpurun_out/gloo2_scene0.json
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 2 --dist-backend gloo --scene 20 --spp 16 --frame fixed --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/gloo2_10k.json 2> gpurun_out/gloo2_10k.err \
  || { echo rc=$?; tail -20 gpurun_out/gloo2_10k.err; exit 1; }
tail -c 800 gpurun_out/gloo2_10k.json
echo done
