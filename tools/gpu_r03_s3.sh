#!/bin/bash
# Round-3 session 3: mixed-world walk (new tests first, then final_scene A/B), spill tests, full suite,
# default bench, scene-0 traffic, 2-rank gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -40 "gpurun_out/$name.log" >&2; exit $rc; fi
}
step pytest_new 300 python3 -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread -k "mixed or colour_stack or deep_unwind or seeding"
step s3_mixed 300 python3 bench.py --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --pipelined-steps 0
RT_MIXED=0 step s3_lane 300 python3 bench.py --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --pipelined-steps 0
step pytest_gpu 600 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread
step bench 400 python3 bench.py
step traffic_s0 300 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/traffic_s0" --sets "FETCH_SIZE;WRITE_SIZE" --scene 0 --spp 512 --bounces 16 --ppm
step gloo2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 3 --warmup 1 --spp 64 --dist-backend gloo --no-e2e --pipelined-steps 0
tail -2 gpurun_out/s3_*.log gpurun_out/bench.log gpurun_out/gloo2.log
