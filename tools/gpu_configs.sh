#!/bin/bash
# Every BASELINE.json config that fits one GPU, through bench.py (one JSON line each) into
# gpurun_out/configs.jsonl.  Config 4 (10k spheres, 8 GPUs) and 5 (4K, 8 GPUs) are run here as their
# one-GPU workloads; the driver's N-GPU runs cover the row sharding.  Each step has its own limit; a
# fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {  # name, limit, bench args...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" python3 bench.py "$@" > "gpurun_out/cfg_$name.log" 2> "gpurun_out/cfg_$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  [ $rc -ne 0 ] && { tail -5 "gpurun_out/cfg_$name.err" >&2; exit $rc; }
  tail -1 "gpurun_out/cfg_$name.log" >> gpurun_out/configs.jsonl
}
run c2_scene0_1080p ${LIM:-300} --scene 0 --spp 512 --bounces 16 --steps 5 --warmup 1
run c3_scene1_cornell ${LIM:-300} --scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1
run c3_scene17_perlin ${LIM:-300} --scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1
run c4_scene20_10k ${LIM:-300} --scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1
run c5_scene0_4k ${LIM:-300} --scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1
# final_scene (raytracing.cu:2151-2202; §8f row 1, not a BASELINE config) at the reference's 800x800, d40,
# a bounded spp (the reference's own spp would take minutes per frame)
[ -n "${WITH_FINAL:-}" ] && run c6_scene3_final ${LIM:-300} --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1
cat gpurun_out/configs.jsonl
