#!/bin/bash
# rocprofv3 --kernel-trace --stats of bench.py's isolated frames for every BASELINE config (one pass each)
# into gpurun_out/prof_cfg/<name>/.  Each step has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_cfg
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_cfg/$name" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --pipelined-steps 0 --no-cpu-baseline --no-e2e "$@" > "gpurun_out/prof_cfg/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "gpurun_out/prof_cfg/$name.log"; exit $rc; }
  return 0
}
run c3_scene1_cornell --scene 1 --spp 1024 --bounces 50
run c3_scene17_perlin --scene 17 --spp 1024 --bounces 50
run c4_scene20_10k --scene 20 --spp 256 --bounces 16
run c5_scene0_4k --scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50
run c6_scene3_final --scene 3 --width 800 --height 800 --spp 64 --bounces 40
