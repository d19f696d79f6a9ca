#!/bin/bash
# r05 final 4: rocprofv3 kernel-trace summaries of the bench command on the other BASELINE configs (final tree), each
# under its own limit -> profiles/r05_f4_kernel_stats_<config>.csv (+ the bench line)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/f4_$name" -o run -- python3 bench.py \
    --pipelined-steps 0 --no-cpu-baseline --no-e2e "$@" > "gpurun_out/f4_$name.log" 2>&1 || { echo "$name failed"; tail -5 "gpurun_out/f4_$name.log"; exit 1; }
  echo "$name ok"
}
run c3_cornell --scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1
run c3_perlin --scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1
run c4_10k --scene 20 --spp 256 --steps 3 --warmup 1
run c5_4k --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1
echo done
