#!/bin/bash
# final_scene at the bench configuration (800x800, spp 64, d40) on the current tree
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step c6_final 400 python3 bench.py --scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1
