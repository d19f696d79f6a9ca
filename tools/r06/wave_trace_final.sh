#!/bin/bash
# r06: per-wave timelines of the final tree (scene 0 and the 10k config at full spp): where the single frame idles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/wave_trace
mkdir -p $O
timeout -k 10 300 python3 tools/wave_trace.py --scene 0 --spp 512 --bounces 16 > $O/scene0.txt 2>&1 || { tail -5 $O/scene0.txt; exit 1; }
timeout -k 10 300 python3 tools/wave_trace.py --scene 20 --spp 256 --bounces 16 > $O/10k.txt 2>&1 || { tail -5 $O/10k.txt; exit 1; }
tail -25 $O/scene0.txt; tail -25 $O/10k.txt
