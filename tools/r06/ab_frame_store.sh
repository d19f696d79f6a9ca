#!/bin/bash
# r06: frame-store A/Bs under LLVM 22 — Perlin with tile-major output (round 5: +15-21 % under LLVM 20), the 10k scene's
# tile frame with non-temporal stores, and the untile kernel on the high-priority stream vs the caller's stream
# (rocprofv3 kernel stats of the default bench, pipelined leg included)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
VARIANTS="row|RT_TILED_OUT=0;tiled|RT_TILED_OUT=1" ROUNDS=3 LIM=300 BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh $O/ab_perlin_tiled.jsonl || exit 1
VARIANTS="def|RT_AB=0;nt|RT_JIT_OPTS=-DRT_NT_FRAME" ROUNDS=3 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh $O/ab_10k_nt.jsonl || exit 1
for v in prio noprio; do
  e=""; [ $v = noprio ] && e="RT_UNTILE_PRIO=0"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_untile_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/untile_$v.json 2> $O/untile_$v.err || { tail -3 $O/untile_$v.err; exit 1; }
done
find $O/prof_untile_* -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -i "untile\|render\"" "$f" | cut -c1-200; done
