#!/bin/bash
# r06: tile-major parity subset, then the untile kernel's duration under rocprofv3 in the default bench (its pipelined leg
# overlaps the next frame's render kernel): untile at top issue priority (default) vs RT_UNTILE_PRIO=0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "tiled_output or fused_ppm" > $O/untile_tests.txt 2>&1 || { tail -5 $O/untile_tests.txt; exit 1; }
tail -1 $O/untile_tests.txt
for v in prio noprio; do
  e="RT_AB=0"; [ $v = noprio ] && e="RT_UNTILE_PRIO=0"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_untile2_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/untile2_$v.json 2> $O/untile2_$v.err || { tail -3 $O/untile2_$v.err; exit 1; }
done
find $O/prof_untile2_* -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -i "untile\|static_render\"" "$f" | cut -c1-220; done
