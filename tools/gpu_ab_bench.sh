#!/bin/bash
# Same-box A/B of bench.py's single-frame step (base tree _base vs this tree), alternating, N rounds.
# Each step has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for side in base new; do
    d=.; [ $side = base ] && d=_base
    (cd $d && timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e --pipelined-steps 0 ${BENCH_ARGS:-}) > gpurun_out/abb_${side}_r$r.json 2> gpurun_out/abb_${side}_r$r.err || { echo "$side r$r failed"; tail -5 gpurun_out/abb_${side}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms_per_step', d['ms_per_step'], d['kernel_ms'])" gpurun_out/abb_${side}_r$r.json "$side r$r"
  done
done
