#!/bin/bash
# One knob swept in this tree with tools/tune.py (isolated frames, configs alternated in one process),
# per case scene:spp:bounces.  SWEEP="RT_X=0,RT_X=1" CASES="0:512:16 1:256:50" bash tools/gpu_sweep.sh
# Each step has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cs in ${CASES:-0:512:16}; do
  IFS=: read -r sc spp b <<< "$cs"
  timeout -k 10 400 python3 tools/tune.py --scene "$sc" --spp "$spp" --bounces "$b" --configs "$SWEEP" --rounds ${ROUNDS:-3} > gpurun_out/sweep_s$sc.log 2>&1 || { echo "s$sc failed"; tail -5 gpurun_out/sweep_s$sc.log; exit 1; }
  echo "== scene $sc spp $spp d$b"; grep median gpurun_out/sweep_s$sc.log
done
