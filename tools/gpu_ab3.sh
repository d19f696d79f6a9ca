#!/bin/bash
# Same-box A/B/C: base tree (_base), this tree, this tree with extra env (AB_ENV), per case scene:spp:bounces.
# Each step has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for cs in ${AB_CASES:-20:32:16}; do
    IFS=: read -r sc spp b <<< "$cs"
    for side in base new env; do
      d=.; [ $side = base ] && d=_base
      e=""; [ $side = env ] && e="$AB_ENV"
      (cd $d && env $e timeout -k 10 180 python3 tools/tune.py --scene "$sc" --spp "$spp" --bounces "$b" --configs RT_JIT_FOLD=1 --rounds 3) > gpurun_out/ab3_${side}_s${sc}_r$r.log 2>&1 || { echo "ab3_${side}_s${sc}_r$r failed"; tail -5 gpurun_out/ab3_${side}_s${sc}_r$r.log; exit 1; }
    done
  done
done
grep -H median gpurun_out/ab3_*.log
