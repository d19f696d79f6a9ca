#!/bin/bash
# Same-box A/B: times tools/tune.py in a baseline tree (AB_BASE, default _base: a git worktree of the
# commit to compare against, built with `make` there; drop ./_base from .gpurunignore for the call) and
# in this tree, alternating, per case (scene:spp:bounces).
#   AB_CASES="0:128:16 1:64:50 17:64:50 20:32:16" AB_CONFIG="RT_JIT_FOLD=1" bash tools/gpu_ab.sh
# Each GPU step runs under its own limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
base=${AB_BASE:-_base}
step() {  # name, limit, dir, command...
  local name=$1 lim=$2 dir=$3; shift 3
  (cd "$dir" && timeout -k 10 "$lim" "$@") > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
for r in 1 2; do
  for cs in ${AB_CASES:-0:128:16 1:64:50 17:64:50}; do
    IFS=: read -r sc spp b <<< "$cs"
    for side in base new; do
      d=.; [ $side = base ] && d=$base
      step "ab_${side}_s${sc}_r$r" 180 "$d" python3 tools/tune.py --scene "$sc" --spp "$spp" --bounces "$b" \
        --configs "${AB_CONFIG:-RT_JIT_FOLD=1}" --rounds 3
    done
  done
done
grep -H "median" gpurun_out/ab_*.log
