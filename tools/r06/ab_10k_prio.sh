#!/bin/bash
# r06: the 10k frame's tail (waves end at 77 % of the span in the median): mixed hot waves (RT_PRIO_MIX=1, the costliest
# quarter of the tiles handed out pixel by pixel over every wave), tail issue priority (RT_TAIL_PRIO=1), vs the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
VARIANTS="def|RT_AB=0;pmix|RT_PRIO_MIX=1;tprio|RT_TAIL_PRIO=1" ROUNDS=3 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/r06/ab_10k_prio.jsonl || exit 1
