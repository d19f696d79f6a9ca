#!/bin/bash
# Round-3 session 14: final_scene knob sweep (mixed walk leaf size / dynamic-macro threshold, sparse hot
# waves lanes x tiles), same box, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export ROUNDS=2
export VARIANTS="base|;leaf2|RT_MIX_LEAF=2;leaf8|RT_MIX_LEAF=8;dyn32|RT_MIX_DYN_MIN=32;dyn256|RT_MIX_DYN_MIN=256;l1t16|RT_PRIO_LANES=1;l4t16|RT_PRIO_LANES=4;l2t8|RT_PRIO_TILES=8;l2t32|RT_PRIO_TILES=32"
export BENCH_ARGS="--scene 3 --width 800 --height 800 --spp 64 --bounces 40 --steps 2 --warmup 1"
timeout -k 10 1000 bash tools/gpu_ab_env.sh gpurun_out/ab_final_knobs.jsonl || exit $?
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('gpurun_out/ab_final_knobs.jsonl'): j=json.loads(l); d[j['label']].append(j['ms_per_step'])
print(dict(d))"
