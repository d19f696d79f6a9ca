#!/bin/bash
# r06: the 10k camera rays' candidate-list entries read with the non-temporal hint (RT_NT_LISTS): can the list reads
# stop evicting partially written tile-frame lines from L2?  Render-kernel bytes (PMC) and a same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06/nt_lists
mkdir -p $O
for v in def ntl; do
  e="RT_AB=0"; [ $v = ntl ] && e="RT_JIT_OPTS=-DRT_NT_LISTS"
  env $e timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/$O/$v" --sets "FETCH_SIZE;WRITE_SIZE;TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum" \
    --scene 20 --width 1920 --height 1080 --spp 256 --bounces 16 --ppm > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v/summary.json')); k=[x for x in d['merged'] if x.endswith('_render')][0]; m=d['merged'][k]; print('$v', {a: b for a, b in m.items()})"
done
VARIANTS="def|RT_AB=0;ntl|RT_JIT_OPTS=-DRT_NT_LISTS" ROUNDS=3 LIM=300 BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" \
  bash tools/gpu_ab_env.sh gpurun_out/r06/ab_10k_nt_lists.jsonl || exit 1
