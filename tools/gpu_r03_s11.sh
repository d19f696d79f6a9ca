#!/bin/bash
# Round-3 session 11: sparse hot waves (RT_PRIO_LANES x RT_PRIO_TILES) on every BASELINE config shape:
# Perlin fine-tuning, then scene 0, Cornell, the 10k scene and the other noise scene (19).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)" >&2; tail -40 "gpurun_out/$name.log" >&2; exit $rc; fi
}
export ROUNDS=2
VARIANTS="base|;l2t8|RT_PRIO_LANES=2 RT_PRIO_TILES=8;l2t12|RT_PRIO_LANES=2 RT_PRIO_TILES=12;l2t16|RT_PRIO_LANES=2 RT_PRIO_TILES=16;l2t24|RT_PRIO_LANES=2 RT_PRIO_TILES=24;l3t16|RT_PRIO_LANES=3 RT_PRIO_TILES=16;l4t12|RT_PRIO_LANES=4 RT_PRIO_TILES=12" \
BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 3 --warmup 1" step ab_s17 600 bash tools/gpu_ab_env.sh gpurun_out/ab_sparse_s17b.jsonl
VARIANTS="base|;l4t16|RT_PRIO_LANES=4 RT_PRIO_TILES=16;l2t16|RT_PRIO_LANES=2 RT_PRIO_TILES=16;l8t32|RT_PRIO_LANES=8 RT_PRIO_TILES=32" \
BENCH_ARGS="--scene 0 --spp 512 --bounces 16 --steps 5 --warmup 1" step ab_s0 600 bash tools/gpu_ab_env.sh gpurun_out/ab_sparse_s0.jsonl
VARIANTS="base|;l4t16|RT_PRIO_LANES=4 RT_PRIO_TILES=16;l2t16|RT_PRIO_LANES=2 RT_PRIO_TILES=16;l8t32|RT_PRIO_LANES=8 RT_PRIO_TILES=32" \
BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 3 --warmup 1" step ab_s1 600 bash tools/gpu_ab_env.sh gpurun_out/ab_sparse_s1.jsonl
VARIANTS="base|;l4t16|RT_PRIO_LANES=4 RT_PRIO_TILES=16;l8t32|RT_PRIO_LANES=8 RT_PRIO_TILES=32" \
BENCH_ARGS="--scene 20 --spp 256 --bounces 16 --steps 3 --warmup 1" step ab_s20 600 bash tools/gpu_ab_env.sh gpurun_out/ab_sparse_s20.jsonl
VARIANTS="base|;l2t16|RT_PRIO_LANES=2 RT_PRIO_TILES=16;l4t16|RT_PRIO_LANES=4 RT_PRIO_TILES=16" \
BENCH_ARGS="--scene 19 --spp 1024 --bounces 50 --steps 3 --warmup 1" step ab_s19 600 bash tools/gpu_ab_env.sh gpurun_out/ab_sparse_s19.jsonl
for f in gpurun_out/ab_sparse_*.jsonl; do echo "$f"; python3 -c "
import json,sys,collections
d=collections.defaultdict(list)
for l in open(sys.argv[1]): j=json.loads(l); d[j['label']].append(j['ms_per_step'])
print({k: v for k,v in d.items()})" "$f"; done
