#!/bin/bash
# r05 s29: the deep kernels' LDS unwind batch (RT_UNWIND_LDS_DEEP 8 -> 6 lands Cornell's static kernel at 80 VGPRs without
# spills offline): same-box A/Bs on Cornell, Perlin and the 4K d50 config (RT_DEBUG register lines kept)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s29_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s29_steps.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
V="def|RT_AB=0;b6|RT_JIT_OPTS=-DRT_UNWIND_LDS_DEEP=6;b5|RT_JIT_OPTS=-DRT_UNWIND_LDS_DEEP=5"
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 1 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s29_ab_cornell 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s29_cornell.jsonl
ROUNDS=2 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 17 --spp 1024 --bounces 50 --steps 2 --warmup 1" \
  step s29_ab_perlin 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s29_perlin.jsonl
ROUNDS=1 LIM=300 VARIANTS="$V" BENCH_ARGS="--scene 0 --width 3840 --height 2160 --spp 2048 --bounces 50 --steps 2 --warmup 1" \
  step s29_ab_4k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s29_4k.jsonl
for f in gpurun_out/ab_s29_*.jsonl; do echo "== $f"; python3 -c "
import json,sys,collections
r=collections.defaultdict(list)
for l in open('$f'):
    d=json.loads(l); r[d['label']].append(d['kernel_ms']['render_median'])
print(dict(r))"; done
