#!/bin/bash
# r05 s13: tail pieces (RT_TAIL_CHUNK / RT_TAIL_GEN: the last ids of the longest-first order handed out in small pieces):
# parity tests; wave traces of the 10k and scene-0 frames with and without; same-box A/Bs of both configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/s13_steps.log
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/s13_steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step s13_tail_tests 400 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread -k "tail_pieces or tail_issue or tile_schedules"
step s13_wt_10k_def 200 python3 tools/wave_trace.py --scene 20 --spp 64
step s13_wt_10k_t8 200 python3 tools/wave_trace.py --scene 20 --spp 64 --env RT_TAIL_CHUNK=8
step s13_wt_10k_t1 200 python3 tools/wave_trace.py --scene 20 --spp 64 --env RT_TAIL_CHUNK=1
step s13_wt_s0_def 200 python3 tools/wave_trace.py --scene 0 --spp 512
step s13_wt_s0_t8 200 python3 tools/wave_trace.py --scene 0 --spp 512 --env RT_TAIL_CHUNK=8
ROUNDS=2 VARIANTS="def|RT_TAIL_CHUNK=0;t8|RT_TAIL_CHUNK=8;t1|RT_TAIL_CHUNK=1;t8g2|RT_TAIL_CHUNK=8 RT_TAIL_GEN=2" \
  BENCH_ARGS="--scene 20 --spp 256 --steps 3 --warmup 1" step s13_ab_10k 900 bash tools/gpu_ab_env.sh gpurun_out/ab_s13_10k.jsonl
ROUNDS=2 VARIANTS="def|RT_TAIL_CHUNK=0;t8|RT_TAIL_CHUNK=8;t1|RT_TAIL_CHUNK=1" \
  BENCH_ARGS="--steps 5 --warmup 1" step s13_ab_scene0 600 bash tools/gpu_ab_env.sh gpurun_out/ab_s13_scene0.jsonl
tail -n 3 gpurun_out/s13_tail_tests.log
for f in gpurun_out/s13_wt_*.log; do echo "== $f"; sed -n 2,8p "$f"; done
cut -c1-200 gpurun_out/ab_s13_10k.jsonl gpurun_out/ab_s13_scene0.jsonl
