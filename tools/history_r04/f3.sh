#!/bin/bash
# r04 final 3 (final tree: span fix, viewport point carried): full -m gpu suite, smoke, the default bench line, the
# rocprofv3 kernel-trace summary of its frames, the carried-point A/B on scene 0 (tools/r04/v19.sh's variants, one
# round), PMC of the scene-0 and 10k kernels.
# -> profiles/r04_f3_pytest_gpu.txt, r04_f3_bench.json, r04_f3_kernel_stats.csv, r04_ab_f3_scene0.jsonl, r04_f3_pmc_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...   (stop on any failure)
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "gpurun_out/$name.log" | head -20; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
step pytest_gpu 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
tail -1 gpurun_out/pytest_gpu.log
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
tail -c 400 gpurun_out/bench.log
step rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 bench.py --steps 3 --warmup 1 --pipelined-steps 0 --no-cpu-baseline --no-e2e
L=$PWD/ablib
ROUNDS=1 VARIANTS="pp|RT_AB_NEW=1;nopp|RT_HIP_LIB=$L/librt_hip_ae039e0.so;base|RT_HIP_LIB=$L/librt_hip_r04base.so" \
  BENCH_ARGS="--steps 6 --warmup 1" bash tools/gpu_ab_env.sh gpurun_out/ab_f3_scene0.jsonl || exit $?
step pmc_s0 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s0" --scene 0 --spp 128 --ppm
step pmc_s20 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s20" --scene 20 --spp 32 --ppm
echo done
