#!/bin/bash
# r05 final 1 (final tree): full -m gpu suite, smoke, the default bench line, the rocprofv3 kernel-trace summary of the
# same bench command, `bench.py --gpus 2` on the one-GPU box (must fail loudly, status 2), PMC of the scene-0 kernel.
# -> profiles/r05_f1_pytest_gpu.txt, r05_f1_bench.json, r05_f1_kernel_stats.csv, r05_f1_gpus2.txt, r05_pmc/f1_*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name, limit, command...   (stop on any failure)
  local name=$1 lim=$2; shift 2
  echo "== $name $(date +%T)" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/f1_steps.log >&2
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" "gpurun_out/$name.log" | head -20; tail -20 "gpurun_out/$name.log"; exit $rc; fi
}
step f1_pytest_gpu 900 python3 -u -m pytest tests -v -m gpu --timeout 180 --timeout-method thread
tail -1 gpurun_out/f1_pytest_gpu.log
step f1_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step f1_bench 600 python3 bench.py
tail -c 600 gpurun_out/f1_bench.log
step f1_rocprof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/f1_prof" -o run -- python3 bench.py
# N=2 on a one-GPU box: the launcher must refuse (status 2, "needs 2 GPUs"), before any rank starts
timeout -k 10 120 python3 bench.py --gpus 2 > gpurun_out/f1_gpus2.log 2>&1
echo "bench.py --gpus 2 rc=$?" | tee -a gpurun_out/f1_gpus2.log gpurun_out/f1_steps.log
step f1_pmc_s0 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/f1_pmc_s0" --scene 0 --spp 128 --ppm
echo done
