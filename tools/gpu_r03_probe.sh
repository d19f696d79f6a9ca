#!/bin/bash
# Round-3 opening session: host CPU share probe, pytest -m gpu, PMC of the 10k-sphere and final_scene
# render kernels.  Each GPU step has its own limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.log >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
}
{
  echo "nproc: $(nproc)"; echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>&1)"
  echo "cpuset: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>&1)"
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
  lscpu | head -25; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"
} > gpurun_out/host_probe.log 2>&1
step pytest_gpu 600 python3 -u -m pytest tests -q -m gpu -x --timeout 180 --timeout-method thread
step pmc_s20 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s20" --scene 20 --spp 256 --bounces 16
step pmc_s3 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s3" --scene 3 --width 800 --height 800 --spp 16 --bounces 40
cat gpurun_out/host_probe.log
