#!/bin/bash
# ISA-surgery probes of the failing tree's (bce6c5e) 6-wave accel kernel on scene 20 (64x36, spp 2, d16)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}/_old"
export TMPDIR=/tmp RT_JIT_CACHE_DIR=0
O=../gpurun_out/surg
mkdir -p $O
for v in none readlane writelane both llvm22; do
  for rep in 1 2; do
    RT_JIT_LOAD_ACCEL=co/e_$v.co timeout -k 10 120 python3 tools/r05/dbg20.py --spp 2 "$v|" > $O/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.$rep.log; exit 1; }
    grep -v amdgpu.ids $O/$v.$rep.log | grep "differing\|loaded"
  done
done
