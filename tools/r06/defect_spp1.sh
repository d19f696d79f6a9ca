#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}/_old"
export TMPDIR=/tmp RT_JIT_CACHE_DIR=0
O=../gpurun_out/spp1
mkdir -p $O
for spp in 1 4; do
RT_JIT_LOAD_ACCEL=co/e_none.co timeout -k 10 120 python3 tools/r05/dbg20.py --spp $spp --save $O/s$spp "none|" > $O/none$spp.log 2>&1 || { echo "failed"; tail -5 $O/none$spp.log; exit 1; }
grep differing $O/none$spp.log
done
RT_JIT_LOAD_ACCEL=co/e_none.co timeout -k 10 120 python3 tools/r05/dbg20.py --spp 1 --bounces 1 --save $O/b1 "none|" > $O/b1.log 2>&1 || exit 1
grep differing $O/b1.log
RT_JIT_LOAD_ACCEL=co/e_none.co timeout -k 10 120 python3 tools/r05/dbg20.py --spp 1 --bounces 2 --save $O/b2 "none|" > $O/b2.log 2>&1 || exit 1
grep differing $O/b2.log
