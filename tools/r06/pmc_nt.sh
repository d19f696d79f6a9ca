#!/bin/bash
# r06: render-kernel HBM bytes of the 10k config with non-temporal tile-frame stores (RT_NT_FRAME) vs the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06/pmc_nt
mkdir -p $O
for v in def nt; do
  e="RT_AB=0"; [ $v = nt ] && e="RT_JIT_OPTS=-DRT_NT_FRAME"
  env $e timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/$O/$v" --sets "FETCH_SIZE;WRITE_SIZE;TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum" \
    --scene 20 --width 1920 --height 1080 --spp 256 --bounces 16 --ppm > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
done
