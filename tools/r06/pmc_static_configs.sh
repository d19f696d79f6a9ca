#!/bin/bash
# r06: final-tree lane utilisation and instruction counts of the Cornell, Perlin and 4K kernels (reduced spp)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06/pmc_static
mkdir -p $O
S1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
S2="SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE"
run() {
  timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/$O/$1" --sets "$S1;$S2" "${@:2}" --ppm > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1/summary.json')); k=[x for x in d['merged'] if x.endswith('_render')][0]; m=d['merged'][k]; print('$1', k, d['derived'][k], 'VALU %.3g SALU %.3g' % (m['SQ_INSTS_VALU'], m['SQ_INSTS_SALU']))"
}
run cornell_spp128 --scene 1 --spp 128 --bounces 50 && run perlin_spp128 --scene 17 --spp 128 --bounces 50 && run s0_4k_spp64 --scene 0 --width 3840 --height 2160 --spp 64 --bounces 50
