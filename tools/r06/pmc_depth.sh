#!/bin/bash
# r06: VALU lane utilisation by path depth — camera rays only (d1) against deeper limits — on scene 0 and the 10k
# config: how much of the idle lane share is the bounce rays' divergence rather than empty lanes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06/pmc_depth
mkdir -p $O
S1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
S2="SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE"
run() {  # name scene spp bounces
  timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/$O/$1" --sets "$S1;$S2" --scene $2 --spp $3 --bounces $4 --ppm \
    > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1/summary.json')); k=[x for x in d['merged'] if x.endswith('_render')][0]; print('$1', k, d['derived'][k])"
}
run s0_d1 0 128 1 && run s0_d2 0 128 2 && run s0_d4 0 128 4 && run s0_d16 0 128 16 && run 10k_d1 20 32 1 && run 10k_d16 20 32 16
