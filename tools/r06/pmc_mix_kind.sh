#!/bin/bash
# r06: PMC of the mixed walk's render kernel (final_scene, spp 16) with and without kind-scheduled trips
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06/pmc_mix_kind
mkdir -p $O
S1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES"
S2="SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE"
for v in def kind; do
  e="RT_AB=0"; [ $v = kind ] && e="RT_JIT_OPTS=-DRT_MIX_KIND=1"
  env $e timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/$O/$v" --sets "$S1;$S2" --scene 3 --width 800 --height 800 \
    --spp 16 --bounces 40 --ppm > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v/summary.json')); k=[x for x in d['merged'] if x.endswith('_render')][0]; m=d['merged'][k]; print('$v', k, d['derived'][k], 'VALU %.3g SALU %.3g' % (m['SQ_INSTS_VALU'], m['SQ_INSTS_SALU']))"
done
