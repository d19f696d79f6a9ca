#!/bin/bash
# final_scene PMC of rt_mixed_render (pausable walk, packed chains): issue vs wait, lane utilisation
mkdir -p gpurun_out
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >&2; return $rc; }
step pmc_s3 600 python3 tools/profile_pmc.py --out "$PWD/gpurun_out/pmc_s3" --sets "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_BRANCH,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES;SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE" --scene 3 --width 800 --height 800 --spp 16 --bounces 40 --ppm
