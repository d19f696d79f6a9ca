#!/bin/bash
# r05 final 2 (final tree): every BASELINE config through bench.py (+ final_scene), then the render kernel's HBM traffic
# of each (FETCH_SIZE x2 + WRITE_SIZE, separate passes) for profiles/hbm_traffic.json (tools/r04/apply_traffic.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
WITH_FINAL=1 bash tools/gpu_configs.sh || exit $?
bash tools/gpu_traffic_configs.sh || exit $?
echo done
