#!/bin/bash
# r06: Perlin render-kernel HBM traffic measured three times in a row (the fetch varied between runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r06/perlin_traffic
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 tools/profile_pmc.py --out "$PWD/$O/run$i" --sets "FETCH_SIZE;WRITE_SIZE" --scene 17 --width 1920 --height 1080 \
    --spp 1024 --bounces 50 --ppm > $O/run$i.log 2>&1 || { tail -20 $O/run$i.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/run$i/summary.json')); k=[x for x in d['merged'] if x.endswith('_render')][0]; print('run$i', d['merged'][k])"
done
