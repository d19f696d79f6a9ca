#!/bin/bash
# r06: PMC of the scene-0 and 10k render kernels on the LLVM 22 build (lane utilisation, issue / wait cycles, bytes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/pmc
mkdir -p $O
timeout -k 10 600 python3 tools/profile_pmc.py --out "$PWD/$O/s0" --scene 0 --spp 128 --ppm > $O/s0.log 2>&1 || { tail -5 $O/s0.log; exit 1; }
timeout -k 10 600 python3 tools/profile_pmc.py --out "$PWD/$O/10k" --scene 20 --spp 32 --ppm > $O/10k.log 2>&1 || { tail -5 $O/10k.log; exit 1; }
python3 - <<'PY'
import json
for n in ("s0", "10k"):
    d = json.load(open(f"gpurun_out/r06/pmc/{n}/summary.json"))
    print(n, json.dumps(d.get("derived", {}))[:1500])
PY
