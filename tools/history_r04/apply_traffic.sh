#!/bin/bash
# After tools/r04/v10.sh / f1.sh: write every profiled workload's bytes into profiles/hbm_traffic.json (bench.py
# roofline.traffic) and keep the summaries under profiles/<dir> (default r04_v10_traffic).  Runs here (no GPU).
#   bash tools/r04/apply_traffic.sh [dir]
cd "$(dirname "$0")/../.."
DIR=${1:-r04_v10_traffic}
while read -r name kernel; do
  [ -z "$name" ] && continue
  python3 tools/traffic_from_pmc.py "gpurun_out/traffic_cfg/$name/summary.json" "$name" "$kernel" > /dev/null || exit 1
  mkdir -p "profiles/$DIR/$name"
  cp "gpurun_out/traffic_cfg/$name/summary.json" "profiles/$DIR/$name/summary.json"
done < gpurun_out/traffic_cfg/kernels.txt
DIR=$DIR python3 - <<'PY'
import json, os
d = json.load(open("profiles/hbm_traffic.json"))
target = "profiles/" + os.environ["DIR"]
for k, v in d.items():
    if "source" in v and "gpurun_out/traffic_cfg" in v["source"]:
        v["source"] = v["source"].replace("gpurun_out/traffic_cfg", target)
    print(f"{k:55s} render {v['bytes']/1e6:8.1f} MB  step {v.get('step_bytes', 0)/1e6:8.1f} MB")
json.dump(d, open("profiles/hbm_traffic.json", "w"), indent=1)
PY
