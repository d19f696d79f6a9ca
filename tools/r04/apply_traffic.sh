#!/bin/bash
# After tools/r04/v10.sh: write every profiled workload's bytes into profiles/hbm_traffic.json (bench.py
# roofline.traffic) and keep the summaries under profiles/r04_v10_traffic/.  Runs here (no GPU).
cd "$(dirname "$0")/../.."
while read -r name kernel; do
  [ -z "$name" ] && continue
  python3 tools/traffic_from_pmc.py "gpurun_out/traffic_cfg/$name/summary.json" "$name" "$kernel" > /dev/null || exit 1
  mkdir -p "profiles/r04_v10_traffic/$name"
  cp "gpurun_out/traffic_cfg/$name/summary.json" "profiles/r04_v10_traffic/$name/summary.json"
done < gpurun_out/traffic_cfg/kernels.txt
python3 - <<'PY'
import json
d = json.load(open("profiles/hbm_traffic.json"))
for k, v in d.items():
    if "source" in v and "r04" not in v["source"] and "traffic_cfg" in v["source"]:
        v["source"] = v["source"].replace("gpurun_out/traffic_cfg", "profiles/r04_v10_traffic")
    print(f"{k:55s} render {v['bytes']/1e6:8.1f} MB  step {v.get('step_bytes', 0)/1e6:8.1f} MB")
json.dump(d, open("profiles/hbm_traffic.json", "w"), indent=1)
PY
