"""Write profiles/hbm_traffic.json (bench.py roofline.traffic) from a profile_pmc.py summary.

    python3 tools/traffic_from_pmc.py <summary.json> <workload> [kernel=rt_static_render] [launches=1]
HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) KiB x 1024 / launches: FETCH_SIZE doubled per
MI355X_MICROARCH.md §HBM (gfx950 reports half of wide reads), WRITE_SIZE as reported.
`step_bytes` is the same sum over every kernel of the profiled step (seeding, schedule probe, tile order,
render, runtime fills / copies), with the per-kernel split in `step_kernels`.
"""
import json, sys
from pathlib import Path

summ, workload = Path(sys.argv[1]), sys.argv[2]
kernel = sys.argv[3] if len(sys.argv) > 3 else "rt_static_render"
launches = int(sys.argv[4]) if len(sys.argv) > 4 else 1
m = json.loads(summ.read_text())["merged"][kernel]
fetch = m["FETCH_SIZE"] * 1024 * 2 / launches
write = m["WRITE_SIZE"] * 1024 / launches
out = Path(__file__).resolve().parents[1] / "profiles" / "hbm_traffic.json"
d = json.loads(out.read_text()) if out.exists() else {}
merged = json.loads(summ.read_text())["merged"]
split = {}
for k, v in merged.items():
    b = (2 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)) * 1024 / launches
    split[k.replace("rt::(anonymous namespace)::", "").split("(")[0]] = int(b)
d[workload] = {"bytes": int(fetch + write), "fetch_bytes_x2": int(fetch), "write_bytes": int(write), "kernel": kernel,
               "step_bytes": sum(split.values()), "step_kernels": split,
               "source": f"{summ} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, {launches} launch(es))",
               "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE as reported, KiB x 1024"}
out.write_text(json.dumps(d, indent=1) + "\n")
print(json.dumps(d[workload], indent=1))
