#!/usr/bin/env python3
"""Collect PMC counters for the render kernel in separate rocprofv3 passes and summarize.

    python3 tools/profile_pmc.py --out gpurun_out/pmc [workload args...]

Each pass is its own rocprofv3 process (--pmc + --kernel-trace only, never with trace domains).
Writes <out>/summary.json: per pass, per kernel, the summed counter values, plus derived metrics.
"""
import csv, json, os, subprocess, sys
from collections import defaultdict
from pathlib import Path

PASSES = [
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH",
     "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"],
    ["SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_SMEM", "GRBM_GUI_ACTIVE"],
    ["SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32",
     "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64"],
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
]


def main():
    args = sys.argv[1:]
    out = Path(args[args.index("--out") + 1]) if "--out" in args else Path("gpurun_out/pmc")
    if "--out" in args:
        i = args.index("--out"); del args[i:i + 2]
    passes = PASSES
    if "--sets" in args:   # custom passes: "A,B;C,D"
        i = args.index("--sets")
        passes = [x.split(",") for x in args[i + 1].split(";")]
        del args[i:i + 2]
    out = out.resolve()
    out.mkdir(parents=True, exist_ok=True)
    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, TMPDIR="/tmp")
    summary = {"workload": args, "passes": []}
    for k, counters in enumerate(passes):
        d = out / f"pass{k}"
        cmd = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "--output-format", "csv", "-d", str(d), "-o", "run",
               "--", sys.executable, str(repo / "tools" / "pmc_workload.py"), *args]
        r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=900)
        (out / f"pass{k}.log").write_text(r.stdout[-20000:] + "\n---\n" + r.stderr[-20000:])
        if r.returncode != 0:
            print(f"pass {k} failed rc={r.returncode}", file=sys.stderr)
            sys.exit(r.returncode if r.returncode > 0 else 3)
        vals = defaultdict(lambda: defaultdict(float))
        for f in d.rglob("*counter_collection.csv"):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    vals[row["Kernel_Name"]][row["Counter_Name"]] += float(row["Counter_Value"])
        summary["passes"].append({k2: dict(v) for k2, v in vals.items()})
        print(f"pass {k} ok", flush=True)
    merged = defaultdict(dict)
    for p in summary["passes"]:
        for kname, v in p.items():
            merged[kname].update(v)
    derived = {}
    for kname, v in merged.items():
        dd = {}
        if v.get("SQ_ACTIVE_INST_VALU"):
            dd["valu_lane_util"] = v.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * v["SQ_ACTIVE_INST_VALU"])
        if v.get("SQ_WAVE_CYCLES"):
            dd["valu_issue_frac_of_wave_cycles"] = v.get("SQ_ACTIVE_INST_VALU", 0) / v["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in v or "WRITE_SIZE" in v:
            dd["hbm_bytes_fetch_x2_plus_write"] = 1024 * (2 * v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0))
            dd["hbm_bytes_raw"] = 1024 * (v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0))
        derived[kname] = dd
    summary["merged"] = merged
    summary["derived"] = derived
    (out / "summary.json").write_text(json.dumps(summary, indent=1))
    print(json.dumps(derived, indent=1))


if __name__ == "__main__":
    main()
