#!/bin/bash
# Same-box A/B of environment variants of one bench.py configuration, alternating, ROUNDS rounds:
#   VARIANTS="label1|ENV=A ENV2=B;label2|ENV=C" BENCH_ARGS="--scene 20 --spp 256" bash tools/gpu_ab_env.sh out.jsonl
# PIPE=K adds the two-frames-in-flight leg (K steps).  One JSON line per run into <out.jsonl>: {"label", "env", "round", "ms_per_step", "kernel_ms", "value", frac}.
# Each run has its own limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=${1:-gpurun_out/ab_env.jsonl}
mkdir -p "$(dirname "$out")"
IFS=';' read -ra VS <<< "$VARIANTS"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in "${VS[@]}"; do
    label=${v%%|*}; envs=${v#*|}; [ "$envs" = "$v" ] && envs=""
    log="gpurun_out/ab_${label}_r$r"
    env $envs timeout -k 10 "${LIM:-240}" python3 bench.py --no-cpu-baseline --no-e2e --pipelined-steps ${PIPE:-0} ${BENCH_ARGS:-} \
      > "$log.json" 2> "$log.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$label r$r failed rc=$rc" >&2; tail -5 "$log.err" >&2; exit $rc; fi
    python3 - "$log.json" "$label" "$envs" "$r" >> "$out" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rf = d["roofline"]
print(json.dumps({"label": sys.argv[2], "env": sys.argv[3], "round": int(sys.argv[4]), "value": d["value"],
                  "ms_per_step": d["ms_per_step"], "kernel_ms": d["kernel_ms"], "frac": rf["frac"],
                  "executed": rf.get("executed"), "traversal": d["config"].get("traversal"),
                  "pipelined": (d.get("pipelined") or {}).get("value"), "step_traffic": rf.get("step_traffic")}))
PY
    tail -1 "$out" | cut -c1-220 >&2
  done
done
