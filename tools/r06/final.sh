#!/bin/bash
# r06 final-tree records on one box: GPU suite, smoke, the default bench, rocprofv3 stats of the default bench command,
# every config through bench.py (+ final_scene), rocprofv3 stats of each config, and the two-rank gloo rehearsal of the
# N>1 path (ranks share the box's GPU; the gathered rows are checked against the oracle).  Each step under its own limit;
# the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06/${TAG:-final}
mkdir -p $O
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" "$O/$name.log" | head -5; tail -3 "$O/$name.log"; exit $rc; fi
}
[ -z "$SKIP_TESTS" ] && step pytest_gpu 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
[ -z "$SKIP_TESTS" ] && step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py
step rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_bench" -o run -- python3 bench.py --no-cpu-baseline --no-e2e
[ -n "$SKIP_CONFIGS" ] && exit 0
step configs 1500 env WITH_FINAL=1 bash tools/gpu_configs.sh
cp gpurun_out/configs.jsonl $O/configs.jsonl
step prof_configs 1800 bash tools/gpu_prof_configs.sh
mkdir -p $O/prof_cfg && cp -r gpurun_out/prof_cfg/*/ $O/prof_cfg/ 2>/dev/null
step gloo2_scene0 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e
step gloo2_10k 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --dist-backend gloo --frame fixed --scene 20 --spp 16 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e
grep -h '"gather_bit_exact"' $O/gloo2_*.log | python3 -c "import sys, json; [print(json.dumps(json.loads(l)['distributed'])) for l in sys.stdin]"
