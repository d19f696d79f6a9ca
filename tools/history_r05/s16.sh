#!/bin/bash
# r05 s16: scene-20 mismatch bisect — the 6-wave kernel compiled without the tail-piece code, without the pool code, without
# both (RT_JIT_OPTS), against the oracle; the one-pixel printf build at the failing register budget
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/r05/dbg20.py "def|" "notail|RT_JIT_OPTS=-DRT_NO_TAIL_CODE" "nopool|RT_JIT_OPTS=-DRT_NO_POOL_CODE" \
  "neither|RT_JIT_OPTS=-DRT_NO_TAIL_CODE -DRT_NO_POOL_CODE" > gpurun_out/s16.log 2>&1; echo "rc=$?"
grep -v amdgpu.ids gpurun_out/s16.log
