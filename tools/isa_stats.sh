#!/bin/bash
# Offline ISA statistics of the scene-specialised kernel for a catalog scene (no GPU needed):
#   tools/isa_stats.sh <scene> [outdir]
# Writes the hipRTC source, compiles it with hipcc for gfx950 (same flags), prints VGPR/SGPR/spill
# counts and the static instruction mix of rt_static_render.
set -e
sc=${1:-0}; out=${2:-/tmp/isa}; mkdir -p "$out"
repo=$(cd "$(dirname "$0")/.." && pwd)
python3 - "$sc" "$out" <<PY
import sys; sys.path.insert(0, "$repo")
import cuda_raytracing_amd as rt
w, _ = rt.build_scene(int(sys.argv[1]))
src, v = rt.static_source(w.scene())
open(sys.argv[2] + "/k.hip", "w").write("#include <hip/hip_runtime.h>\n" + src)
PY
cd "$out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize $ISA_FLAGS -I"$repo/cuda_raytracing_amd/csrc/device" --cuda-device-only \
  -c k.hip -o k.o -save-temps 2>&1 | grep -E "error" || true
s=$(ls k-hip-amdgcn-amd-amdhsa-gfx950.s)
awk '/^rt_static_render:/,/s_endpgm/' "$s" > k0.s
grep -A30 "^    .name:           rt_static_render$" "$s" | grep -E "vgpr_count|sgpr_count|spill" || true
grep -B30 "^    .name:           rt_static_render$" "$s" | grep -E "vgpr_count|sgpr_count|spill" || true
echo "static: total $(grep -cE '^\s+[sv]_' k0.s)  valu $(grep -cE '^\s+v_' k0.s)  salu $(grep -cE '^\s+s_' k0.s)"
