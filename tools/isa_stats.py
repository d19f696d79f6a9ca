#!/usr/bin/env python3
"""Offline register / scratch / instruction statistics of the run-time compiled render kernels.

    python3 tools/isa_stats.py <scene> [--trav static|accel|lane] [--bounces 16] [--out /tmp/isa]

Fetches the hipRTC source a render would build (rt_kernel_source), compiles it with hipcc for gfx950
with the same numerics flags, and prints, per kernel: VGPRs, SGPRs, spills and the private (scratch)
segment size — scratch traffic is HBM traffic the algorithm does not ask for.  No GPU needed.
"""
import argparse
import ctypes as C
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("scene", type=int)
    ap.add_argument("--trav", default="static", choices=("static", "accel", "lane", "mixed"))
    ap.add_argument("--bounces", type=int, default=16)
    ap.add_argument("--out", default="/tmp/isa")
    ap.add_argument("--flags", default="")
    a = ap.parse_args()
    import cuda_raytracing_amd as rt
    from cuda_raytracing_amd import _abi
    w, _ = rt.build_scene(a.scene)
    trav = {"static": rt.RT_TRAV_STATIC, "accel": rt.RT_TRAV_ACCEL, "lane": rt.RT_TRAV_LANE, "mixed": rt.RT_TRAV_MIXED}[a.trav]
    buf = C.create_string_buffer(1 << 24)
    rc = _abi.hip_lib().rt_kernel_source(C.byref(w.scene()), trav, a.bounces, buf, len(buf))
    if rc != 0:
        sys.exit(f"rt_kernel_source: {_abi.status_string(rc)}")
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    (out / "k.hip").write_text("#include <hip/hip_runtime.h>\n" + buf.value.decode())
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-slp-vectorize", *a.flags.split(),
           f"-I{REPO / 'cuda_raytracing_amd/csrc/device'}", "--cuda-device-only", "-c", "k.hip", "-o", "k.o",
           "-save-temps"]
    r = subprocess.run(cmd, cwd=out, capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr[-3000:])
    s = next(out.glob("k-hip-amdgcn-amd-amdhsa-gfx950.s")).read_text()
    # kernel metadata blocks (YAML in the .s): one per kernel
    for m in re.finditer(r"\n\s+- \.agpr_count:.*?\.name:\s+(\S+).*?(?=\n\s+- \.agpr_count:|\n\.end_amdgpu_metadata)", s, re.S):
        blk = m.group(0)
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
        print(f"{m.group(1):28s} vgpr {get('vgpr_count'):>4} sgpr {get('sgpr_count'):>4} "
              f"vgpr_spill {get('vgpr_spill_count'):>4} sgpr_spill {get('sgpr_spill_count'):>4} "
              f"scratch(private_segment_fixed_size) {get('private_segment_fixed_size'):>5} B/lane")
    def count(body, prefix):
        return len(re.findall(r"^\s+" + prefix, body, re.M))
    for name in re.findall(r"^(rt_\w+):\s*$", s, re.M):
        body = s.split(f"\n{name}:", 1)[1].split("s_endpgm", 1)[0]
        print(f"{name:28s} static instructions: valu {count(body, 'v_')} salu {count(body, 's_')} "
              f"scratch ops {count(body, 'scratch_')} global ops {count(body, 'global_')}")


if __name__ == "__main__":
    main()
