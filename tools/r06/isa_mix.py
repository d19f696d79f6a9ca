#!/usr/bin/env python3
"""Offline instruction mix of the render kernel a scene builds (rt_kernel_build + RT_JIT_DUMP), for comparing
compile options without a GPU:  RT_JIT_SLP=1 python3 tools/r06/isa_mix.py 0 static 16
Prints the kernel's resource figures and static counts of VALU (packed f32 separately), SALU, moves, branches."""
import collections, os, re, subprocess, sys, tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
import torch  # noqa: F401  (the same library order as tests / bench)
import cuda_raytracing_amd as rt

scene, trav, mb = int(sys.argv[1]), sys.argv[2], int(sys.argv[3])
T = {"static": rt.RT_TRAV_STATIC, "accel": rt.RT_TRAV_ACCEL, "mixed": rt.RT_TRAV_MIXED, "lane": rt.RT_TRAV_LANE}[trav]
d = Path(tempfile.mkdtemp())
os.environ["RT_JIT_DUMP"] = str(d)
w, _ = rt.build_scene(scene)
k = rt.kernel_build(w.scene(), T, mb)
asm = "".join(subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", str(c)], capture_output=True,
                             text=True, check=True).stdout for c in d.glob("*.co"))
ops = [m.group(1) for m in re.finditer(r"^\s+(v_\w+|s_\w+|ds_\w+|global_\w+|buffer_\w+|scratch_\w+)", asm, re.M)]
c = collections.Counter(ops)
cat = collections.Counter()
for op, n in c.items():
    if op.startswith("v_pk_") and op.endswith("f32"): cat["valu_pk_f32"] += n
    elif op.startswith("v_mov") or op.startswith("v_cndmask"): cat["valu_mov_cnd"] += n
    elif op.startswith("v_readlane") or op.startswith("v_writelane"): cat["valu_lane"] += n
    elif op.startswith("v_"): cat["valu_other"] += n
    elif op.startswith("s_cbranch") or op.startswith("s_branch"): cat["branch"] += n
    elif op.startswith("s_"): cat["salu"] += n
    else: cat["mem"] += n
print({x: k[x] for x in ("vgprs", "sgprs", "scratch_bytes", "vgpr_spills", "sgpr_spills")}, dict(cat),
      "total", sum(c.values()))
print("top:", c.most_common(25))
