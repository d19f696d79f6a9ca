#!/usr/bin/env python3
"""Scene-20 (10k spheres) parity probe: one small frame per environment variant against the oracle, per channel.

    python3 tools/r05/dbg20.py [--scene 20] [--size 64x36] [--spp 16] [--bounces 16] "LABEL|ENV=V ENV2=V" ...

Prints, per variant: the traversal, the differing pixels per channel and the first differing pixels.
"""
import argparse
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=20)
ap.add_argument("--size", default="64x36")
ap.add_argument("--spp", type=int, default=16)
ap.add_argument("--bounces", type=int, default=16)
ap.add_argument("--save", default="")
ap.add_argument("variants", nargs="*", default=["def|"])
a = ap.parse_args()

import cuda_raytracing_amd as rt  # noqa: E402
from conftest import oracle_render  # noqa: E402

W, H = (int(x) for x in a.size.split("x"))
w, s = rt.build_scene(a.scene)
cam, W, H = rt.camera_from_settings(s, W, H)
p = rt.make_params(s, W, H, spp=a.spp, bounces=a.bounces)
rc, ref, _ = oracle_render(w.scene(), cam, p)
assert rc == 0
rb = ref.view(np.uint32)
for v in a.variants:
    label, _, envs = v.partition("|")
    saved = dict(os.environ)
    for kv in envs.split():
        k, _, val = kv.partition("=")
        os.environ[k] = val.replace("+", " ")   # '+' stands for a space inside a value
    try:
        fb, st = rt.render(w.scene(), cam, p, with_stats=True)
    finally:
        os.environ.clear()
        os.environ.update(saved)
    if a.save:
        np.save(f"{a.save}_{label}.npy", fb)
        np.save(f"{a.save}_ref.npy", ref)
    gb = fb.view(np.uint32)
    diff = gb != rb
    per_ch = diff.reshape(-1, 3).sum(axis=0).tolist()
    px = np.argwhere(diff.any(axis=2))
    print(f"{label:10s} trav {st.traversal} levels {st.rc_lds_levels} differing px {len(px)} per channel {per_ch} "
          f"first {px[:4].tolist()}", flush=True)
