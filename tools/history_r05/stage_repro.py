#!/usr/bin/env python3
"""r05: reproduce the staged-write mismatch of test_fused_ppm_bytes_match_host_tonemap[0-96-54-8-16] (RT_STAGE_SLOTS=4):
which pixels of the float frame and of the PPM bytes differ from the oracle, per 8x8 tile."""
import os, sys
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO)); sys.path.insert(0, str(REPO / "tests"))
import torch
import cuda_raytracing_amd as rt
from conftest import oracle_render, bits
CASES = [(0, 96, 54, 8, 16), (0, 96, 54, 16, 16), (0, 96, 56, 8, 16), (1, 40, 40, 4, 50), (1, 96, 54, 8, 16), (0, 96, 53, 8, 16),
         (0, 96, 54, 8, 4), (0, 64, 54, 8, 16)]
for (idx, W, H, spp, b) in CASES:
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.full((H, W, 3), float("nan"), dtype=torch.float32, device="cuda")
    out8 = torch.full((H, W, 3), 7, dtype=torch.uint8, device="cuda")
    ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream, out8.data_ptr())
    st = ctx.timing()
    torch.cuda.synchronize()
    fb = out.cpu().numpy()
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    badf = (bits(fb) != bits(ref)).any(-1)
    bad8 = (out8.cpu().numpy() != rt.tonemap(ref)).any(-1)
    tiles = sorted({(int(r) // 8, int(c) // 8) for r, c in np.argwhere(badf | bad8)})
    o8 = out8.cpu().numpy()
    unwritten = int((o8[bad8] == 7).all(-1).sum()) if bad8.any() else 0
    print(f"scene {idx} {W}x{H} spp {spp} d{b}: float bad {int(badf.sum())}, bytes bad {int(bad8.sum())} (still the fill: {unwritten}), "
          f"nan {int(np.isnan(fb).any(-1).sum())}, tiles {tiles[:14]}", flush=True)
    if bad8.any():
        r, c = np.argwhere(bad8)[0]
        print("   first bad", (int(r), int(c)), "got", o8[r, c].tolist(), "want", rt.tonemap(ref)[r, c].tolist(), flush=True)
    ctx.close()
