"""Seeding-kernel time (rocrand_init per pixel) per RT_SEED_PER_THREAD value.

    python3 tools/seed_time.py 16 32 64 128
"""
import os, statistics, sys
from pathlib import Path
import numpy as np
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cuda_raytracing_amd as rt

w, s = rt.build_scene(0)
cam, W, H = rt.camera_from_settings(s, 1920, 1080)
p = rt.make_params(s, W, H, spp=1, bounces=16)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
ref = None
for v in sys.argv[1:] or ["64"]:
    os.environ["RT_SEED_PER_THREAD"] = v
    ctx = rt.RenderContext(w.scene(), 0)
    ts = []
    for r in range(6):
        ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        ts.append(ctx.timing().init_ms)
        img = out.cpu().numpy().view(np.uint32)
        if ref is None:
            ref = img.copy()
        assert np.array_equal(img, ref), "frame changed"
    print(f"per_thread {v}: seed median {statistics.median(ts[1:]):.3f} ms", flush=True)
