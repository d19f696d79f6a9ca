"""A/B render-context options (env knobs read at context creation) in ONE process, interleaved rounds (guide §5.4 rule 24).

Times are render + schedule (probe and tile sort) kernel time.  Every configuration must produce a bit-identical frame (the schedule never changes what a lane
computes); the script asserts that and prints median render ms per configuration.
    python3 tools/tune.py --scene 0 --spp 64 --configs RT_TRAVERSAL=0,RT_TRAVERSAL=1 --rounds 3
"""
import argparse, json, os, statistics, sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np
import cuda_raytracing_amd as rt

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=0)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--bounces", type=int, default=16)
ap.add_argument("--configs", default="RT_TRAVERSAL=0,RT_TRAVERSAL=1",
                help="comma-separated env assignments (';' joins several), one render context each")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--out", default="")
a = ap.parse_args()

w, s = rt.build_scene(a.scene)
cam, W, H = rt.camera_from_settings(s, a.width, a.height)
p = rt.make_params(s, W, H, spp=a.spp, bounces=a.bounces)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
ctxs = {}
for c in a.configs.split(","):
    saved = dict(os.environ)
    for kv in c.split(";"):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    ctxs[c] = rt.RenderContext(w.scene(), 0)
    os.environ.clear(); os.environ.update(saved)
times = {c: [] for c in ctxs}
ref = None
for r in range(a.rounds + 1):
    for c, ctx in ctxs.items():
        ctx.render_into(cam, p, out.data_ptr(), stream)
        t = ctx.timing()
        img = out.cpu().numpy().view(np.uint32)
        if ref is None:
            ref = img.copy()
        assert np.array_equal(img, ref), f"config {c} changed the frame"
        if r > 0:
            times[c].append(t.render_ms + t.sched_ms)
res = {c: {"median_ms": statistics.median(v), "min_ms": min(v),
           "msamples_s": W * H * a.spp / statistics.median(v) / 1e3} for c, v in times.items()}
for c, v in sorted(res.items(), key=lambda kv: kv[1]["median_ms"]):
    print(f"{c:24s} median {v['median_ms']:8.3f} ms  min {v['min_ms']:8.3f}  {v['msamples_s']:8.1f} Msamples/s", flush=True)
if a.out:
    Path(a.out).write_text(json.dumps({"args": vars(a), "results": res}, indent=1))
