"""Throughput of K consecutive frames with 1 vs N frames in flight (separate contexts + streams)."""
import argparse, sys, time
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cuda_raytracing_amd as rt

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=0)
ap.add_argument("--spp", type=int, default=512)
ap.add_argument("--frames", type=int, default=6)
ap.add_argument("--inflight", default="1,2,3")
a = ap.parse_args()
w, s = rt.build_scene(a.scene)
cam, W, H = rt.camera_from_settings(s, 1920, 1080)
p = rt.make_params(s, W, H, spp=a.spp, bounces=16)
for nf in [int(x) for x in a.inflight.split(",")]:
    ctxs = [rt.RenderContext(w.scene(), 0) for _ in range(nf)]
    streams = [torch.cuda.Stream() for _ in range(nf)]
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(nf)]
    def run(frames):
        pending = []
        for k in range(frames):
            i = k % nf
            if len(pending) == nf:
                ctxs[pending.pop(0)].timing()
            ctxs[i].render_into(cam, p, outs[i].data_ptr(), streams[i].cuda_stream)
            pending.append(i)
        for i in pending:
            ctxs[i].timing()
    run(nf)                      # warm-up (JIT, buffers)
    torch.cuda.synchronize()
    t = time.perf_counter()
    run(a.frames)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"inflight {nf}: {dt / a.frames * 1e3:.2f} ms/frame  {W * H * a.spp * a.frames / dt / 1e6:.0f} Msamples/s", flush=True)
    for c in ctxs:
        c.close()
