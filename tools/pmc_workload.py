"""Profiling workload: one render of a bench configuration through the C-ABI.

    --ppm   render through a context into torch device buffers with the fused PPM bytes (bench path)
    --probe-only / default: rt_render one-shot (float frame copied back)
"""
import argparse, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=0)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--bounces", type=int, default=16)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--ppm", action="store_true")
a = ap.parse_args()
if a.ppm:
    import torch  # noqa: F401  (one HIP runtime per process)
import cuda_raytracing_amd as rt
w, s = rt.build_scene(a.scene)
cam, W, H = rt.camera_from_settings(s, a.width, a.height)
p = rt.make_params(s, W, H, spp=a.spp, bounces=a.bounces)
if a.ppm:
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    out8 = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    for _ in range(a.reps):
        ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream, out8.data_ptr())
        st = ctx.timing()
    ctx.close()
else:
    for _ in range(a.reps):
        fb, st = rt.render(w.scene(), cam, p, with_stats=True)
print(f"render {st.render_ms:.3f} ms seed {st.init_ms:.3f} ms  {W*H*a.spp/st.render_ms/1e3:.1f} Msamples/s", flush=True)
