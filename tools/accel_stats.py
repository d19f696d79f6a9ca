"""Verified sphere traversal diagnostics: fallback rate (rays re-traced with the reference walk).

    python3 tools/accel_stats.py --scene 20 --spp 64
"""
import argparse, sys
from pathlib import Path
import torch  # noqa: F401
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cuda_raytracing_amd as rt

ap = argparse.ArgumentParser()
ap.add_argument("--scene", type=int, default=20)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--bounces", type=int, default=16)
a = ap.parse_args()
w, s = rt.build_scene(a.scene)
cam, W, H = rt.camera_from_settings(s, a.width, a.height)
_, sc = rt.render(w.scene(), cam, rt.make_params(s, W, H, spp=a.spp, bounces=a.bounces, flags=rt.RT_FLAG_COUNT),
                  with_stats=True)
c = sc.counter_dict()
traces = c["samples"] + c["bounces"]
_, st = rt.render(w.scene(), cam, rt.make_params(s, W, H, spp=a.spp, bounces=a.bounces), with_stats=True)
print(f"scene {a.scene} {W}x{H} spp {a.spp}: traversal {st.traversal}, tree {st.accel_spheres} spheres depth "
      f"{st.accel_depth}; traces {traces}, fallbacks {st.accel_fallbacks} ({st.accel_fallbacks / max(traces, 1):.2e}); "
      f"render {st.render_ms:.2f} ms; reference visits/trace: bvh {c['visit_bvh'] / traces:.1f} sphere "
      f"{c['visit_sphere'] / traces:.1f}")
