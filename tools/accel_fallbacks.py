"""Verified-walk fallback rate: rays handed back to the reference walk per traced ray (diagnostics).

    python3 tools/accel_fallbacks.py [scene spp bounces ...]
Traced rays = samples + scattering bounces (one ray per camera sample and per scattered hit, counting run).
"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: F401
import cuda_raytracing_amd as rt

args = [int(x) for x in sys.argv[1:]] or [20, 16, 16, 2, 16, 16]
for idx, spp, b in zip(args[0::3], args[1::3], args[2::3]):
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 1920, 1080)
    _, st = rt.render(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b), with_stats=True)
    _, sc = rt.render(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_COUNT), with_stats=True)
    c = sc.counter_dict()
    rays = c["samples"] + c["bounces"]
    print(f"scene {idx}: {st.accel_fallbacks} fallbacks / {rays} rays = {st.accel_fallbacks / rays:.5f}; render {st.render_ms:.2f} ms; "
          f"tree {st.accel_spheres} spheres depth {st.accel_depth}", flush=True)
