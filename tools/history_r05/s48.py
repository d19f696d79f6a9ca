#!/usr/bin/env python3
"""r05 s48: a 1080p render (scene, spp, bounces), tile-major vs row-major output, with RT_DEBUG launch/occupancy lines (stderr)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import cuda_raytracing_amd as rt  # noqa: E402

scene, spp = int(sys.argv[1]), int(sys.argv[2])
bounces = int(sys.argv[3]) if len(sys.argv) > 3 else 50
w, s = rt.build_scene(scene)
cam, W, H = rt.camera_from_settings(s, 1920, 1080)
p = rt.make_params(s, W, H, spp=spp, bounces=bounces)
for tiled in ("0", "1", "0", "1"):
    os.environ["RT_TILED_OUT"] = tiled
    t = time.time()
    fb, st = rt.render(w.scene(), cam, p, with_stats=True)
    print(f"tiled {tiled} render_kernel_ms {st.render_kernel_ms:.2f} tiled_out {st.tiled_out} pool {st.rc_pool_chunks} "
          f"levels {st.rc_lds_levels} lds {st.scene_in_lds} jit_ms {st.jit_ms:.0f} wall {time.time() - t:.2f}", flush=True)
