"""Shared test setup.

Markers: `gpu` = needs an MI355X (runs the HIP library); everything else runs on CPU only and never
calls into the HIP library beyond dlopen/symbol checks.
"""
from __future__ import annotations

import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP render library)")


@pytest.fixture(scope="session")
def manifest():
    return json.loads((GOLDEN / "manifest.json").read_text())


@pytest.fixture(scope="session")
def golden_frames():
    return dict(np.load(GOLDEN / "frames.npz"))


@pytest.fixture(scope="session")
def golden_scenes():
    return dict(np.load(GOLDEN / "scenes.npz"))


def oracle_render(sc, cam, p):
    """CPU oracle (test infrastructure) -> (fb, stats)."""
    from cuda_raytracing_amd import _abi
    out = np.zeros((max(p.row_count, 0), p.width, 3), np.float32)
    st = _abi.Stats()
    rc = _abi.oracle_lib().rt_render_cpu(C.byref(sc), C.byref(cam), C.byref(p),
                                         out.ctypes.data_as(C.c_void_p), C.byref(st))
    return rc, out, st


def camera_from_manifest(case):
    from cuda_raytracing_amd import Camera, vec3
    cam = Camera()
    for f in ("pixel00", "delta_u", "delta_v", "center", "defocus_u", "defocus_v"):
        setattr(cam, f, vec3(*case["camera"][f]))
    cam.defocus_angle = case["camera"]["defocus_angle"]
    return cam


def blob_scene(golden_scenes, idx):
    from cuda_raytracing_amd import BlobScene
    k = f"s{idx}"
    return BlobScene(golden_scenes[f"{k}_hittables"].tobytes(), golden_scenes[f"{k}_refs"],
                     golden_scenes[f"{k}_textures"].tobytes(), int(golden_scenes[f"{k}_root"][0]))


def params_for(case, manifest):
    from cuda_raytracing_amd import Params, vec3
    s = manifest["scenes"][f"s{case['scene']}"]["settings"]
    p = Params()
    p.width, p.height = case["width"], case["height"]
    p.row_offset, p.row_stride, p.row_count = 0, 1, case["height"]
    p.samples_per_pixel, p.max_bounces = case["spp"], case["bounces"]
    p.background = vec3(*s["background"])
    p.seed = 1234
    p.flags = 0
    return p


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def image_scene():
    """Spheres and quads with a synthetic image texture (the reference's earthmap.jpg is absent):
    exercises sphere_get_uv (rt_acosf / rt_atan2f), planar u,v and image_texture_get_pixel's clamp."""
    import cuda_raytracing_amd as rt
    w = rt.World(capacity=64)
    yy, xx = np.mgrid[0:19, 0:37].astype(np.float32)
    tex = np.stack([xx / 36.0, yy / 18.0, 0.25 + 0.5 * ((xx + yy) % 3 == 0)], axis=-1).astype(np.float32)
    img = w.image_pixels(tex)
    w.sphere((0, 0, -2), 0.8, img)
    w.sphere((1.2, 0.3, -2.5), 0.5, img)
    w.quad((-3, -1, -4), (6, 0, 0), (0, 0, 3.5), img)
    w.sphere((-1.3, 0.2, -1.8), 0.4, w.metal((0.8, 0.8, 0.8), 0.1))
    return w
