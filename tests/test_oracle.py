"""The CPU oracle: pinned against rocRAND's KAT, libm, analytic scenes and the golden fixtures (CPU only).

Parity status: the reference binary (CUDA + cuRAND) is unbuildable here, so the
oracle is "parity unpinned" against it; these tests pin everything that CAN be pinned.
"""
from __future__ import annotations

import ctypes as C
import json
import struct

import numpy as np
import pytest

import cuda_raytracing_amd as rt
from cuda_raytracing_amd import _abi
from conftest import GOLDEN, bits, blob_scene, camera_from_manifest, oracle_render, params_for


def test_rng_kat_matches_rocrand():
    kat = json.loads((GOLDEN / "rng_kat.json").read_text())
    L = _abi.oracle_lib()
    for case in kat["cases"]:
        out = np.zeros(8, np.float32)
        L.rt_oracle_uniforms(case["seed"], case["subsequence"], out.ctypes.data_as(C.c_void_p), 8)
        assert out.view(np.uint32).tolist() == case["uniform_bits"], case


def test_rng_kat_survey_values():
    # rocrand_init(1234, 1000000, 0) -> 0.863288283, 0.196769729
    out = np.zeros(2, np.float32)
    _abi.oracle_lib().rt_oracle_uniforms(1234, 1000000, out.ctypes.data_as(C.c_void_p), 2)
    assert np.allclose(out, [0.863288283, 0.196769729], atol=1e-9)


def test_sinf_substitute_is_faithful():
    L = _abi.oracle_lib()
    libm = C.CDLL("libm.so.6")
    libm.sinf.restype = C.c_float
    libm.sinf.argtypes = [C.c_float]
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(-50, 50, 20000), rng.uniform(-5000, 5000, 20000)]).astype(np.float32)
    ours = np.array([L.rt_oracle_sinf(float(x)) for x in xs], np.float32)
    ref = np.sin(xs.astype(np.float64))
    ulp = np.spacing(np.abs(ref).astype(np.float32))
    assert np.all(np.abs(ours.astype(np.float64) - ref) <= ulp)   # faithful (< 1 ulp of the true value)
    # it is the correctly rounded sine on every sample (glibc's sinf is faithful, ~98.7 % correctly rounded)
    cr = ref.astype(np.float32)
    assert np.array_equal(ours.view(np.uint32), cr.view(np.uint32))
    glibc = np.array([libm.sinf(float(x)) for x in xs], np.float32)
    assert (ours.view(np.uint32) == glibc.view(np.uint32)).mean() > 0.98


def test_pow5_substitute():
    L = _abi.oracle_lib()
    for x in np.linspace(0, 1, 257, dtype=np.float32):
        assert abs(L.rt_oracle_pow5f(float(x)) - float(x) ** 5) <= np.spacing(np.float32(float(x) ** 5))


def _render(world, W=16, H=12, spp=4, b=8, bg=(0.7, 0.8, 1.0), lookfrom=(0, 0, 0), lookat=(0, 0, -1), vfov=90.0):
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom, s.lookat, s.vfov = rt.vec3(*lookfrom), rt.vec3(*lookat), vfov
    s.background = rt.vec3(*bg)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    rc, fb, st = oracle_render(world.scene(), cam, p)
    assert rc == 0
    return fb, st


def test_analytic_empty_world_is_background():
    w = rt.World()
    w.sphere((0, 0, 100), 0.5, w.lambert((1, 1, 1)))     # behind the camera: never hit
    fb, st = _render(w)
    bg = np.array([0.7, 0.8, 1.0], np.float32)
    # every sample returns the background; sum of 4 copies * (1/4) is exact
    assert np.array_equal(fb, np.broadcast_to(bg * np.float32(4) * np.float32(0.25), fb.shape).astype(np.float32))
    assert st.counters[_abi.CNT_NAMES.index("bounces")] == 0


def test_analytic_light_wall():
    # a diffuse light quad filling the view: every camera ray ends on it; lights never scatter
    w = rt.World()
    w.quad((-50, -50, -1), (100, 0, 0), (0, 100, 0), w.light((2, 3, 4)))
    fb, _ = _render(w, bg=(0, 0, 0))
    assert np.array_equal(fb, np.full(fb.shape, [2, 3, 4], np.float32))


def test_analytic_mirror():
    # a fuzz-0 mirror facing the camera reflects straight back to the background behind the camera:
    # result = albedo * bg + 0 per sample
    w = rt.World()
    w.quad((-50, -50, -1), (100, 0, 0), (0, 100, 0), w.metal((0.5, 0.25, 1.0), 0.0))
    fb, st = _render(w, W=8, H=6, spp=2, b=4, bg=(0.5, 0.5, 0.5))
    want = np.float32([0.5, 0.25, 1.0]) * np.float32(0.5)
    assert np.array_equal(fb, np.broadcast_to(want * np.float32(2) * np.float32(0.5), fb.shape).astype(np.float32))


def test_zero_bounces_renders_black():
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 8, 4)
    p = rt.make_params(s, W, H, spp=3, bounces=0)
    rc, fb, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and not fb.any()
    p = rt.make_params(s, W, H, spp=3, bounces=256)      # rc_stack.max_count is u8: 256 -> 0
    rc, fb2, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and not fb2.any()


def test_oracle_rejects_bad_params():
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 8, 4)
    for kw in (dict(spp=0), dict(row_offset=4), dict(row_stride=0), dict(row_count=5)):
        p = rt.make_params(s, W, H, **{k: v for k, v in kw.items() if k == "spp"} or {})
        if "row_offset" in kw:
            p.row_offset = kw["row_offset"]
        if "row_stride" in kw:
            p.row_stride = kw["row_stride"]
        if "row_count" in kw:
            p.row_count = kw["row_count"]
        rc, _, _ = oracle_render(w.scene(), cam, p)
        assert rc == _abi.RT_ERR_INVALID_ARG, kw


def test_oracle_reproduces_golden(manifest, golden_frames, golden_scenes):
    for case in manifest["cases"]:
        idx = case["scene"]
        if f"s{idx}_hittables" in golden_scenes:
            sc = blob_scene(golden_scenes, idx).scene()
        else:
            w, _ = rt.build_scene(idx)
            sc = w.scene()
        rc, fb, st = oracle_render(sc, camera_from_manifest(case), params_for(case, manifest))
        assert rc == 0
        assert np.array_equal(bits(fb), bits(golden_frames[case["name"] + "_fb"])), case["name"]
        assert st.counter_dict()["samples"] == case["counters"]["samples"]


def test_oracle_shard_invariance():
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 40, 23)
    full = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=4, bounces=8))[1]
    for world in (2, 3, 8):
        shards = []
        for rank in range(world):
            off, stride, cnt = rt.shard_rows(H, rank, world)
            p = rt.make_params(s, W, H, spp=4, bounces=8, row_offset=off, row_stride=stride, row_count=cnt)
            shards.append(oracle_render(w.scene(), cam, p)[1])
        assert np.array_equal(bits(rt.unshard(shards, H, W)), bits(full)), world


def test_oracle_stack_within_reference_allocation():
    # the reference never overflows its hit stack on these scenes (8/12, 10/14)
    for idx, want in ((0, 8), (1, 10)):
        w, s = rt.build_scene(idx)
        cam, W, H = rt.camera_from_settings(s, 32, 32)
        _, _, st = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=2, bounces=8))
        assert st.counter_dict()["max_stack"] <= w.reference_stack_depth()
        assert st.counter_dict()["max_stack"] <= want


def test_atan2_acos_substitutes_are_correctly_rounded():
    # rt_atan2f / rt_acosf (sphere_get_uv, image textures only): correctly rounded on every sample,
    # and the exact IEEE special cases of atan2f/acosf
    import math
    L = _abi.oracle_lib()
    rng = np.random.default_rng(11)
    ys = np.concatenate([rng.uniform(-1, 1, 20000), rng.uniform(-1e3, 1e3, 5000)]).astype(np.float32)
    xs = np.concatenate([rng.uniform(-1, 1, 20000), rng.uniform(-1e-3, 1e-3, 5000)]).astype(np.float32)
    for y, x in zip(ys, xs):
        assert np.float32(L.rt_oracle_atan2f(float(y), float(x))) == np.float32(math.atan2(float(y), float(x)))
    for x in np.concatenate([rng.uniform(-1, 1, 20000), 1 - rng.uniform(0, 1e-4, 2000)]).astype(np.float32):
        assert np.float32(L.rt_oracle_acosf(float(x))) == np.float32(math.acos(float(x)))
    for y, x in [(0.0, 0.0), (-0.0, 0.0), (0.0, -0.0), (-0.0, -0.0), (1.0, -0.0), (1e-40, 1e-40), (3e38, 1.0),
                 (math.inf, math.inf), (-math.inf, 1.0), (1.0, -math.inf)]:
        got, want = np.float32(L.rt_oracle_atan2f(y, x)), np.float32(math.atan2(y, x))
        assert got == want and np.signbit(got) == np.signbit(want), (y, x)
    assert L.rt_oracle_acosf(1.0) == 0.0 and np.float32(L.rt_oracle_acosf(-1.0)) == np.float32(math.pi)
    assert math.isnan(L.rt_oracle_acosf(1.5))


def test_image_texture_scene_renders():
    from conftest import image_scene
    w = image_scene()
    fb, _ = _render(w, W=24, H=16, spp=4, b=6)
    assert np.isfinite(fb).all() and fb.max() > 0
    # not the magenta of a missing image: the texel gradient shows up
    assert len(np.unique(fb.reshape(-1, 3), axis=0)) > 50


@pytest.mark.parametrize("tile_w", ["8", "32", "64"])
@pytest.mark.parametrize("width,row_offset,row_stride,rows", [(1920, 0, 1, 3), (37, 3, 5, 17), (3840, 7, 8, 2), (1, 0, 1, 5),
                                                                 (13, 0, 1, 2)])
def test_rng_table_states_match_the_oracles_seeding(width, row_offset, row_stride, rows, tile_w, monkeypatch):
    # the render kernel's fused seeding, restated on the host (rt_rng_table_states: phase base of (row, column & (tw-1))
    # times the column table of J^(tw * (column >> log2 tw)), tw = the tile width, the tables the kernel reads): every
    # pixel's first draws equal the oracle's rocrand_init draws for subsequence (global row) * width + column
    import ctypes as C
    from cuda_raytracing_amd import _abi
    monkeypatch.setenv("RT_TILE_W", tile_w)
    st = np.zeros((rows * width, 6), np.uint32)
    assert _abi.hip_lib().rt_rng_table_states(1234, width, row_offset, row_stride, rows, st.ctypes.data_as(C.c_void_p)) == 0
    L = _abi.oracle_lib()
    cols = sorted(set(range(min(width, 11))) | {width - 1, width // 2, max(0, width - 9), min(width - 1, 33), min(width - 1, 70)})
    for k in range(rows):
        for j in cols:
            d, x0, x1, x2, x3, x4 = (int(v) for v in st[k * width + j])
            got = []
            for _ in range(4):
                t = (x0 ^ (x0 >> 2)) & 0xffffffff
                x0, x1, x2, x3 = x1, x2, x3, x4
                x4 = (x4 ^ (x4 << 4) ^ t ^ (t << 1)) & 0xffffffff
                d = (d + 362437) & 0xffffffff
                got.append(np.float32(np.float32((d + x4) & 0xffffffff) * np.float32(2.0 ** -32) + np.float32(2.0 ** -32)))
            ref = np.zeros(4, np.float32)
            L.rt_oracle_uniforms(1234, (row_offset + k * row_stride) * width + j, ref.ctypes.data_as(C.c_void_p), 4)
            assert np.array_equal(np.array(got, np.float32), ref), (k, j)
