"""Scene-specialised traversal (scene_codegen.cpp + rt_jit.cpp) on the CPU: source generation and a
hipRTC cross-compile for gfx950.  No device is touched (hipRTC is only the compiler)."""
from __future__ import annotations

import pytest

import cuda_raytracing_amd as rt


@pytest.mark.parametrize("idx,visits", [(0, 21), (1, 31), (17, 3)])
def test_expansion_visits(idx, visits):
    # pre-order expansion of hit()'s DFS: one visit per node reached from the root (BVH subtrees,
    # group children, transform enter/exit counted once per node here)
    w, _ = rt.build_scene(idx)
    src, v = rt.static_source(w.scene())
    assert v == visits
    assert "struct StaticTrace" in src and "stk[" not in src
    assert src.count("box_hit(") == src.count("vc.k[1u]")   # every BVH visit is counted like the DFS


def test_expansion_budget():
    w, _ = rt.build_scene(rt.RT_SCENE_RANDOM_10K)
    with pytest.raises(rt.RenderError) as e:
        rt.static_source(w.scene(), max_visits=256)
    assert e.value.code == -6


@pytest.mark.parametrize("idx", [1, 17])
def test_hiprtc_compiles_for_gfx950(idx):
    # Cornell box: quads under rotate+translate; perlin_spheres: the noise texture variant
    w, _ = rt.build_scene(idx)
    rt.static_compile(w.scene(), "gfx950")


# ---- variant bits of the run-time kernels (rt_kernel_source: the host's decisions, no GPU) ----
def _variant_of(idx, trav, bounces, monkeypatch, **env):
    import ctypes as C
    import re
    from cuda_raytracing_amd import _abi
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w, _ = rt.build_scene(idx)
    buf = C.create_string_buffer(1 << 24)
    assert _abi.hip_lib().rt_kernel_source(C.byref(w.scene()), trav, bounces, buf, len(buf)) == 0
    m = re.search(r"render_body<(\d+), \w+", buf.value.decode())
    return int(m.group(1))


K_VAR_RC_LDS, K_VAR_RC_POOL, K_VAR_TAIL, K_VAR_TILED = 1 << 20, 1 << 25, 1 << 26, 1 << 27


def test_kernel_variants_deep_pool_and_lds_only(monkeypatch):
    # Perlin d50 (32-bit grey codes): HBM levels remain, so the deep-level pool's code is in; d16: not a deep kernel;
    # RT_RC_POOL=0: no pool.  Cornell d50 (8-bit codes): every level in LDS (kVarRcLds), no pool
    v = _variant_of(17, rt.RT_TRAV_STATIC, 50, monkeypatch)
    assert v & K_VAR_RC_POOL and not v & K_VAR_RC_LDS
    assert not _variant_of(17, rt.RT_TRAV_STATIC, 16, monkeypatch) & K_VAR_RC_POOL
    assert not _variant_of(17, rt.RT_TRAV_STATIC, 50, monkeypatch, RT_RC_POOL="0") & K_VAR_RC_POOL
    c = _variant_of(1, rt.RT_TRAV_STATIC, 50, monkeypatch)
    assert c & K_VAR_RC_LDS and not c & K_VAR_RC_POOL


def test_kernel_variants_opt_in_paths(monkeypatch):
    # tile-major output by default, noise textures included since round 6 (RT_TILED_OUT=0 and output staging decide
    # otherwise); no tail-piece code unless asked
    v = _variant_of(0, rt.RT_TRAV_STATIC, 16, monkeypatch)
    assert v & K_VAR_TILED and not v & K_VAR_TAIL
    assert _variant_of(17, rt.RT_TRAV_STATIC, 50, monkeypatch) & K_VAR_TILED
    assert not _variant_of(17, rt.RT_TRAV_STATIC, 50, monkeypatch, RT_TILED_OUT="0") & K_VAR_TILED
    assert _variant_of(17, rt.RT_TRAV_STATIC, 50, monkeypatch, RT_TILED_OUT="1") & K_VAR_TILED
    assert not _variant_of(0, rt.RT_TRAV_STATIC, 16, monkeypatch, RT_TILED_OUT="0") & K_VAR_TILED
    assert not _variant_of(0, rt.RT_TRAV_STATIC, 16, monkeypatch, RT_STAGE_SLOTS="4") & K_VAR_TILED
