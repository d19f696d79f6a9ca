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
