"""The render kernels as launched (MI355X): registers, scratch and compiler of every BASELINE config's kernel
(rt_stats.kernel, ABI 6), and the device bounds checks (RT_CHECKS=1 builds, rt_body.h RT_CHECK).

Round 5 found a mis-render / GPU fault in a register-budget build of the verified sphere walk; round 6 traced it to a
LLVM 20 register-allocator defect and moved the run-time kernels to ROCm 7.2's hipRTC.  These tests pin the
outcome on the device: the kernels the five BASELINE configs launch have no scratch and no spilled VGPR and were built
by that compiler, and the checked builds render bit-exact frames and name an index that leaves its capacity."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import cuda_raytracing_amd as rt
from cuda_raytracing_amd import _abi
from conftest import bits, oracle_render

pytestmark = pytest.mark.gpu

# BASELINE configs 2-5: (scene, W, H, depth); a 2-row shard at spp 2 launches the same kernel as the full frame (the
# kernel variant follows the scene, the depth and the frame width, not the sample count or the row count)
CONFIGS = [(0, 1920, 1080, 16), (1, 1920, 1080, 50), (17, 1920, 1080, 50), (20, 1920, 1080, 16), (0, 3840, 2160, 50)]


def _ctx_render(scene, cam, p):
    ctx = rt.RenderContext(scene)
    try:
        out = torch.empty((p.row_count, p.width, 3), dtype=torch.float32, device="cuda")
        ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        try:
            st = ctx.timing()
        except rt.RenderError as e:
            return None, e, ctx.note()
        return out.cpu().numpy(), st, ctx.note()
    finally:
        ctx.close()


@pytest.mark.parametrize("idx,W,H,b", CONFIGS)
def test_baseline_config_kernels_launch_without_spills(idx, W, H, b):
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    off = H // 2
    p = rt.make_params(s, W, H, spp=2, bounces=b, row_offset=off, row_stride=1, row_count=2)
    fb, st, _ = _ctx_render(w.scene(), cam, p)
    k = st.kernel.as_dict()
    assert k["run_time"] == 1, k
    assert k["scratch_bytes"] == 0 and k["vgpr_spills"] == 0, k
    assert "clang version 22" in k["compiler"] and k["loader"].startswith("helper:"), k
    assert k["blocks_per_cu"] >= 1
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("idx,W,H,spp,b,flags", [
    (0, 64, 36, 4, 16, 0),                          # scene-specialised
    (0, 64, 36, 4, 16, rt.RT_FLAG_FORCE_LANE),      # per-lane DFS
    (1, 40, 40, 4, 50, 0),                          # Cornell, deep colour stack in LDS
    (17, 48, 27, 4, 50, 0),                         # Perlin, deep-level pool + HBM levels
    (20, 64, 36, 4, 16, 0),                         # verified sphere walk + candidate lists
    (2, 48, 27, 4, 16, 0),                          # verified sphere walk
    (3, 40, 40, 2, 40, 0),                          # verified mixed walk (final_scene)
])
def test_device_checks_pass_bit_exact(monkeypatch, idx, W, H, spp, b, flags):
    monkeypatch.setenv("RT_CHECKS", "1")
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b, flags=flags)
    fb, st, note = _ctx_render(w.scene(), cam, p)
    assert not isinstance(st, rt.RenderError), note
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


def test_device_check_names_a_stack_overflow(monkeypatch):
    # a per-lane stack three entries deep (test aid, RT_CHECKS builds only) for scene 0's walk, which needs 12
    monkeypatch.setenv("RT_CHECKS", "1")
    monkeypatch.setenv("RT_CHECK_STACK_CAP", "3")
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 32, 18)
    p = rt.make_params(s, W, H, spp=2, bounces=8, flags=rt.RT_FLAG_FORCE_LANE)
    fb, err, note = _ctx_render(w.scene(), cam, p)
    assert isinstance(err, rt.RenderError) and err.code == _abi.RT_ERR_DEVICE_CHECK, (err, note)
    assert "lane DFS stack" in note and "capacity 3" in note, note
