"""HIP render path vs the CPU oracle and the golden fixtures — bit-exact (MI355X only).

Tolerance: none.  Every case compares the float32 framebuffer bit patterns.  All GPU work goes through
the C-ABI (librt_hip.so); the oracle is only the checker.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

import torch  # noqa: F401  one HIP runtime per process (see cuda_raytracing_amd._abi)

import cuda_raytracing_amd as rt
from cuda_raytracing_amd import _abi
from conftest import bits, blob_scene, camera_from_manifest, oracle_render, params_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    n = C.c_int()
    _abi.hip_lib().rt_device_count(C.byref(n))
    assert n.value > 0, "no HIP device: the GPU tests must run on an MI355X (no CPU fallback exists)"


def gpu(sc, cam, p):
    return rt.render(sc, cam, p, with_stats=True)


def test_golden_frames(manifest, golden_frames, golden_scenes):
    for case in manifest["cases"]:
        idx = case["scene"]
        if f"s{idx}_hittables" in golden_scenes:
            sc = blob_scene(golden_scenes, idx).scene()
        else:
            w, _ = rt.build_scene(idx)
            sc = w.scene()
        fb, st = gpu(sc, camera_from_manifest(case), params_for(case, manifest))
        assert np.array_equal(bits(fb), bits(golden_frames[case["name"] + "_fb"])), case["name"]
        assert np.array_equal(rt.tonemap(fb), golden_frames[case["name"] + "_u8"])


@pytest.mark.parametrize("idx", list(range(rt.RT_SCENE_COUNT)))
def test_every_catalog_scene_vs_oracle(idx):
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 24, 16)
    p = rt.make_params(s, W, H, spp=3, bounces=min(s.max_bounces, 50))
    fb, _ = gpu(w.scene(), cam, p)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("idx,W,H,spp,b", [(0, 96, 54, 8, 16), (1, 40, 40, 8, 50), (17, 64, 36, 4, 50),
                                          (2, 48, 27, 4, 16), (20, 48, 27, 2, 16)])
def test_counters_equal_oracle(idx, W, H, spp, b):
    # same traversal, same shading events: the per-kind visit counts must match exactly
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_COUNT)
    fb, st = gpu(w.scene(), cam, p)
    rc, ref, ost = oracle_render(w.scene(), cam, p)
    assert np.array_equal(bits(fb), bits(ref))
    g, o = st.counter_dict(), ost.counter_dict()
    for k in ("visit_sphere", "visit_bvh", "visit_triangle", "visit_quad", "visit_translate", "visit_yrotate",
              "visit_group", "bounces", "shades", "perlin", "samples"):
        assert g[k] == o[k], (k, g[k], o[k])
    assert g["max_stack"] <= st.stack_needed and g["stack_overflow"] == 0
    assert o["max_stack"] <= st.stack_needed


@pytest.mark.parametrize("idx", [0, 1, 17])
def test_lds_and_global_scene_agree(idx):
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 48, 32)
    p = rt.make_params(s, W, H, spp=4, bounces=16)
    a, sa = gpu(w.scene(), cam, p)
    p.flags = rt.RT_FLAG_GLOBAL_SCENE
    b, sb = gpu(w.scene(), cam, p)
    assert sa.scene_in_lds == 1 and sb.scene_in_lds == 0
    assert np.array_equal(bits(a), bits(b))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_row_shards_reassemble(world):
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 70, 41)
    full, _ = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=4, bounces=8))
    shards = []
    for r in range(world):
        off, stride, cnt = rt.shard_rows(H, r, world)
        shards.append(gpu(w.scene(), cam, rt.make_params(s, W, H, spp=4, bounces=8, row_offset=off,
                                                         row_stride=stride, row_count=cnt))[0])
    assert np.array_equal(bits(rt.unshard(shards, H, W)), bits(full))


def test_edge_sizes_and_params():
    w, s = rt.build_scene(0)
    sc = w.scene()
    for W, H, spp, b in [(1, 1, 1, 1), (1, 7, 3, 4), (65, 1, 2, 4), (63, 2, 5, 40), (129, 3, 1, 255)]:
        cam, W2, H2 = rt.camera_from_settings(s, W, H)
        p = rt.make_params(s, W2, H2, spp=spp, bounces=b)
        fb, _ = gpu(sc, cam, p)
        rc, ref, _ = oracle_render(sc, cam, p)
        assert rc == 0 and np.array_equal(bits(fb), bits(ref)), (W, H, spp, b)
    cam, W, H = rt.camera_from_settings(s, 16, 9)
    for b in (0, 256):       # u8 max_count: no tracing at all -> exact zeros
        fb, _ = gpu(sc, cam, rt.make_params(s, W, H, spp=2, bounces=b))
        assert not fb.any() and not np.signbit(fb).any()
    empty, _ = gpu(sc, cam, rt.make_params(s, W, H, spp=2, bounces=4, row_count=0))
    assert empty.shape == (0, W, 3)
    for bad in (dict(spp=0), dict(row_offset=9), dict(row_stride=0)):
        p = rt.make_params(s, W, H, spp=bad.get("spp", 2), bounces=4)
        if "row_offset" in bad:
            p.row_offset = bad["row_offset"]
        if "row_stride" in bad:
            p.row_stride = bad["row_stride"]
        with pytest.raises(rt.RenderError) as e:
            gpu(sc, cam, p)
        assert e.value.code == _abi.RT_ERR_INVALID_ARG


def test_malformed_scenes_are_rejected():
    w, s = rt.build_scene(0)
    b = w.blobs()
    cam, W, H = rt.camera_from_settings(s, 8, 8)
    p = rt.make_params(s, W, H, spp=1, bounces=4)

    def attempt(rec, refs, tex, root):
        with pytest.raises(rt.RenderError) as e:
            rt.render(rt.BlobScene(rec, refs, tex, root).scene(), cam, p)
        assert e.value.code == _abi.RT_ERR_SCENE

    rec = bytearray(b["hittables"])
    rec[0:4] = (9).to_bytes(4, "little")                       # unknown record kind
    attempt(bytes(rec), b["refs"], b["textures"], b["root"])
    refs = b["refs"].copy()
    refs[0] = 60000                                            # WorldRef to a missing record
    attempt(b["hittables"], refs, b["textures"], b["root"])
    attempt(b["hittables"], b["refs"], b["textures"][:40], b["root"])   # texture offsets past the arena
    attempt(b["hittables"], b["refs"], b["textures"], 99)      # root beyond the ref list


def test_full_size_rows_match_oracle():
    # BASELINE config 2 geometry (1920x1080, d16) at reduced spp: three full-width rows from the GPU
    # frame must equal the oracle's rendering of the same rows (shard-invariant RNG)
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 1920, 1080)
    full, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=4, bounces=16))
    again, _ = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=4, bounces=16))
    assert np.array_equal(bits(full), bits(again))                    # deterministic
    p = rt.make_params(s, W, H, spp=4, bounces=16, row_offset=1, row_stride=539, row_count=3)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(full[1::539][:3]), bits(ref))
    assert np.isfinite(full).all() and (full >= 0).all()


def test_context_reuse_and_torch_buffers():
    w, s = rt.build_scene(17)
    cam, W, H = rt.camera_from_settings(s, 40, 30)
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    for spp in (2, 5, 2):
        p = rt.make_params(s, W, H, spp=spp, bounces=20)
        ctx.render_into(cam, p, out.data_ptr(), stream.cuda_stream)
        st = ctx.timing()
        assert st.render_ms > 0 and st.samples == W * H * spp
        ref, _ = gpu(w.scene(), cam, p)
        assert np.array_equal(bits(out.cpu().numpy()), bits(ref))
    ctx.close()


TRAVERSALS = [(rt.RT_FLAG_FORCE_LANE, rt.RT_TRAV_LANE), (rt.RT_FLAG_FORCE_PACKET, rt.RT_TRAV_PACKET),
              (rt.RT_FLAG_FORCE_STATIC, rt.RT_TRAV_STATIC)]


@pytest.mark.parametrize("idx", [0, 1, 8, 13, 15, 16, 17, 18, 19])
def test_every_traversal_matches_oracle(idx):
    # the three traversal policies (per-lane DFS, wave packet, hipRTC straight-line) must all reproduce
    # the oracle bit for bit, with identical per-kind visit counts
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 40, 24)
    p = rt.make_params(s, W, H, spp=3, bounces=min(s.max_bounces, 50), flags=rt.RT_FLAG_COUNT)
    rc, ref, ost = oracle_render(w.scene(), cam, p)
    assert rc == 0
    for force, want in TRAVERSALS:
        p.flags = rt.RT_FLAG_COUNT | force
        fb, st = gpu(w.scene(), cam, p)
        assert st.traversal == want, (force, st.traversal)
        assert np.array_equal(bits(fb), bits(ref)), (idx, want)
        g, o = st.counter_dict(), ost.counter_dict()
        for k in ("visit_sphere", "visit_bvh", "visit_triangle", "visit_quad", "visit_translate",
                  "visit_yrotate", "visit_group", "bounces", "shades", "perlin", "samples"):
            assert g[k] == o[k], (idx, want, k, g[k], o[k])


def test_auto_policy_and_fallback():
    # small scenes go through the specialised kernel, the 10k-sphere scene exceeds the visit budget
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 16, 9)
    _, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=1, bounces=4))
    assert st.traversal == rt.RT_TRAV_STATIC and st.jit_visits > 0
    _, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=1, bounces=4, flags=rt.RT_FLAG_NO_JIT))
    assert st.traversal != rt.RT_TRAV_STATIC
    w, s = rt.build_scene(rt.RT_SCENE_RANDOM_10K)
    cam, W, H = rt.camera_from_settings(s, 16, 9)
    fb, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=1, bounces=4, flags=rt.RT_FLAG_FORCE_STATIC))
    assert st.traversal == rt.RT_TRAV_ACCEL and st.accel_spheres > 10000
    rc, ref, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=1, bounces=4))
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("sched", ["0", "1", "2", "3"])
def test_tile_schedules_agree(sched, monkeypatch):
    # the schedule (longest-first probe order, row-major, reversed) only changes which lane renders a
    # pixel when; frames must stay bit-identical to the oracle (spp >= 16 enables the probe in auto)
    monkeypatch.setenv("RT_SCHED", sched)
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 37, 21)
    p = rt.make_params(s, W, H, spp=16, bounces=8)
    fb, _ = gpu(w.scene(), cam, p)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("idx,W,H,spp", [(0, 96, 54, 24), (20, 64, 36, 16), (3, 48, 48, 16), (17, 64, 36, 16)])
@pytest.mark.parametrize("tail", ["0", "1"])
def test_tail_issue_priority_agrees(idx, W, H, spp, tail, monkeypatch):
    # RT_TAIL_PRIO only reorders the SIMD's issue once the queue is drained: frames stay oracle-exact on every
    # traversal it can run under (static, verified sphere walk, verified mixed walk, noise scenes)
    monkeypatch.setenv("RT_TAIL_PRIO", tail)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=16)
    fb, _ = gpu(w.scene(), cam, p)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("idx,W,H,spp", [(0, 96, 54, 24), (20, 64, 36, 16), (3, 48, 48, 16), (17, 64, 36, 16)])
@pytest.mark.parametrize("chunk,gen", [("1", "1"), ("8", "0.5"), ("32", "4")])
def test_tail_pieces_agree(idx, W, H, spp, chunk, gen, monkeypatch):
    # RT_TAIL_CHUNK hands the last ids of the longest-first order out in pieces of 1..32 pixels from their own
    # counter (seeded per piece at pickup): which lane renders a pixel changes, the frame must not — with whole tiles
    # before (scene 0, 10k), split costliest tiles and sparse hot waves (Perlin), mixed hot waves (final_scene); at
    # these sizes the tail covers part of the frame (gen 0.5) or all of it (gen 4)
    monkeypatch.setenv("RT_TAIL_CHUNK", chunk)
    monkeypatch.setenv("RT_TAIL_GEN", gen)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=16)
    fb, _ = gpu(w.scene(), cam, p)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("idx", [0, 1, 2, 8, 13, 18, 19])
def test_folded_and_unfolded_static_traversal(idx):
    # exact constant folding of primitive tests (scene_codegen.cpp) must not change a single bit
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 48, 27)
    p = rt.make_params(s, W, H, spp=4, bounces=min(s.max_bounces, 50), flags=rt.RT_FLAG_FORCE_STATIC)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    a, sa = gpu(w.scene(), cam, p)
    p.flags = rt.RT_FLAG_FORCE_STATIC | rt.RT_FLAG_NO_FOLD
    b, sb = gpu(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(a), bits(ref)) and np.array_equal(bits(b), bits(ref))
    if sa.traversal == rt.RT_TRAV_STATIC:
        assert sa.folded == 1 and sb.folded == 0 and sa.fold_rerenders == 0


@pytest.mark.parametrize("tries", ["1", "2", "3", "0/4", "0/63", "3/2"])
@pytest.mark.parametrize("idx", [0, 1, 8])
def test_capped_rejection_tries_agree(idx, tries, monkeypatch):
    # deferring an unfinished rejection loop to the next round (after RT_MAX_TRIES tries, or once at
    # most RT_DEFER_LANES lanes still reject) must not change any draw or result
    cap, _, defer = tries.partition("/")
    monkeypatch.setenv("RT_MAX_TRIES", cap)
    monkeypatch.setenv("RT_DEFER_LANES", defer or "0")
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 33, 19)
    for force in (rt.RT_FLAG_FORCE_STATIC, rt.RT_FLAG_FORCE_LANE, rt.RT_FLAG_FORCE_PACKET):
        p = rt.make_params(s, W, H, spp=5, bounces=min(s.max_bounces, 50), flags=force | rt.RT_FLAG_COUNT)
        fb, st = gpu(w.scene(), cam, p)
        rc, ref, ost = oracle_render(w.scene(), cam, p)
        assert rc == 0 and np.array_equal(bits(fb), bits(ref)), (idx, tries, force)
        assert st.counter_dict()["shades"] == ost.counter_dict()["shades"]


@pytest.mark.parametrize("idx", [1, 2, 13, 17, 20])
def test_offline_and_jit_lane_kernels_agree(idx):
    # the offline all-kinds lane kernel (RT_FLAG_NO_JIT) and the kind-specialised hipRTC one
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 36, 20)
    p = rt.make_params(s, W, H, spp=3, bounces=min(s.max_bounces, 50), flags=rt.RT_FLAG_FORCE_LANE | rt.RT_FLAG_COUNT)
    a, sa = gpu(w.scene(), cam, p)
    p.flags = rt.RT_FLAG_FORCE_LANE | rt.RT_FLAG_NO_JIT | rt.RT_FLAG_COUNT
    b, sb = gpu(w.scene(), cam, p)
    rc, ref, ost = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(a), bits(ref)) and np.array_equal(bits(b), bits(ref))
    assert sa.counter_dict()["visit_bvh"] == sb.counter_dict()["visit_bvh"] == ost.counter_dict()["visit_bvh"]


def test_device_tonemap_matches_host():
    # pixels_to_ppm bytes on the GPU == the host conversion, including specials and clamp edges
    import torch
    rng = np.random.default_rng(7)
    vals = rng.uniform(-0.5, 1.6, size=(301, 7, 3)).astype(np.float32)
    flat = vals.reshape(-1)
    specials = np.array([0.0, -0.0, 1.0, 0.998001, 0.998002, 0.999, 1e-30, 1e-45, np.inf, -np.inf, np.nan,
                         0.25, 0.5, 255.0 / 256.0, (255.0 / 256.0) ** 2], np.float32)
    flat[:len(specials)] = specials
    host = rt.tonemap(vals)
    dev = rt.tonemap_device(torch.from_numpy(vals).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)
    # a rendered frame, odd pixel count (tail path of the 4-wide kernel)
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 37, 11)
    fb = rt.render(w.scene(), cam, rt.make_params(s, W, H, spp=4, bounces=8))
    dev = rt.tonemap_device(torch.from_numpy(fb).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), rt.tonemap(fb))


def test_image_texture_scene_vs_oracle():
    # image textures with texels (UV variant: rt_acosf / rt_atan2f, planar u,v, texel clamp) — every
    # traversal policy against the oracle
    from conftest import image_scene
    w = image_scene()
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom, s.lookat, s.vfov = rt.vec3(0, 0, 0), rt.vec3(0, 0, -1), 90.0
    cam, W, H = rt.camera_from_settings(s, 40, 24)
    p = rt.make_params(s, W, H, spp=4, bounces=6)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and len(np.unique(ref.reshape(-1, 3), axis=0)) > 50
    for force, _want in TRAVERSALS:
        p.flags = force
        fb, _ = gpu(w.scene(), cam, p)
        assert np.array_equal(bits(fb), bits(ref)), force


def test_earth_scene_with_a_texture_file_vs_oracle(tmp_path, monkeypatch):
    # the catalog's earth scene (raytracing.cu:2042-2052) with an earthmap.jpg present (the reference
    # repository does not ship one): a progressive 4:2:0 JPEG written here, decoded like stbi_loadf
    # (tests/test_image_load.py pins that against stb itself), rendered on the GPU and by the oracle from
    # the same arena bytes
    import image_corpus
    pic = image_corpus.picture(64, 128, seed=3)
    (tmp_path / "earthmap.jpg").write_bytes(image_corpus.pil_bytes(pic, "JPEG", quality=85, progressive=True,
                                                                   subsampling=2))
    monkeypatch.chdir(tmp_path)
    idx = [rt.scene_name(i) for i in range(rt.RT_SCENE_COUNT)].index("earth")
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 128, 72)
    p = rt.make_params(s, W, H, spp=2, bounces=6)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    px = ref.reshape(-1, 3)
    assert rc == 0 and len(np.unique(px, axis=0)) > 100   # textured
    assert not np.any((px[:, 0] > 0) & (px[:, 1] == 0) & (px[:, 2] > 0))   # no magenta (failed-load) texel
    fb, st = gpu(w.scene(), cam, p)
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("idx,W,H,spp", [(2, 64, 36, 4), (20, 64, 36, 4), (20, 160, 90, 6), (2, 128, 72, 8)])
def test_verified_sphere_traversal_matches_oracle(idx, W, H, spp):
    # SAH tree walk + per-ray proof against the reference tree (fallback to the reference walk)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=16, flags=rt.RT_FLAG_FORCE_ACCEL)
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_ACCEL and st.accel_spheres > 0
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


def _rows_match_oracle(w, s, cam, W, H, spp, b, full, stride):
    """Rows 0, stride, 2*stride, ... of a GPU frame against the oracle's render of exactly those rows (the RNG
    subsequence is the global pixel index, so a row subset is comparable)."""
    n = (H - 1) // stride + 1
    p = rt.make_params(s, W, H, spp=spp, bounces=b, row_offset=0, row_stride=stride, row_count=n)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    got = full[0::stride]
    assert got.shape == ref.shape
    bad = np.argwhere(bits(got) != bits(ref))
    assert bad.size == 0, f"{len(bad)} values differ vs the oracle, first at row {bad[0][0] * stride} col {bad[0][1]}"


@pytest.mark.parametrize("idx,W,H,spp,b", [(20, 480, 270, 16, 16), (2, 480, 270, 16, 50)])
def test_verified_sphere_traversal_matches_reference_walk_large(idx, W, H, spp, b):
    # millions of rays: the verified walk against the reference walk on the GPU (itself oracle-exact), and
    # every 7th row of the verified walk's frame against the oracle itself
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    a, sa = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_FORCE_ACCEL))
    c, sc = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_FORCE_LANE))
    assert sa.traversal == rt.RT_TRAV_ACCEL and sc.traversal == rt.RT_TRAV_LANE
    assert np.array_equal(bits(a), bits(c))
    _rows_match_oracle(w, s, cam, W, H, spp, b, a, 7)


@pytest.mark.parametrize("idx,W,H,spp,b", [(0, 480, 270, 16, 16), (1, 320, 320, 8, 50), (17, 480, 270, 8, 50),
                                          (16, 400, 400, 8, 50)])
def test_static_fast_paths_match_reference_walk_large(idx, W, H, spp, b):
    # millions of rays: the folded straight-line kernel (exact folding, division without
    # div_scale/div_fixup, shared reciprocals, deferred rejection, deep-path unwind) against the
    # plain per-lane reference walk, which is itself bit-exact against the oracle at small sizes
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    a, sa = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_FORCE_STATIC))
    c, sc = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_FORCE_LANE | rt.RT_FLAG_NO_JIT))
    assert sa.traversal == rt.RT_TRAV_STATIC and sa.folded == 1 and sc.traversal == rt.RT_TRAV_LANE
    assert np.array_equal(bits(a), bits(c))
    _rows_match_oracle(w, s, cam, W, H, spp, b, a, 7)   # and every 7th row of it against the oracle


def _uniforms_from_states(st: np.ndarray, n: int) -> np.ndarray:
    """rocrand_uniform draws of XORWOW states [6, m] (d, x0..x4): numpy restatement, float32."""
    d, x0, x1, x2, x3, x4 = (st[k].astype(np.uint32).copy() for k in range(6))
    out = np.empty((st.shape[1], n), dtype=np.float32)
    inv = np.float32(2.0 ** -32)
    for k in range(n):
        t = x0 ^ (x0 >> np.uint32(2))
        x0, x1, x2, x3 = x1, x2, x3, x4
        x4 = (x4 ^ (x4 << np.uint32(4))) ^ (t ^ (t << np.uint32(1)))
        d = d + np.uint32(362437)
        out[:, k] = (d + x4).astype(np.float32) * inv + inv   # f*inv exact, one rounding of the sum
    return out


@pytest.mark.parametrize("width,rows,row_offset,row_stride", [(3840, 3, 2157, 1), (3840, 4, 1, 541),
                                                             (1920, 2, 1078, 1), (2715, 3, 5, 509)])
def test_device_seeding_matches_oracle_at_full_size(width, rows, row_offset, row_stride):
    # init_gpu_data (:1591-1606) at BASELINE sizes: subsequence = global pixel index up to 8.3 M (4K);
    # every pixel of the sampled rows vs the oracle's own rocRAND-equivalent seeding, 8 draws each
    st = rt.seed_states(1234, width, row_offset, row_stride, rows)
    got = _uniforms_from_states(st, 8)
    L = _abi.oracle_lib()
    ref = np.empty(8, dtype=np.float32)
    for k in range(rows):
        g0 = (row_offset + k * row_stride) * width
        for j in list(range(0, width, 97)) + [width - 1]:
            L.rt_oracle_uniforms(1234, g0 + j, ref.ctypes.data_as(C.c_void_p), 8)
            assert np.array_equal(got[k * width + j].view(np.uint32), ref.view(np.uint32)), (k, j)


@pytest.mark.parametrize("scene,args", [(0, ["s4", "b4", "w64", "h36"]), (17, ["s2", "b50", "w48", "h27"])])
def test_cli_writes_the_oracle_ppm(scene, args, tmp_path):
    # the reference's CLI surface (main.cu:29-131, `./raytracing 0 s4 b4` is BASELINE config 1) end to
    # end on the GPU: catalog scene -> BVH -> camera -> rt_render -> settings.img_name as P6 bytes
    import subprocess
    from conftest import REPO
    exe = REPO / "bin" / "raytracing"
    assert exe.exists(), "bin/raytracing not built (make cli)"
    r = subprocess.run([str(exe), str(scene), *args], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    w, s = rt.build_scene(scene)
    opts = {a[0]: int(a[1:]) for a in args}
    cam, W, H = rt.camera_from_settings(s, opts["w"], opts["h"])
    p = rt.make_params(s, W, H, spp=opts["s"], bounces=opts["b"])
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    data = (tmp_path / s.img_name.decode()).read_bytes()
    header = f"P6\n{W} {H}\n255\n".encode()
    assert data.startswith(header)
    assert data[len(header):] == rt.tonemap(ref).tobytes()


@pytest.mark.parametrize("idx,W,H,spp,b", [(0, 96, 54, 8, 16), (17, 64, 36, 4, 50), (1, 40, 40, 4, 50), (0, 33, 7, 2, 0)])
def test_fused_ppm_bytes_match_host_tonemap(idx, W, H, spp, b):
    # rt_context_render_ppm: the render kernel writes each finished pixel's P6 bytes; they must equal the
    # host pixels_to_ppm conversion of the float frame it writes alongside (b = 0: the all-zero path)
    import torch
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    out8 = torch.full((H, W, 3), 7, dtype=torch.uint8, device="cuda")
    ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream, out8.data_ptr())
    torch.cuda.synchronize()
    fb = out.cpu().numpy()
    assert np.array_equal(out8.cpu().numpy(), rt.tonemap(fb))
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("tiled", ["1", "0", "auto"])
@pytest.mark.parametrize("tile_w", ["8", "32"])
@pytest.mark.parametrize("idx,W,H,spp,b", [(0, 96, 54, 8, 16), (17, 64, 36, 4, 50), (1, 40, 40, 4, 50), (20, 72, 44, 2, 8),
                                           (3, 40, 40, 2, 8), (0, 33, 7, 2, 16), (0, 260, 20, 1, 4)])
def test_tiled_output_matches_oracle(idx, W, H, spp, b, tile_w, tiled, monkeypatch):
    # Tile-major output (the default, since round 6 with noise textures too; RT_TILED_OUT=0: each pixel stored row-major
    # with its bytes by the render kernel, =1: tile-major):
    # the render kernel writes the float frame tile-major and untile_kernel writes the caller's row-major floats and
    # the P6 bytes in 128-column bands — bit-identical to the oracle and to the host tonemap, partial edge tiles and
    # bands included, on the static (LDS-only and pooled deep kernels), verified sphere and mixed walks, 8x8 and 32x2
    import torch
    if tiled == "auto":
        monkeypatch.delenv("RT_TILED_OUT", raising=False)
    else:
        monkeypatch.setenv("RT_TILED_OUT", tiled)
    monkeypatch.setenv("RT_TILE_W", tile_w)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.full((H, W, 3), -1.0, dtype=torch.float32, device="cuda")
    out8 = torch.full((H, W, 3), 7, dtype=torch.uint8, device="cuda")
    ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream, out8.data_ptr())
    torch.cuda.synchronize()
    fb = out.cpu().numpy()
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))
    assert np.array_equal(out8.cpu().numpy(), rt.tonemap(ref))
    fb2, st = gpu(w.scene(), cam, p)   # the one-shot entry point (host copy of the floats)
    assert np.array_equal(bits(fb2), bits(ref))
    assert st.tiled_out == (0 if tiled == "0" else 1)   # tile-major by default, noise scenes included (round 6)


def _random_world(seed: int):
    """A random scene outside the catalog: every primitive kind, transform and material kind of the
    reference's builder API (raytracing.cu:1775-2005), sizes and placements drawn from `seed`."""
    g = np.random.default_rng(seed)
    w = rt.World(capacity=512)
    u = lambda lo, hi, n=3: tuple(float(x) for x in g.uniform(lo, hi, n))  # noqa: E731

    def material():
        k = g.integers(0, 7)
        if k == 0:
            return w.metal(u(0.2, 1.0), float(g.uniform(0, 1)))
        if k == 1:
            return w.dielectric(float(g.uniform(1.1, 2.4)))
        if k == 2:
            return w.light(u(0.5, 6.0))
        if k == 3:
            return w.checker(float(g.uniform(0.2, 3)), u(0, 1), u(0, 1))
        if k == 4 and seed % 3 == 0:
            return w.noise(float(g.uniform(0.5, 6)))
        return w.lambert(u(0, 1))

    for _ in range(int(g.integers(4, 28))):
        kind = int(g.integers(0, 6))
        xf = int(g.integers(0, 4))
        kw = dict(xf=xf, angle=float(g.uniform(-180, 180)), offset=u(-1.5, 1.5))
        c = u(-3, 3)
        m = material()
        if kind == 0:
            w.sphere(c, float(g.uniform(0.1, 1.2)), m, **kw)
        elif kind == 1:
            w.moving_sphere(c, u(-0.5, 0.5), float(g.uniform(0.1, 0.8)), m, **kw)
        elif kind == 2:
            w.quad(c, u(-2, 2), u(-2, 2), m, **kw)
        elif kind == 3:
            w.triangle(c, u(-2, 2), u(-2, 2), m, **kw)
        elif kind == 4:
            a = np.array(c)
            w.box(tuple(a), tuple(a + g.uniform(0.2, 1.5, 3)), m, **kw)
        else:
            a = np.array(c)
            b = a + g.uniform(0.3, 1.5, 3)
            w.pyramid(tuple(a), (float(b[0]), float(a[1]), float(b[2])),
                      (float((a[0] + b[0]) / 2), float(b[1]), float((a[2] + b[2]) / 2)), m, **kw)
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom = rt.vec3(*u(-8, 8))
    s.lookat = rt.vec3(*u(-1, 1))
    s.vfov = float(g.uniform(20, 90))
    s.defocus_angle = float(g.choice([0.0, 0.0, g.uniform(0.1, 2.0)]))
    s.background = rt.vec3(*((0.0, 0.0, 0.0) if seed % 4 == 1 else u(0.2, 1.0)))
    return w, s


@pytest.mark.parametrize("seed", list(range(int(__import__("os").environ.get("RT_FUZZ_SEEDS", "12")))))
def test_random_scenes_vs_oracle(seed):
    # scenes no catalog entry covers (mixed kinds under translate/rotate, lights, checker/noise
    # textures, motion blur, defocus, black backgrounds): auto policy and the forced traversals,
    # bit-exact against the oracle
    w, s = _random_world(seed)
    cam, W, H = rt.camera_from_settings(s, 48, 27)
    p = rt.make_params(s, W, H, spp=4, bounces=10)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    fb, st = gpu(w.scene(), cam, p)
    assert np.array_equal(bits(fb), bits(ref)), f"auto policy (traversal {st.traversal})"
    for force, _want in TRAVERSALS:
        p.flags = force
        fb, _ = gpu(w.scene(), cam, p)
        assert np.array_equal(bits(fb), bits(ref)), force


def _random_sphere_world(seed: int):
    """All-sphere world for the verified SAH walk: random sizes (incl. a ground sphere), exact
    duplicates (bitwise-equal roots: the tie fallback), moving spheres, every material kind."""
    g = np.random.default_rng(1000 + seed)
    w = rt.World(capacity=2048)
    mats = [w.lambert((0.5, 0.5, 0.5)), w.metal((0.8, 0.7, 0.6), 0.2), w.dielectric(1.5),
            w.light((4.0, 4.0, 4.0)), w.checker(1.0, (0.2, 0.3, 0.1), (0.9, 0.9, 0.9))]
    w.sphere((0.0, -1000.0, 0.0), 1000.0, mats[0])
    n = int(g.integers(64, 400))
    for k in range(n):
        c = (float(g.uniform(-8, 8)), float(g.uniform(0, 3)), float(g.uniform(-8, 8)))
        r = float(g.choice([0.05, 0.2, 0.5, 1.0, float(g.uniform(0.01, 2))]))
        m = mats[int(g.integers(0, len(mats)))]
        if k % 17 == 0:
            w.moving_sphere(c, (0.0, float(g.uniform(0, 0.5)), 0.0), r, m)
        else:
            w.sphere(c, r, m)
        if k % 23 == 0:
            w.sphere(c, r, m)   # exact duplicate: equal roots, the reference's DFS order decides
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom = rt.vec3(float(g.uniform(-12, 12)), float(g.uniform(1, 6)), float(g.uniform(-12, 12)))
    s.lookat = rt.vec3(0.0, 0.5, 0.0)
    s.vfov = float(g.uniform(20, 70))
    s.defocus_angle = float(g.choice([0.0, 0.6]))
    s.background = rt.vec3(0.7, 0.8, 1.0)
    return w, s


@pytest.mark.parametrize("seed", list(range(int(__import__("os").environ.get("RT_FUZZ_SEEDS", "12")) // 2)))
def test_random_sphere_worlds_verified_walk(seed):
    w, s = _random_sphere_world(seed)
    cam, W, H = rt.camera_from_settings(s, 64, 36)
    p = rt.make_params(s, W, H, spp=4, bounces=12)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    p.flags = rt.RT_FLAG_FORCE_ACCEL
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_ACCEL
    assert np.array_equal(bits(fb), bits(ref))


# ---- BASELINE configs at their full frame size: strided rows (first and last included) vs the oracle ----
# (scene, W, H, spp, bounces, row stride): the GPU renders the WHOLE frame (reduced spp), the oracle the
# rows 0, s, 2s, ..., H-1 of it (the RNG subsequence is the global pixel index, so any row set is
# comparable); once with the auto policy and once with the forced reference lane walk
FULL_SIZE_CONFIGS = [
    (0, 1920, 1080, 4, 16, 83),       # config 2
    (1, 1920, 1080, 2, 50, 83),       # config 3 (scene 1 as indexed: Cornell box)
    (17, 1920, 1080, 2, 50, 83),      # config 3 (the Perlin spheres the config names)
    (20, 1920, 1080, 2, 16, 83),      # config 4 (10k random spheres)
    (0, 3840, 2160, 1, 50, 127),      # config 5
]


@pytest.mark.parametrize("idx,W,H,spp,b,stride", FULL_SIZE_CONFIGS)
@pytest.mark.parametrize("force", [0, rt.RT_FLAG_FORCE_LANE])
def test_full_size_config_rows_match_oracle(idx, W, H, spp, b, stride, force):
    assert (H - 1) % stride == 0   # the strided rows end on the last row
    w, s = rt.build_scene(idx)
    cam, W2, H2 = rt.camera_from_settings(s, W, H)
    assert (W2, H2) == (W, H)
    full, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=spp, bounces=b, flags=force))
    if force:
        assert st.traversal == rt.RT_TRAV_LANE
    p = rt.make_params(s, W, H, spp=spp, bounces=b, row_offset=0, row_stride=stride, row_count=(H - 1) // stride + 1)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    got = full[0::stride]
    assert got.shape == ref.shape
    bad = np.argwhere(bits(got) != bits(ref))
    assert bad.size == 0, f"{len(bad)} values differ, first at row {bad[0][0] * stride} col {bad[0][1]}"


@pytest.mark.parametrize("idx,W,H,spp,b,rows", [
    (0, 1920, 1080, 512, 16, 2),      # config 2
    (1, 1920, 1080, 1024, 50, 1),     # config 3 (Cornell)
    (17, 1920, 1080, 1024, 50, 2),    # config 3 (Perlin)
    (20, 1920, 1080, 256, 16, 2),     # config 4
    (0, 3840, 2160, 2048, 50, 1),     # config 5
])
def test_full_spp_config_rows_match_oracle(idx, W, H, spp, b, rows):
    # every BASELINE config at its FULL sample count and depth: a shard of rows through the middle of the frame (the
    # rows' own global pixel indices seed their RNG streams), rendered by the default policy, equals the oracle's
    # rendering of the same rows bit for bit
    w, s = rt.build_scene(idx)
    cam, W2, H2 = rt.camera_from_settings(s, W, H)
    assert (W2, H2) == (W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b, row_offset=H // 2, row_stride=37, row_count=rows)
    fb, st = gpu(w.scene(), cam, p)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and fb.shape == ref.shape == (rows, W, 3)
    bad = np.argwhere(bits(fb) != bits(ref))
    assert bad.size == 0, f"{len(bad)} values differ, first at {bad[0].tolist()}"


def test_fold_violation_rerenders_exactly(monkeypatch):
    # force the folded kernel's ray-bound flag (RT_FOLD_CHECK_BOUND lowers its threshold): rt_render must
    # re-render unfolded BEFORE copying the frame out, stats or not, and the PPM bytes of the context path
    # must come from the re-rendered frame too
    monkeypatch.setenv("RT_FOLD_CHECK_BOUND", "0.25")
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 40, 24)
    p = rt.make_params(s, W, H, spp=3, bounces=8)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_STATIC and st.fold_rerenders == 1
    assert np.array_equal(bits(fb), bits(ref))
    fb2 = rt.render(w.scene(), cam, p)            # no stats requested: the check still runs
    assert np.array_equal(bits(fb2), bits(ref))
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    out8 = torch.full((H, W, 3), 7, dtype=torch.uint8, device="cuda")
    ctx.render_into(cam, p, out.data_ptr(), torch.cuda.current_stream().cuda_stream, out8.data_ptr())
    st = ctx.timing()
    torch.cuda.synchronize()
    assert st.fold_rerenders == 1
    assert np.array_equal(bits(out.cpu().numpy()), bits(ref))
    assert np.array_equal(out8.cpu().numpy(), rt.tonemap(ref))
    ctx.close()


def test_failed_render_never_reports_stale_timings():
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 32, 18)
    ctx = rt.RenderContext(w.scene(), 0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ctx.render_into(cam, rt.make_params(s, W, H, spp=2, bounces=4), out.data_ptr(), stream)
    st = ctx.timing()
    assert st.render_ms > 0 and st.samples == W * H * 2
    bad = rt.make_params(s, W, H, spp=2, bounces=4)
    bad.row_stride = 0
    with pytest.raises(rt.RenderError):
        ctx.render_into(cam, bad, out.data_ptr(), stream)
    st = ctx.timing()
    assert st.render_ms == 0 and st.samples == 0 and st.init_ms == 0
    ctx.render_into(cam, rt.make_params(s, W, H, spp=2, bounces=4), out.data_ptr(), stream)
    assert ctx.timing().samples == W * H * 2
    ctx.close()


def test_code_object_disk_cache(tmp_path):
    # a second process finds the scene-specialised kernels on disk (no hipRTC compile) and writes the
    # same PPM bytes; the CLI reports the end-to-end time of the whole reference render() region
    import os
    import subprocess
    from conftest import REPO
    exe = REPO / "bin" / "raytracing"
    env = dict(os.environ, RT_JIT_CACHE_DIR=str(tmp_path / "cache"))
    outs = []
    for k in range(2):
        d = tmp_path / f"run{k}"
        d.mkdir()
        r = subprocess.run([str(exe), "0", "s2", "b4", "w64", "h36"], cwd=d, capture_output=True, text=True,
                           timeout=180, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        outs.append((r.stdout, b"".join(f.read_bytes() for f in sorted(d.glob("*.ppm")))))
    assert "[compiled" in outs[0][0] and "[disk cache" in outs[1][0], (outs[0][0], outs[1][0])
    assert "End-to-end:" in outs[1][0]
    assert outs[0][1] and outs[0][1] == outs[1][1]
    assert list((tmp_path / "cache").glob("rt_*.co"))


@pytest.mark.parametrize("idx", [17, 19])
@pytest.mark.parametrize("env", [{}, {"RT_COOP_NOISE": "0"}, {"RT_COOP_NOISE": "8", "RT_PRIO_CHUNK": "64"},
                                 {"RT_PRIO_LANES": "64", "RT_PRIO_CHUNK": "8"}, {"RT_PRIO_LANES": "64"},
                                 {"RT_PRIO_LANES": "2", "RT_PRIO_TILES": "6"},
                                 {"RT_PRIO_LANES": "1", "RT_PRIO_TILES": "300"}])
def test_cooperative_noise_octaves_vs_oracle(idx, env, monkeypatch):
    # noise scenes: perlin_turbulence's octaves spread over 2/4/8 lanes per noise lane (render_body's
    # cooperative block), the costliest tiles handed out pixel by pixel, waves holding them kept sparse
    # (the default on noise scenes; RT_PRIO_LANES=64 turns it off; 300 tiles = every tile of this
    # frame) — the frame is the oracle's
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, 192, 108)
    p = rt.make_params(s, W, H, spp=16, bounces=50)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_STATIC
    assert np.array_equal(bits(fb), bits(ref))


# ---- colour stack (ray_color's attenuation stack, raytracing.cu:1253-1276,1362-1368) past its LDS levels ----
# RT_RC_LDS_LEVELS pins the LDS levels low (4, and 5: odd, so the 16-bit kernels' level pairs round up to 6),
# so every path deeper than that pushes and unwinds HBM levels; RT_FLAG_RC_AUDIT counts the HBM slots the
# render wrote (> 0 proves the spill path ran) — on every traversal policy, against the oracle
SPILL_FORCES = [0, rt.RT_FLAG_FORCE_LANE, rt.RT_FLAG_FORCE_PACKET, rt.RT_FLAG_FORCE_STATIC]


def _spill_check(w, s, W, H, spp, b, forces, want_levels):
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    for force in forces:
        p.flags = force | rt.RT_FLAG_RC_AUDIT
        fb, st = gpu(w.scene(), cam, p)
        assert np.array_equal(bits(fb), bits(ref)), (force, st.traversal)
        assert st.rc_lds_levels in want_levels, (force, st.rc_lds_levels)
        assert st.rc_hbm_slots > 0, (force, st.traversal)


@pytest.mark.parametrize("levels", ["4", "5"])
@pytest.mark.parametrize("idx,W,H,spp", [(1, 40, 40, 4), (17, 48, 27, 4), (20, 48, 27, 2)])
def test_colour_stack_hbm_levels_vs_oracle(idx, W, H, spp, levels, monkeypatch):
    monkeypatch.setenv("RT_RC_LDS_LEVELS", levels)
    w, s = rt.build_scene(idx)
    forces = SPILL_FORCES + ([rt.RT_FLAG_FORCE_ACCEL] if idx == 20 else [])
    L = int(levels)   # 16-bit codes round the LDS levels up to even, 8-bit codes (kVarByte) to a multiple of 4
    _spill_check(w, s, W, H, spp, 50, forces, {L, L + 1, (L + 3) // 4 * 4})


@pytest.mark.parametrize("levels", ["4", "5"])
@pytest.mark.parametrize("seed", [1, 6])
def test_colour_stack_hbm_levels_random_worlds(seed, levels, monkeypatch):
    monkeypatch.setenv("RT_RC_LDS_LEVELS", levels)
    w, s = _random_world(seed)
    # a closed diffuse room around the camera and the random objects: paths end only at lights, at
    # absorbing metal bounces or at depth 50, so many are deeper than the LDS levels
    w.box((-20.0, -20.0, -20.0), (20.0, 20.0, 20.0), w.lambert((0.8, 0.75, 0.7)))
    L = int(levels)
    _spill_check(w, s, 48, 27, 8, 50, SPILL_FORCES, {L, L + 1, (L + 3) // 4 * 4})


def _pool_render(w, s, W, H, spp, b, force, pool, monkeypatch):
    monkeypatch.setenv("RT_RC_POOL", str(pool))
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=b)
    p.flags = force | rt.RT_FLAG_RC_AUDIT
    return gpu(w.scene(), cam, p), cam, p


# ---- deep-level pool (kVarRcPool, RT_RC_POOL): a path's levels past the LDS ones in one of its wave's LDS chunks
# when one is free at its first deep push, else in HBM.  Few chunks (2: most deep paths overflow to HBM, chunks are
# taken and returned every round) and many (32), on the static, per-lane and verified sphere walks, bit-exact; the
# chunks keep levels out of HBM (fewer audited HBM slots than the same render without a pool) ----
@pytest.mark.parametrize("idx,W,H,spp,forces", [
    (1, 40, 40, 4, [0, rt.RT_FLAG_FORCE_LANE]),
    (17, 48, 27, 4, [0, rt.RT_FLAG_FORCE_LANE]),
    (20, 48, 27, 2, [rt.RT_FLAG_FORCE_ACCEL]),
])
def test_colour_stack_pool_vs_oracle(idx, W, H, spp, forces, monkeypatch):
    monkeypatch.setenv("RT_RC_LDS_LEVELS", "4")
    w, s = rt.build_scene(idx)
    cam, W2, H2 = rt.camera_from_settings(s, W, H)
    rc, ref, _ = oracle_render(w.scene(), cam, rt.make_params(s, W2, H2, spp=spp, bounces=50))
    assert rc == 0
    for force in forces:
        (fb0, st0), _, _ = _pool_render(w, s, W, H, spp, 50, force, 0, monkeypatch)
        assert st0.rc_pool_chunks == 0 and st0.rc_hbm_slots > 0, (force, st0.traversal)
        assert np.array_equal(bits(fb0), bits(ref)), (force, st0.traversal)
        for pool in (2, 32):
            (fb, st), _, _ = _pool_render(w, s, W, H, spp, 50, force, pool, monkeypatch)
            assert np.array_equal(bits(fb), bits(ref)), (force, pool, st.traversal)
            assert 0 < st.rc_pool_chunks <= pool, (force, pool, st.rc_pool_chunks)
            assert st.rc_lds_levels == st0.rc_lds_levels
            # (2 chunks: a lane may write a level to HBM in one path and to a chunk in another, so only "not more")
            assert (st.rc_hbm_slots < st0.rc_hbm_slots) if pool == 32 else (st.rc_hbm_slots <= st0.rc_hbm_slots), \
                (force, pool, st.rc_hbm_slots, st0.rc_hbm_slots)


@pytest.mark.parametrize("seed", [1, 6])
def test_colour_stack_pool_random_worlds(seed, monkeypatch):
    # the closed room of test_colour_stack_hbm_levels_random_worlds: many paths reach depth 50, so chunks run out
    monkeypatch.setenv("RT_RC_LDS_LEVELS", "4")
    w, s = _random_world(seed)
    w.box((-20.0, -20.0, -20.0), (20.0, 20.0, 20.0), w.lambert((0.8, 0.75, 0.7)))
    cam, W, H = rt.camera_from_settings(s, 48, 27)
    rc, ref, _ = oracle_render(w.scene(), cam, rt.make_params(s, W, H, spp=8, bounces=50))
    assert rc == 0
    for force in SPILL_FORCES:
        for pool in (1, 4, 32):
            (fb, st), _, _ = _pool_render(w, s, 48, 27, 8, 50, force, pool, monkeypatch)
            assert np.array_equal(bits(fb), bits(ref)), (force, pool, st.traversal)
            assert st.rc_pool_chunks > 0 or force == rt.RT_FLAG_FORCE_PACKET, (force, pool)


@pytest.mark.parametrize("idx,W,H,spp", [(17, 64, 36, 8), (0, 64, 36, 4)])
def test_colour_stack_pool_automatic_levels(idx, W, H, spp, monkeypatch):
    # levels chosen by the host (no RT_RC_LDS_LEVELS): the pool takes its bytes from the per-lane levels at d50
    w, s = rt.build_scene(idx)
    cam, W2, H2 = rt.camera_from_settings(s, W, H)
    rc, ref, _ = oracle_render(w.scene(), cam, rt.make_params(s, W2, H2, spp=spp, bounces=50))
    assert rc == 0
    (fb0, st0), _, _ = _pool_render(w, s, W, H, spp, 50, 0, 0, monkeypatch)
    (fb, st), _, _ = _pool_render(w, s, W, H, spp, 50, 0, 16, monkeypatch)
    assert np.array_equal(bits(fb0), bits(ref)) and np.array_equal(bits(fb), bits(ref))
    if st0.rc_lds_levels < 50:   # a kernel with HBM levels: the pool is used (its per-lane levels follow the pool
        # kernel's own residency, which may differ) and keeps levels out of HBM
        assert st.rc_pool_chunks > 0
        assert st.rc_hbm_slots <= st0.rc_hbm_slots


@pytest.mark.parametrize("b", [16, 17])
@pytest.mark.parametrize("idx", [1, 17])
def test_deep_unwind_switch_vs_oracle(idx, b, monkeypatch):
    # max_bounces > kDeepBounces (16) selects the batched HBM unwind (kVarDeep): both sides of the switch
    monkeypatch.setenv("RT_RC_LDS_LEVELS", "4")
    w, s = rt.build_scene(idx)
    _spill_check(w, s, 40, 30, 6, b, [0, rt.RT_FLAG_FORCE_LANE], {4, 5})


# ---- verified traversal of mixed worlds (RT_TRAV_MIXED): the reference DFS above the transform-free
# subtrees, a SAH walk + reach proof inside them (mixed_accel.cpp, MixedTraceK) ----
def _mixed_world(seed: int):
    """final_scene-like (raytracing.cu:2151-2202) at random: a grid of boxes of random heights, a cluster of
    spheres under y-rotation + translation, transformed boxes and pyramids (groups inside transforms), loose
    quads / triangles / spheres, a light.  Large enough for dynamic macros (>= 64 primitives below nodes
    with transforms)."""
    g = np.random.default_rng(5000 + seed)
    w = rt.World(capacity=4000)
    ground = w.lambert((0.48, 0.83, 0.53))
    n = int(g.integers(6, 11))
    for i in range(n):
        for j in range(n):
            x0, z0 = -5.0 + i * 1.0, -5.0 + j * 1.0
            w.box((x0, 0.0, z0), (x0 + 1.0, float(g.uniform(0.05, 1.2)), z0 + 1.0), ground)
    mats = [w.lambert((0.73, 0.73, 0.73)), w.metal((0.8, 0.8, 0.9), float(g.uniform(0, 1))), w.dielectric(1.5),
            w.checker(0.5, (0.2, 0.3, 0.1), (0.9, 0.9, 0.9))]
    for _ in range(int(g.integers(10, 60))):
        c = tuple(float(x) for x in g.uniform(0, 1.6, 3))
        w.sphere(c, 0.1, mats[0], xf=rt.RT_XF_YROTATE_TRANSLATE, angle=15.0, offset=(-1.0, 2.7, 0.95))
    for _ in range(int(g.integers(1, 5))):
        a = g.uniform(-3, 3, 3)
        w.box(tuple(a), tuple(a + g.uniform(0.3, 1.0, 3)), mats[int(g.integers(0, 4))],
              xf=int(g.integers(1, 4)), angle=float(g.uniform(-90, 90)), offset=tuple(float(x) for x in g.uniform(-1, 1, 3)))
    a = g.uniform(-2, 2, 3)
    w.pyramid(tuple(a), (float(a[0] + 1), float(a[1]), float(a[2] + 1)), (float(a[0] + 0.5), float(a[1] + 1), float(a[2] + 0.5)),
              mats[0], xf=rt.RT_XF_YROTATE, angle=30.0)
    for _ in range(int(g.integers(1, 6))):
        c = tuple(float(x) for x in g.uniform(-3, 3, 3))
        k = int(g.integers(0, 3))
        if k == 0:
            w.sphere(c, float(g.uniform(0.2, 0.8)), mats[int(g.integers(0, 4))])
        elif k == 1:
            w.quad(c, tuple(float(x) for x in g.uniform(-1, 1, 3)), tuple(float(x) for x in g.uniform(-1, 1, 3)), mats[0])
        else:
            w.triangle(c, tuple(float(x) for x in g.uniform(-1, 1, 3)), tuple(float(x) for x in g.uniform(-1, 1, 3)), mats[3])
    w.quad((-1.0, 4.5, -1.0), (2.0, 0.0, 0.0), (0.0, 0.0, 2.0), w.light((7.0, 7.0, 7.0)))
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom = rt.vec3(float(g.uniform(-6, 6)), float(g.uniform(2, 5)), float(g.uniform(-9, -6)))
    s.lookat = rt.vec3(0.0, 1.0, 0.0)
    s.vfov = float(g.uniform(30, 60))
    s.background = rt.vec3(*((0.0, 0.0, 0.0) if seed % 2 else (0.5, 0.6, 0.8)))
    return w, s


def test_mixed_traversal_final_scene_vs_oracle():
    w, s = rt.build_scene(3)   # final_scene: 400 boxes, 1000 rotated + translated spheres
    info = rt.mixed_build(w.scene())
    assert info and info["macros"] > 0 and info["dynamic"] > 0
    cam, W, H = rt.camera_from_settings(s, 80, 80)
    p = rt.make_params(s, W, H, spp=3, bounces=40)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_MIXED and st.mix_macros == info["macros"]
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("seed", list(range(int(__import__("os").environ.get("RT_FUZZ_SEEDS", "12")) // 2)))
def test_random_mixed_worlds_verified_walk(seed):
    w, s = _mixed_world(seed)
    assert rt.mixed_build(w.scene())
    cam, W, H = rt.camera_from_settings(s, 64, 36)
    p = rt.make_params(s, W, H, spp=4, bounces=12)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    p.flags = rt.RT_FLAG_FORCE_MIXED
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_MIXED
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("seed", [3, 7, 9])
def test_random_scenes_forced_mixed_walk(seed):
    # the small random worlds of test_random_scenes_vs_oracle through the mixed walk (static macros only)
    w, s = _random_world(seed)
    cam, W, H = rt.camera_from_settings(s, 48, 27)
    p = rt.make_params(s, W, H, spp=4, bounces=10)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    p.flags = rt.RT_FLAG_FORCE_MIXED
    fb, st = gpu(w.scene(), cam, p)
    assert np.array_equal(bits(fb), bits(ref)), st.traversal


def test_mixed_walk_fallback_path_vs_oracle(monkeypatch):
    # RT_MIX_PROVE=0: every macro walk is handed back to the reference's expansion of its root
    monkeypatch.setenv("RT_MIX_PROVE", "0")
    w, s = _mixed_world(1)
    cam, W, H = rt.camera_from_settings(s, 48, 27)
    p = rt.make_params(s, W, H, spp=3, bounces=10, flags=rt.RT_FLAG_FORCE_MIXED)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    fb, st = gpu(w.scene(), cam, p)
    assert rc == 0 and st.traversal == rt.RT_TRAV_MIXED and st.mix_fallbacks > 0
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("env", [{"RT_DEFER_TRACE": "64", "RT_TRACE_MIN": "1"}, {"RT_MIX_PAUSE": "0"},
                                 {"RT_MIX_PACK": "0"}, {"RT_MIX_PAUSE": "0", "RT_MIX_PACK": "0"},
                                 {"RT_PRIO_MIX": "1", "RT_PRIO_LANES": "4", "RT_PRIO_TILES": "8"},
                                 {"RT_PRIO_MIX": "1", "RT_PRIO_LANES": "2", "RT_PRIO_TILES": "100000"}])
def test_mixed_walk_pause_and_packed_chains(monkeypatch, env):
    # the walk paused between reference steps (forced early: any round with <= 1/4 of its walkers left)
    # and sphere chains packed into their head records, each on and off, vs the oracle
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for w, s, size, spp, b in ((*rt.build_scene(3), 72, 3, 40), (*_mixed_world(2), 64, 4, 12)):
        cam, W, H = rt.camera_from_settings(s, size, size)
        p = rt.make_params(s, W, H, spp=spp, bounces=b, flags=rt.RT_FLAG_FORCE_MIXED)
        rc, ref, _ = oracle_render(w.scene(), cam, p)
        assert rc == 0
        fb, st = gpu(w.scene(), cam, p)
        assert st.traversal == rt.RT_TRAV_MIXED
        assert np.array_equal(bits(fb), bits(ref)), env


def test_mixed_walk_final_scene_full_size_rows():
    # the final_scene frame (800x800, d40) at reduced spp: every 61st row (first and last) vs the oracle
    w, s = rt.build_scene(3)
    cam, W, H = rt.camera_from_settings(s, 800, 800)
    full, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=2, bounces=40))
    assert st.traversal == rt.RT_TRAV_MIXED
    stride = 47
    p = rt.make_params(s, W, H, spp=2, bounces=40, row_offset=0, row_stride=stride, row_count=(H - 1) // stride + 1)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    assert np.array_equal(bits(full[0::stride]), bits(ref))


def _checker_of_image_world():
    """Spheres whose checker texture has an image child (texture_get_color follows the checker recursion down
    to the image, raytracing.cu:366-384): their u,v must be computed although the material's own texture is a
    checker.  The builder API makes checkers of two solids only, so the checker's even TextureRef is patched in
    the arena bytes to point at the image texture."""
    import struct
    w = rt.World(capacity=512)
    yy, xx = np.mgrid[0:23, 0:41].astype(np.float32)
    img = w.image_pixels(np.stack([xx / 40.0, yy / 22.0, 0.3 + 0.4 * ((xx + 2 * yy) % 5 == 0)], axis=-1).astype(np.float32))
    chk = w.checker(0.9, (0.9, 0.2, 0.1), (0.1, 0.8, 0.3))
    g = np.random.default_rng(77)
    w.sphere((0.0, -100.5, -2.0), 100.0, w.lambert((0.5, 0.5, 0.5)))
    for _ in range(80):   # a transform-free subtree for the SAH walk
        c = (float(g.uniform(-3, 3)), float(g.uniform(-0.3, 1.5)), float(g.uniform(-6, -1.5)))
        w.sphere(c, float(g.uniform(0.1, 0.35)), chk if g.uniform() < 0.6 else w.metal((0.8, 0.7, 0.6), 0.2))
    w.box((-0.5, -0.5, -3.0), (0.5, 0.5, -2.0), chk, xf=rt.RT_XF_YROTATE_TRANSLATE, angle=25.0, offset=(1.0, 0.0, 0.0))
    b = w.blobs()
    tex = bytearray(b["textures"])
    chk_off = struct.unpack_from("<Q", bytes(chk.payload), 0)[0]
    img_off = struct.unpack_from("<Q", bytes(img.payload), 0)[0]
    assert struct.unpack_from("<I", tex, chk_off)[0] == 1 and struct.unpack_from("<I", tex, img_off)[0] == 2
    struct.pack_into("<Q", tex, chk_off + 16, img_off)   # checker.even -> the image texture
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom, s.lookat, s.vfov = rt.vec3(0, 1.0, 1.0), rt.vec3(0, 0.2, -3), 70.0
    return rt.BlobScene(b["hittables"], b["refs"], bytes(tex), b["root"]), s


def test_checker_of_image_spheres_compute_uv_vs_oracle():
    # the lazy sphere-u,v flag must see an image below a checker; every traversal incl. the mixed walk
    bs, s = _checker_of_image_world()
    sc = bs.scene()
    cam, W, H = rt.camera_from_settings(s, 64, 36)
    p = rt.make_params(s, W, H, spp=4, bounces=8)
    rc, ref, _ = oracle_render(sc, cam, p)
    assert rc == 0 and len(np.unique(ref.reshape(-1, 3), axis=0)) > 100
    for force in (0, rt.RT_FLAG_FORCE_MIXED, rt.RT_FLAG_FORCE_LANE, rt.RT_FLAG_FORCE_STATIC):
        p.flags = force
        fb, st = gpu(sc, cam, p)
        assert np.array_equal(bits(fb), bits(ref)), (force, st.traversal)


def test_image_texture_over_2_23_words_vs_oracle():
    # a texel pool of more than 2^23 words (a 1700x1700 float RGB map, 8.67 M words): colour-stack texel codes
    # carry 31-bit word offsets, so such scenes render (they were RT_ERR_UNSUPPORTED with 23-bit codes)
    w = rt.World(capacity=64, arena_bytes=48 << 20)
    h = wd = 1700
    yy, xx = np.mgrid[0:h, 0:wd].astype(np.float32)
    tex = np.stack([xx / (wd - 1), yy / (h - 1), 0.2 + 0.6 * (((xx // 97) + (yy // 89)) % 2)], axis=-1).astype(np.float32)
    assert tex.size > (1 << 23)
    img = w.image_pixels(tex)
    w.sphere((0, 0, -2), 0.8, img)
    w.quad((-3, -1, -4), (6, 0, 0), (0, 0, 3.5), img)
    w.sphere((1.2, 0.3, -2.5), 0.5, w.metal((0.8, 0.8, 0.8), 0.1))
    s = rt.Settings()
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom, s.lookat, s.vfov = rt.vec3(0, 0.3, 0), rt.vec3(0, 0, -1), 90.0
    cam, W, H = rt.camera_from_settings(s, 48, 27)
    p = rt.make_params(s, W, H, spp=4, bounces=8, flags=rt.RT_FLAG_RC_AUDIT)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and len(np.unique(ref.reshape(-1, 3), axis=0)) > 50
    fb, st = gpu(w.scene(), cam, p)
    assert np.array_equal(bits(fb), bits(ref))


# ---- one process, N devices through the C-ABI (rt_render_devices: row deal, RCCL gather, un-permute) ----
def test_render_devices_one_gpu_vs_oracle():
    # the whole multi-device path with N = 1 (the GPU box has one device): RCCL communicator, the shard's render
    # with PPM bytes, the grouped ncclGather of bytes and floats to the root, the un-permute kernel, the copy back
    n_dev = C.c_int()
    _abi.hip_lib().rt_device_count(C.byref(n_dev))
    devices = list(range(min(n_dev.value, 8)))
    for idx, W, H, spp, b in ((0, 96, 54, 8, 16), (20, 64, 36, 2, 16)):
        w, s = rt.build_scene(idx)
        cam, W, H = rt.camera_from_settings(s, W, H)
        p = rt.make_params(s, W, H, spp=spp, bounces=b)
        rc, ref, _ = oracle_render(w.scene(), cam, p)
        assert rc == 0
        f, u8, st = rt.render_devices(w.scene(), cam, p, devices, with_stats=True)
        assert st.devices == len(devices) and st.samples == W * H * spp and st.render_kernel_ms > 0
        assert np.array_equal(bits(f), bits(ref)) and np.array_equal(u8, rt.tonemap(ref))
        # a row subset of the frame (strided rows, as one rank's shard of a larger job) through the same path
        ps = rt.make_params(s, W, H, spp=spp, bounces=b, row_offset=1, row_stride=3)
        rc, refs, _ = oracle_render(w.scene(), cam, ps)
        f2, u2 = rt.render_devices(w.scene(), cam, ps, devices)
        assert np.array_equal(bits(f2), bits(refs)) and np.array_equal(u2, rt.tonemap(refs))
        # bytes only
        none, u3 = rt.render_devices(w.scene(), cam, p, devices, rgb=False)
        assert none is None and np.array_equal(u3, rt.tonemap(ref))


def test_render_devices_rejects_bad_arguments():
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 16, 9)
    p = rt.make_params(s, W, H, spp=1, bounces=4)
    for devs in ([0, 0], [-1], [1 << 20]):
        with pytest.raises(rt.RenderError) as e:
            rt.render_devices(w.scene(), cam, p, devs)
        assert e.value.code == _abi.RT_ERR_INVALID_ARG
    with pytest.raises(rt.RenderError):
        rt.render_devices(w.scene(), cam, p, [0], rgb=False, ppm=False)


def test_kernel_span_within_event_window():
    # rt_stats.render_kernel_ms (first wave start .. last wave end, s_memrealtime) is the kernel alone: positive and
    # never above the stream-event window around the launch
    w, s = rt.build_scene(0)
    cam, W, H = rt.camera_from_settings(s, 320, 180)
    fb, st = gpu(w.scene(), cam, rt.make_params(s, W, H, spp=16, bounces=8))
    assert 0 < st.render_kernel_ms <= st.render_ms * 1.001 + 0.01, (st.render_kernel_ms, st.render_ms)


# ---- the verified sphere walk over the 4-wide tree (RT_ACCEL_WIDTH=4, accel::collapse_wide) ----
# (float 128-B nodes by default; RT_ACCEL_QUANT=1: the quantised 64-B nodes, accel::quantize_wide)
@pytest.mark.parametrize("idx,W,H,spp,quant", [(2, 64, 36, 4, "1"), (20, 160, 90, 6, "1"), (20, 480, 270, 4, "1"),
                                               (2, 64, 36, 4, "0"), (20, 160, 90, 6, "0")])
def test_wide_verified_sphere_traversal_matches_oracle(idx, W, H, spp, quant, monkeypatch):
    monkeypatch.setenv("RT_ACCEL_WIDTH", "4")
    monkeypatch.setenv("RT_ACCEL_QUANT", quant)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=16, flags=rt.RT_FLAG_FORCE_ACCEL)
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_ACCEL and st.accel_spheres > 0
    if W * H <= 160 * 90:
        rc, ref, _ = oracle_render(w.scene(), cam, p)
        assert rc == 0 and np.array_equal(bits(fb), bits(ref))
    else:
        _rows_match_oracle(w, s, cam, W, H, spp, 16, fb, 7)
    # counters: the same reference visits, the 4-wide walk's own executed steps
    pc = rt.make_params(s, W, H, spp=2, bounces=16, flags=rt.RT_FLAG_FORCE_ACCEL | rt.RT_FLAG_COUNT)
    _, sc4 = gpu(w.scene(), cam, pc)
    monkeypatch.setenv("RT_ACCEL_WIDTH", "2")
    _, sc2 = gpu(w.scene(), cam, pc)
    a, b = sc4.counter_dict(), sc2.counter_dict()
    assert a["visit_bvh"] == b["visit_bvh"] and a["visit_sphere"] == b["visit_sphere"]
    assert 0 < a["exec_node"] and 0 < a["exec_prim"]


@pytest.mark.parametrize("seed,quant", [(0, "1"), (1, "1"), (2, "1"), (3, "1"), (4, "1"), (5, "1"), (0, "0"), (3, "0")])
def test_wide_random_sphere_worlds_verified_walk(seed, quant, monkeypatch):
    monkeypatch.setenv("RT_ACCEL_WIDTH", "4")
    monkeypatch.setenv("RT_ACCEL_QUANT", quant)
    _wide_world_vs_oracle(seed)


# the round-4 mis-render (a paused walk's hit flag lost by the 6-wave, register-capped build) on every world that showed
# it on the r04 trees (seeds 0-6: r05 diagnosis, profiles/r05_w4_diag.txt), at the 6 waves every width now asks for and
# at 5
@pytest.mark.parametrize("waves", ["6", "5"])
@pytest.mark.parametrize("seed", [0, 1, 2, 3, 4, 5, 6])
def test_wide_walk_paused_state_register_budgets(seed, waves, monkeypatch):
    monkeypatch.setenv("RT_ACCEL_WIDTH", "4")
    monkeypatch.setenv("RT_ACCEL_QUANT", "0")
    monkeypatch.setenv("RT_ACCEL_WAVES", waves)
    _wide_world_vs_oracle(seed)


def _wide_world_vs_oracle(seed):
    w, s = _random_sphere_world(seed)
    cam, W, H = rt.camera_from_settings(s, 64, 36)
    p = rt.make_params(s, W, H, spp=4, bounces=12)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    p.flags = rt.RT_FLAG_FORCE_ACCEL
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_ACCEL
    assert np.array_equal(bits(fb), bits(ref))


@pytest.mark.parametrize("byte", ["1", "0"])
def test_byte_colour_codes_all_levels_in_lds(byte, monkeypatch):
    # Cornell box (few colour records): 8-bit codes keep all 50 levels in LDS by default (RT_RC_BYTE=0: 16-bit codes,
    # fewer LDS levels); both bit-exact vs the oracle
    monkeypatch.setenv("RT_RC_BYTE", byte)
    w, s = rt.build_scene(1)
    cam, W, H = rt.camera_from_settings(s, 40, 40)
    p = rt.make_params(s, W, H, spp=4, bounces=50, flags=rt.RT_FLAG_RC_AUDIT)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    fb, st = gpu(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))
    if byte == "1":
        assert st.rc_lds_levels >= 50 and st.rc_hbm_slots == 0, (st.rc_lds_levels, st.rc_hbm_slots)


# ---- primary-ray candidate lists of the verified sphere walk (device/prim_lists.h, RT_ACCEL_PRIM) ----
@pytest.mark.parametrize("idx,W,H,spp", [(20, 160, 90, 4), (2, 96, 54, 4)])
def test_primary_candidate_lists_match_oracle(idx, W, H, spp, monkeypatch):
    monkeypatch.setenv("RT_ACCEL_PRIM", "1")   # (default: worlds of >= 2048 spheres)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=16, flags=rt.RT_FLAG_FORCE_ACCEL)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0
    fb, st = gpu(w.scene(), cam, p)
    assert st.traversal == rt.RT_TRAV_ACCEL and np.array_equal(bits(fb), bits(ref))
    # a row shard (lists per shard tile: taller footprints)
    ps = rt.make_params(s, W, H, spp=spp, bounces=16, row_offset=1, row_stride=3, flags=rt.RT_FLAG_FORCE_ACCEL)
    rc, refs, _ = oracle_render(w.scene(), cam, ps)
    fs, _ = gpu(w.scene(), cam, ps)
    assert np.array_equal(bits(fs), bits(refs))
    # the camera rays take the lists: fewer executed node visits than with the lists off, same reference counts
    pc = rt.make_params(s, W, H, spp=2, bounces=16, flags=rt.RT_FLAG_FORCE_ACCEL | rt.RT_FLAG_COUNT)
    _, on = gpu(w.scene(), cam, pc)
    monkeypatch.setenv("RT_ACCEL_PRIM", "0")
    fo, _ = gpu(w.scene(), cam, p)
    _, off = gpu(w.scene(), cam, pc)
    a, b = on.counter_dict(), off.counter_dict()
    assert np.array_equal(bits(fo), bits(ref))
    assert a["visit_bvh"] == b["visit_bvh"] and a["exec_node"] < b["exec_node"], (a, b)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_primary_candidate_lists_random_worlds(seed, monkeypatch):
    # moving spheres, duplicates, defocus (the random verified-walk worlds): bit-exact with the lists on
    monkeypatch.setenv("RT_ACCEL_PRIM", "1")
    w, s = _random_sphere_world(seed)
    cam, W, H = rt.camera_from_settings(s, 64, 36)
    p = rt.make_params(s, W, H, spp=4, bounces=12, flags=rt.RT_FLAG_FORCE_ACCEL)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    fb, st = gpu(w.scene(), cam, p)
    assert rc == 0 and st.traversal == rt.RT_TRAV_ACCEL and np.array_equal(bits(fb), bits(ref))


def test_seed_tables_stream_ordered_between_queued_frames():
    # the per-geometry RNG tables are rewritten when the seed / width / rows change.  Two frames queued back
    # to back on one non-blocking stream with different seeds and widths (no host sync between them): the first must
    # keep the tables it was launched with (stream-ordered upload from pinned staging), both bit-exact vs the oracle
    w, s = rt.build_scene(0)
    ctx = rt.RenderContext(w.scene(), 0)
    stream = torch.cuda.Stream()
    cam_a, Wa, Ha = rt.camera_from_settings(s, 1920, 1080)
    pa = rt.make_params(s, Wa, Ha, spp=32, bounces=16)
    pa.seed = 1234
    cam_b, Wb, Hb = rt.camera_from_settings(s, 400, 224)
    pb = rt.make_params(s, Wb, Hb, spp=4, bounces=16)
    pb.seed = 77
    out_a = torch.empty((Ha, Wa, 3), dtype=torch.float32, device="cuda")
    out_b = torch.empty((Hb, Wb, 3), dtype=torch.float32, device="cuda")
    ctx.render_into(cam_a, pa, out_a.data_ptr(), stream.cuda_stream)
    ctx.render_into(cam_b, pb, out_b.data_ptr(), stream.cuda_stream)   # new seed and width while frame A renders
    ctx.timing()
    stream.synchronize()
    # frame A on a strided row sample (the RNG subsequence is the global pixel index: shard invariance)
    pchk = rt.make_params(s, Wa, Ha, spp=32, bounces=16, row_offset=5, row_stride=97, row_count=len(range(5, Ha, 97)))
    pchk.seed = 1234
    rc, ref_a, _ = oracle_render(w.scene(), cam_a, pchk)
    assert rc == 0 and np.array_equal(bits(out_a.cpu().numpy()[5::97]), bits(ref_a))
    rc, ref_b, _ = oracle_render(w.scene(), cam_b, pb)
    assert rc == 0 and np.array_equal(bits(out_b.cpu().numpy()), bits(ref_b))
    ctx.close()


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("row_bytes", [111, 444])   # a u8 row of 37 px (not a multiple of 4) and a float row
def test_multi_unpermute_matches_numpy(n, row_bytes):
    # the root's un-permute of rt_multi_render (rows dealt round-robin, shards padded to the longest) on one
    # device: shards shorter than max_rows (their padding rows hold garbage that must never be read), word and byte rows
    rows = 29
    max_rows = (rows + n - 1) // n
    g = np.random.default_rng(row_bytes * 10 + n)
    gathered = g.integers(0, 256, size=(n, max_rows, row_bytes), dtype=np.uint8)
    src = torch.from_numpy(gathered).cuda()
    out = torch.zeros((rows, row_bytes), dtype=torch.uint8, device="cuda")
    rc = _abi.hip_lib().rt_multi_unpermute(C.c_void_p(src.data_ptr()), C.c_void_p(out.data_ptr()), rows, n, max_rows,
                                          row_bytes, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    want = np.stack([gathered[k % n, k // n] for k in range(rows)])
    assert np.array_equal(out.cpu().numpy(), want)
    bad = _abi.hip_lib().rt_multi_unpermute(C.c_void_p(src.data_ptr()), C.c_void_p(out.data_ptr()), rows, n,
                                           max_rows - 1, row_bytes, None)
    assert bad == _abi.RT_ERR_INVALID_ARG


@pytest.mark.parametrize("tile_w,slots", [("8", "1"), ("8", "4"), ("32", "4"), ("8", "-1")])
@pytest.mark.parametrize("idx,W,H,spp", [(0, 96, 54, 8), (0, 37, 29, 4), (20, 72, 44, 2)])
def test_staged_tile_writes_partial_tiles(idx, W, H, spp, tile_w, slots, monkeypatch):
    # output staging (RT_STAGE_SLOTS) with partial tiles at the frame's edges: the float frame and the PPM bytes laid out
    # back to back in one allocation, then a guard — a store past either must show (round 5 found the valid mask of a
    # partial tile sign-extended by readfirstlane, which wrote the missing rows' floats into the bytes after the frame)
    import torch
    monkeypatch.setenv("RT_TILE_W", tile_w)
    monkeypatch.setenv("RT_STAGE_SLOTS", slots)
    w, s = rt.build_scene(idx)
    cam, W, H = rt.camera_from_settings(s, W, H)
    p = rt.make_params(s, W, H, spp=spp, bounces=16)
    n = W * H * 3
    buf = torch.full((n * 4 + n + 4096,), 0xA5, dtype=torch.uint8, device="cuda")
    ctx = rt.RenderContext(w.scene(), 0)
    ctx.render_into(cam, p, buf.data_ptr(), torch.cuda.current_stream().cuda_stream, buf.data_ptr() + n * 4)
    ctx.timing()
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    fb = host[:n * 4].view(np.float32).reshape(H, W, 3)
    rc, ref, _ = oracle_render(w.scene(), cam, p)
    assert rc == 0 and np.array_equal(bits(fb), bits(ref))
    assert np.array_equal(host[n * 4:n * 5].reshape(H, W, 3), rt.tonemap(ref))
    assert (host[n * 5:] == 0xA5).all()
    ctx.close()
