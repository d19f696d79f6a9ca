"""Host-side checks of the verified sphere traversal's SAH tree (sphere_accel.cpp), no GPU needed.

The kernel-side argument (device/rt_body.h, AccelTraceK) needs: every sphere of the world exactly once
in the tree, every child box containing its spheres over the motion, M bounding |centre| + radius, and
per sphere the box of its deepest BVH ancestor in the REFERENCE tree.  These are checked here on the
catalog scenes the policy applies to; scenes with other primitives must be rejected.
"""
from __future__ import annotations

import numpy as np
import pytest

import cuda_raytracing_amd as rt

LEAF = 0x80000000


def f(u):
    return np.asarray(u, np.uint32).view(np.float32)


def reference_spheres(sc):
    """sphere record -> deepest BVH ancestor box (x0 x1 y0 y1 z0 z1), walking the reference records
    (rtr_hittable, include/rt_ref_layout.h: 120 B, union at byte 8)."""
    import ctypes as C
    raw = np.frombuffer(C.string_at(sc.hittables, 120 * sc.hittable_count), np.uint8).reshape(-1, 120)
    refs = np.ctypeslib.as_array(sc.refs, shape=(sc.ref_count,))
    kind = raw[:, 0:4].copy().view(np.uint32)[:, 0]
    out = {}
    stack = [(int(refs[sc.root]), None)]
    while stack:
        i, parent = stack.pop()
        if kind[i] == 1:   # BVH: u16 left/right WorldRefs, then the box
            l, r = (int(refs[x]) for x in raw[i, 8:12].copy().view(np.uint16))
            box = tuple(float(x) for x in raw[i, 12:36].copy().view(np.float32))
            stack.append((l, box))
            if r != l:
                stack.append((r, box))
        elif kind[i] == 0:
            assert i not in out
            out[i] = parent
        elif kind[i] == 6:   # group: u16 first, count (u64) at union offset 40
            first = int(raw[i, 8:10].copy().view(np.uint16)[0])
            count = int(raw[i, 48:56].copy().view(np.uint64)[0])
            for k in range(count):
                stack.append(((first + k) & 0xffff, parent))
        else:
            return None
    return out


@pytest.mark.parametrize("idx", [2, rt.RT_SCENE_RANDOM_10K])
def test_tree_covers_every_sphere_once(idx):
    w, _ = rt.build_scene(idx)
    sc = w.scene()
    res = rt.accel_build(sc)
    assert res is not None
    info, nodes, prims = res
    nodes = nodes.reshape(-1, 16)
    prims = prims.reshape(-1, 16)
    assert info["spheres"] == len(prims) and not (info["root"] & LEAF)
    seen = np.zeros(len(prims), np.int32)
    depth_max = 0
    stack = [(info["root"], 1)]
    while stack:
        node, d = stack.pop()
        depth_max = max(depth_max, d)
        q = nodes[node]
        for c in range(2):
            box = f(q[6 * c: 6 * c + 6])
            ref = int(q[12 + c])
            m = float(f(q[14 + c]))
            if ref & LEAF:
                first, cnt = ref & 0xffffff, ((ref >> 24) & 0x7f) + 1
                for k in range(first, first + cnt):
                    seen[k] += 1
                    p = prims[k]
                    c0, mv = f(p[0:3]).astype(np.float64), f(p[3:6]).astype(np.float64)
                    rad = np.sqrt(np.float64(f(p[6])))
                    lo = np.minimum(c0, c0 + mv) - rad
                    hi = np.maximum(c0, c0 + mv) + rad
                    assert np.all(box[0::2] <= lo) and np.all(box[1::2] >= hi), (node, c, k)
                    assert m >= np.linalg.norm(c0) + np.linalg.norm(mv) + rad - 1e-3
            else:
                cb = nodes[ref]
                for cc in range(2):   # the child's boxes lie inside this box
                    inner = f(cb[6 * cc: 6 * cc + 6])
                    assert np.all(box[0::2] <= inner[0::2]) and np.all(box[1::2] >= inner[1::2])
                stack.append((ref, d + 1))
    assert np.all(seen == 1)
    assert depth_max <= info["depth"] + 1


@pytest.mark.parametrize("idx", [2, rt.RT_SCENE_RANDOM_10K])
def test_nodes_are_breadth_first(idx):
    # accel_build.h bfs_order: the root is node 0 and the internal children, listed node by node, are
    # nodes 1, 2, 3, ...: every prefix of the array is a complete top of the tree (the LDS-staged part)
    w, _ = rt.build_scene(idx)
    info, nodes, _ = rt.accel_build(w.scene())
    nodes = nodes.reshape(-1, 16)
    assert info["root"] == 0
    kids = [int(nodes[i, 12 + c]) for i in range(len(nodes)) for c in range(2) if not (int(nodes[i, 12 + c]) & LEAF)]
    assert kids == list(range(1, len(nodes)))


@pytest.mark.parametrize("idx", [2, rt.RT_SCENE_RANDOM_10K])
def test_verification_boxes_are_reference_ancestors(idx):
    w, _ = rt.build_scene(idx)
    sc = w.scene()
    _, _, prims = rt.accel_build(sc)
    prims = prims.reshape(-1, 16)
    ref = reference_spheres(sc)
    assert ref is not None and len(ref) == len(prims)
    for p in prims:
        node = int(p[9])
        want = ref[node]
        got = tuple(float(x) for x in f(p[10:16]))
        assert want is not None and got == want, node


@pytest.mark.parametrize("idx", [0, 1, 17])
def test_other_worlds_are_not_eligible(idx):
    w, _ = rt.build_scene(idx)
    assert rt.accel_build(w.scene()) is None


@pytest.mark.parametrize("idx", [2, rt.RT_SCENE_RANDOM_10K])
def test_wide_tree_is_the_same_tree_four_wide(idx):
    # accel::collapse_wide: every BVH2 leaf appears once among the wide nodes' children, each with its BVH2
    # (padded) box; inner children are wide nodes numbered breadth-first; empty slots never hit
    w, _ = rt.build_scene(idx)
    info, nodes2, _ = rt.accel_build(w.scene())
    wide = rt.accel_build_wide(w.scene())
    assert wide is not None
    winfo, wn = wide
    wn = wn.reshape(-1, 32)
    nodes2 = nodes2.reshape(-1, 16)
    leaves2 = {}
    for q in nodes2:
        for c in range(2):
            if int(q[12 + c]) & LEAF:
                leaves2[int(q[12 + c])] = tuple(q[6 * c: 6 * c + 6])
    leaves4 = {}
    kids = []
    for i, q in enumerate(wn):
        for c in range(4):
            ref = int(q[24 + c])
            box = tuple(int(q[4 * k + c]) for k in range(6))
            bf = f(np.array(box, np.uint32))
            if ref & LEAF:
                assert ref not in leaves4
                leaves4[ref] = tuple(np.array(box, np.uint32))
            elif np.isinf(bf[0]) and bf[0] > 0:   # empty slot: (+inf, -inf) on every axis
                assert ref == 0 and all(np.isinf(bf))
            else:
                kids.append(ref)
                inner = wn[ref]
                for cc in range(4):   # the child's own child boxes lie inside this box
                    ib = f(np.array([inner[4 * k + cc] for k in range(6)], np.uint32))
                    if np.isinf(ib[0]) and ib[0] > 0:
                        continue
                    assert np.all(bf[0::2] <= ib[0::2]) and np.all(bf[1::2] >= ib[1::2])
    assert {k: tuple(np.array(v, np.uint32)) for k, v in leaves2.items()} == leaves4
    assert kids == list(range(1, len(wn)))   # breadth-first
    assert winfo["stack"] == 3 * winfo["depth"] + 1 and winfo["depth"] <= info["depth"]


@pytest.mark.parametrize("idx", [2, rt.RT_SCENE_RANDOM_10K])
def test_quantised_wide_tree_contains_the_float_boxes(idx):
    # accel::quantize_wide (rt_layout.h kAccel4Q*): same refs and numbering as the float 4-wide nodes; the valid
    # mask marks the non-empty slots; every decoded box (origin + q * 2^e, exact in float64) contains its float
    # box widened by 2^-20 of the node's largest |plane| on the axis (the kernel's evaluation rounding), and stays
    # within two steps of it (the quantisation is outward rounding, not a looser box)
    w, _ = rt.build_scene(idx)
    _, wn = rt.accel_build_wide(w.scene())
    qi, qn = rt.accel_build_wide(w.scene(), quant=True)
    wn = wn.reshape(-1, 32)
    qn = qn.reshape(-1, 16)
    assert len(qn) == len(wn) == qi["nodes"]
    for fw, q in zip(wn, qn):
        assert [int(x) for x in q[10:14]] == [int(x) for x in fw[24:28]]
        meta = int(q[3])
        org = f(q[0:3]).astype(np.float64)
        for c in range(4):
            box = f(np.array([fw[4 * k + c] for k in range(6)], np.uint32)).astype(np.float64)
            empty = np.isinf(box[0]) and box[0] > 0
            assert bool(meta >> (24 + c) & 1) == (not empty)
            if empty:
                continue
            for a in range(3):
                lo_all = [f(np.array([fw[8 * a + cc]], np.uint32))[0] for cc in range(4) if meta >> (24 + cc) & 1]
                hi_all = [f(np.array([fw[8 * a + 4 + cc]], np.uint32))[0] for cc in range(4) if meta >> (24 + cc) & 1]
                ep = max(abs(min(lo_all)), abs(max(hi_all))) * 2.0 ** -20
                step = 2.0 ** (((meta >> (8 * a)) & 0xff) - 127)
                ql = (int(q[4 + 2 * a]) >> (8 * c)) & 0xff
                qh = (int(q[5 + 2 * a]) >> (8 * c)) & 0xff
                lo, hi = org[a] + ql * step, org[a] + qh * step
                assert lo <= box[2 * a] - ep and hi >= box[2 * a + 1] + ep, (a, c)
                assert lo > box[2 * a] - ep - 2 * step and hi < box[2 * a + 1] + ep + 2 * step, (a, c)


def _cam_vecs(cam):
    v = lambda x: np.array(x.tolist(), np.float32)  # noqa: E731
    return (v(cam.pixel00), v(cam.delta_u), v(cam.delta_v), v(cam.center), v(cam.defocus_u), v(cam.defocus_v))


def _random_moving_world(seed):
    g = np.random.default_rng(500 + seed)
    w = rt.World(capacity=1024)
    m = w.lambert((0.5, 0.5, 0.5))
    w.sphere((0.0, -1000.0, 0.0), 1000.0, m)
    for k in range(int(g.integers(80, 300))):
        c = (float(g.uniform(-6, 6)), float(g.uniform(0, 3)), float(g.uniform(-6, 6)))
        r = float(g.choice([0.05, 0.3, 1.0]))
        if k % 9 == 0:
            w.moving_sphere(c, (0.0, float(g.uniform(0, 0.6)), 0.0), r, m)
        else:
            w.sphere(c, r, m)
    s = rt.Settings()
    import ctypes as C
    from cuda_raytracing_amd import _abi
    _abi.host_lib().rt_settings_default(C.byref(s))
    s.lookfrom = rt.vec3(float(g.uniform(-10, 10)), float(g.uniform(1, 5)), float(g.uniform(-10, 10)))
    s.lookat = rt.vec3(0.0, 0.5, 0.0)
    s.vfov = float(g.uniform(25, 60))
    s.defocus_angle = float(g.choice([0.0, 0.6, 3.0]))
    return w, s


@pytest.mark.parametrize("case", ["10k", "10k_shard", "rand0", "rand1", "rand2"])
def test_primary_candidate_lists_hold_every_hit(case):
    # device/prim_lists.h (built here on the host by the same code): for camera rays of each tile, generated in
    # float32 as the kernel does (defocus disc, pixel jitter), the closest sphere by brute force over every sphere
    # is in the tile's list, and its axial bound lies within rho + t |d| (the kernel's early exit keeps it)
    if case.startswith("10k"):
        w, s = rt.build_scene(rt.RT_SCENE_RANDOM_10K)
        W, H = 320, 180
    else:
        w, s = _random_moving_world(int(case[-1]))
        W, H = 96, 64
    cam, W, H = rt.camera_from_settings(s, W, H)
    off, stride, rows = (1, 3, (H - 1) // 3) if case == "10k_shard" else (0, 1, H)
    p = rt.make_params(s, W, H, spp=1, bounces=4, row_offset=off, row_stride=stride, row_count=rows)
    res = rt.prim_lists(w.scene(), cam, p, cap=256)
    assert res is not None
    counts, lists, rho = res
    _, _, prims = rt.accel_build(w.scene())
    P = prims.reshape(-1, 16)
    pc = f(P[:, 0:3]).astype(np.float64)
    mv = f(P[:, 3:6]).astype(np.float64)
    rad2 = f(P[:, 6]).astype(np.float64)
    p00, du, dv, C0, dfu, dfv = _cam_vecs(cam)
    g = np.random.default_rng(7)
    tiles_x = (W + 7) // 8
    assert (counts != 0xFFFFFFFF).mean() > 0.9
    checked = 0
    for t in range(len(counts)):
        if counts[t] == 0xFFFFFFFF:
            continue
        n = int(counts[t])
        ids = lists[t, :n, 0].astype(np.int64)
        bnd = f(lists[t, :n, 1]).astype(np.float64)
        assert np.all(np.diff(bnd) >= 0)
        ty, tx = divmod(t, tiles_x)
        for _ in range(3):
            lr = min(ty * 8 + int(g.integers(0, 8)), rows - 1)
            j = min(tx * 8 + int(g.integers(0, 8)), W - 1)
            i = off + lr * stride
            if cam.defocus_angle > 0:
                while True:
                    y, x = np.float32(g.uniform(-1, 1)), np.float32(g.uniform(-1, 1))
                    if x * x + y * y < 1:
                        break
                O = C0 + (x * dfu + y * dfv)
            else:
                O = C0
            xo, yo = np.float32(g.uniform(-0.5, 0.5)), np.float32(g.uniform(-0.5, 0.5))
            pp = p00 + (np.float32(i) * dv + np.float32(j) * du)
            D = ((pp - O) + xo * du) + yo * dv
            tm = np.float64(g.uniform(0, 1))
            o, d = O.astype(np.float64), D.astype(np.float64)
            c = pc + tm * mv
            oc = c - o
            a = d @ d
            b = -2 * (oc @ d)
            cc = (oc * oc).sum(1) - rad2
            disc = b * b - 4 * a * cc
            ok = disc >= 0
            sq = np.sqrt(np.where(ok, disc, 0))
            r1, r2 = (-b - sq) / (2 * a), (-b + sq) / (2 * a)
            root = np.where(r1 > 1e-3, r1, r2)
            root = np.where(ok & (root > 1e-3), root, np.inf)
            k = int(root.argmin())
            if not np.isfinite(root[k]):
                continue
            assert k in set(ids.tolist()), (t, k)
            pos = int(np.nonzero(ids == k)[0][0])
            assert bnd[pos] <= rho + root[k] * np.sqrt(a), (t, k)
            checked += 1
    assert checked > 100
