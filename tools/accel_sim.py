#!/usr/bin/env python3
"""CPU simulation of the verified sphere walk's node visits (diagnostic, no GPU).

    python3 tools/accel_sim.py --scene 20 --rays 20000 [--pad current|none|M0]

Walks the SAH tree of rt.accel_build (node words as the kernel reads them: child boxes pre-padded by
kAccelKappa * M) with the kernel's order (near child first, leaves tested on arrival) for camera rays of the
scene's camera and for one Lambertian bounce from their hit points, and reports node visits / leaf tests per
ray.  --pad none shrinks every child box back by its kappa * M and drops the ray's kappa * |o|_1 share (the
visits an unpadded tree would make: the ceiling of what tighter padding can save); float64 arithmetic, so the
counts are estimates of the kernel's, not bit-exact.
"""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import cuda_raytracing_amd as rt  # noqa: E402

KAPPA = 1.953125e-3


def walk(nodes, prims, root, o, d, pad_mode, tmax0=None):
    """Lockstep DFS over all rays; returns (visits, prim_tests, t_hit, prim_hit)."""
    n = o.shape[0]
    inv = 1.0 / d
    ao = np.abs(o).sum(1)
    pinv = (KAPPA * ao)[:, None] * np.abs(inv) if pad_mode == "current" else np.zeros_like(o)
    NB = nodes.reshape(-1, 16)
    boxes = NB[:, :12].view(np.float32).astype(np.float64).reshape(-1, 2, 6)
    refs = NB[:, 12:14].astype(np.int64)
    ms = NB[:, 14:16].view(np.float32).astype(np.float64)
    if pad_mode == "none":
        b = boxes.copy()
        for c in range(2):
            pad = KAPPA * ms[:, c]
            b[:, c, 0::2] += pad[:, None]
            b[:, c, 1::2] -= pad[:, None]
        boxes = b
    P = prims.reshape(-1, 16)
    pc = P[:, 0:3].view(np.float32).astype(np.float64)
    pr2 = P[:, 6].view(np.float32).astype(np.float64)
    tmax = np.full(n, np.inf) if tmax0 is None else tmax0.copy()
    best = np.full(n, -1)
    stack = np.zeros((n, 64), np.int64)
    sp = np.zeros(n, np.int64)
    node = np.full(n, root, np.int64)
    walking = np.ones(n, bool)
    visits = np.zeros(n, np.int64)
    tests = np.zeros(n, np.int64)
    idx = np.arange(n)

    def box_t(bx, rows):
        oo, ii, pp = o[rows], inv[rows], pinv[rows]
        lo = (bx[:, 0::2] - oo) * ii
        hi = (bx[:, 1::2] - oo) * ii
        tn = np.minimum(lo, hi) - pp
        tf = np.maximum(lo, hi) + pp
        t0 = np.maximum(tn.max(1), 1e-3)
        t1 = np.minimum(tf.min(1), tmax[rows])
        return t1 >= t0, t0

    def leaf(ref, rows, on):
        cnt = np.where(on, ((ref >> 24) & 0x7f) + 1, 0)
        first = ref & 0xffffff
        for k in range(int(cnt.max()) if cnt.size else 0):
            sel = on & (k < cnt)
            r = rows[sel]
            pi = first[sel] + k
            tests[r] += 1
            oc = pc[pi] - o[r]
            dd = d[r]
            a = (dd * dd).sum(1)
            bb = -2 * (dd * oc).sum(1)
            cc = (oc * oc).sum(1) - pr2[pi]
            disc = bb * bb - 4 * a * cc
            ok = disc >= 0
            sq = np.sqrt(np.where(ok, disc, 0))
            t = (-bb - sq) / (2 * a)
            t = np.where((t <= 1e-3) | (t >= tmax[r]), (-bb + sq) / (2 * a), t)
            acc = ok & (t > 1e-3) & (t < tmax[r])
            tmax[r[acc]] = t[acc]
            best[r[acc]] = pi[acc]

    while walking.any():
        rows = idx[walking]
        nd = node[rows]
        visits[rows] += 1
        h0, n0 = box_t(boxes[nd, 0], rows)
        h1, n1 = box_t(boxes[nd, 1], rows)
        near0 = n0 <= n1
        rn = np.where(near0, refs[nd, 0], refs[nd, 1])
        rf = np.where(near0, refs[nd, 1], refs[nd, 0])
        hn = np.where(near0, h0, h1)
        hf = np.where(near0, h1, h0)
        ln = hn & ((rn & 0x80000000) != 0)
        lf = hf & ((rf & 0x80000000) != 0)
        leaf(rn, rows, ln)
        leaf(rf, rows, lf)
        hn &= ~ln
        hf &= ~lf
        both = hn & hf
        r = rows[both]
        stack[r, sp[r]] = rf[both]
        sp[r] += 1
        node[r] = rn[both]
        one = (hn ^ hf)
        node[rows[one]] = np.where(hn, rn, rf)[one]
        none = ~(hn | hf)
        r = rows[none]
        empty = sp[r] == 0
        walking[r[empty]] = False
        r2 = r[~empty]
        sp[r2] -= 1
        node[r2] = stack[r2, sp[r2]]
    return visits, tests, tmax, best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", type=int, default=20)
    ap.add_argument("--rays", type=int, default=20000)
    ap.add_argument("--pad", default="current", choices=["current", "none"])
    a = ap.parse_args()
    w, s = rt.build_scene(a.scene)
    cam, W, H = rt.camera_from_settings(s, 1920, 1080)
    info, nodes, prims = rt.accel_build(w.scene())
    g = np.random.default_rng(1)
    i = g.integers(0, H, a.rays)
    j = g.integers(0, W, a.rays)
    v = lambda x: np.array(x.tolist(), np.float64)  # noqa: E731
    p00, du, dv, c = v(cam.pixel00), v(cam.delta_u), v(cam.delta_v), v(cam.center)
    pp = p00 + i[:, None] * dv + j[:, None] * du
    if cam.defocus_angle > 0:
        ang = g.uniform(0, 2 * np.pi, a.rays)
        rr = np.sqrt(g.uniform(0, 1, a.rays))
        o = c + (rr * np.cos(ang))[:, None] * v(cam.defocus_u) + (rr * np.sin(ang))[:, None] * v(cam.defocus_v)
    else:
        o = np.tile(c, (a.rays, 1))
    d = pp - o + g.uniform(-0.5, 0.5, (a.rays, 1)) * du + g.uniform(-0.5, 0.5, (a.rays, 1)) * dv
    vis, tst, t, best = walk(nodes, prims, info["root"], o, d, a.pad)
    print(f"primary: visits/ray {vis.mean():.2f} tests/ray {tst.mean():.2f} hit {np.mean(best >= 0):.3f}")
    hit = best >= 0
    P = prims.reshape(-1, 16)
    pc = P[:, 0:3].view(np.float32).astype(np.float64)
    ph = o[hit] + t[hit, None] * d[hit]
    nrm = ph - pc[best[hit]]
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    u = g.normal(size=nrm.shape)
    u /= np.linalg.norm(u, axis=1)[:, None]
    d2 = nrm + u
    vis2, tst2, t2, best2 = walk(nodes, prims, info["root"], ph, d2, a.pad)
    print(f"bounce:  visits/ray {vis2.mean():.2f} tests/ray {tst2.mean():.2f} hit {np.mean(best2 >= 0):.3f}")


if __name__ == "__main__":
    main()


def collapse4(nodes, root, width=4):
    """BVH2 (kernel layout) -> wide nodes: each wide node's children = up to `width` BVH2 subtrees chosen by
    repeatedly opening the internal child with the largest box surface.  Returns (boxes [n, width, 6],
    refs [n, width] (-1 empty; >= 0 wide node; leaf refs keep kAccelLeaf), root 0)."""
    NB = nodes.reshape(-1, 16)
    boxes2 = NB[:, :12].view(np.float32).astype(np.float64).reshape(-1, 2, 6)
    refs2 = NB[:, 12:14].astype(np.int64)
    area = lambda b: 2 * ((b[1] - b[0]) * (b[3] - b[2]) + (b[3] - b[2]) * (b[5] - b[4]) + (b[5] - b[4]) * (b[1] - b[0]))  # noqa: E731
    out_boxes, out_refs = [], []
    queue = [root]
    ids = {root: 0}
    while queue:
        nd = queue.pop(0)
        kids = [(boxes2[nd, c], int(refs2[nd, c])) for c in range(2)]
        while len(kids) < width:
            cand = [(area(b), i) for i, (b, r) in enumerate(kids) if not (r & 0x80000000)]
            if not cand:
                break
            _, i = max(cand)
            b, r = kids.pop(i)
            kids += [(boxes2[r, c], int(refs2[r, c])) for c in range(2)]
        bx = np.zeros((width, 6))
        rf = np.full(width, -1, np.int64)
        for i, (b, r) in enumerate(kids):
            bx[i] = b
            if r & 0x80000000:
                rf[i] = r
            else:
                if r not in ids:
                    ids[r] = len(ids)
                    queue.append(r)
                rf[i] = ids[r] | (1 << 40)   # internal marker (resolved below)
        out_boxes.append(bx)
        out_refs.append(rf)
    refs = np.array(out_refs)
    internal = (refs >= 0) & ((refs & (1 << 40)) != 0)
    refs = np.where(internal, refs & ((1 << 40) - 1), refs)
    return np.array(out_boxes), refs, internal


def walk_wide(wboxes, wrefs, winternal, prims, o, d):
    """Ordered walk of the wide tree (nearest hit child next, the others pushed far-to-near)."""
    n = o.shape[0]
    inv = 1.0 / d
    ao = np.abs(o).sum(1)
    pinv = (KAPPA * ao)[:, None] * np.abs(inv)
    P = prims.reshape(-1, 16)
    pc = P[:, 0:3].view(np.float32).astype(np.float64)
    pr2 = P[:, 6].view(np.float32).astype(np.float64)
    W = wboxes.shape[1]
    visits = np.zeros(n, np.int64)
    tests = np.zeros(n, np.int64)
    tmax = np.full(n, np.inf)
    for r in range(n):
        stack = [0]
        while stack:
            nd = stack.pop()
            visits[r] += 1
            hits = []
            for c in range(W):
                ref = wrefs[nd, c]
                if ref < 0 and not winternal[nd, c]:
                    continue
                b = wboxes[nd, c]
                lo = (b[0::2] - o[r]) * inv[r]
                hi = (b[1::2] - o[r]) * inv[r]
                t0 = max((np.minimum(lo, hi) - pinv[r]).max(), 1e-3)
                t1 = min((np.maximum(lo, hi) + pinv[r]).min(), tmax[r])
                if t1 >= t0:
                    hits.append((t0, c))
            hits.sort()
            inner = []
            for t0, c in hits:
                ref = wrefs[nd, c]
                if winternal[nd, c]:
                    inner.append(ref)
                    continue
                cnt = ((ref >> 24) & 0x7f) + 1
                first = ref & 0xffffff
                for k in range(cnt):
                    pi = first + k
                    tests[r] += 1
                    oc = pc[pi] - o[r]
                    a = d[r] @ d[r]
                    bb = -2 * (d[r] @ oc)
                    cc = oc @ oc - pr2[pi]
                    disc = bb * bb - 4 * a * cc
                    if disc < 0:
                        continue
                    sq = np.sqrt(disc)
                    t = (-bb - sq) / (2 * a)
                    if t <= 1e-3 or t >= tmax[r]:
                        t = (-bb + sq) / (2 * a)
                    if 1e-3 < t < tmax[r]:
                        tmax[r] = t
            stack.extend(reversed(inner))
    return visits, tests
