// prim_lists.h — primary-ray candidate lists of the verified sphere walk (host and device).
//
// Every camera ray of a 64-pixel tile (raytracing.cu:1561-1578: origin in the defocus disc around the camera centre C,
// direction = the pixel sample point P on the focus plane - origin, P within half a pixel of the pixel centre) lies
// in the cone  K = union over t >= 0 of Ball(C + t a, rho + t w),  a = the tile footprint's centre Qc - C,
// w = rho + hq, where rho bounds |origin - C| and hq bounds |P - Qc| over the footprint (both widened for the
// rounding of the kernel's ray arithmetic): X(t) - (C + t a) = (1 - t)(O - C) + t (P - Qc), so
// |X(t) - (C + t a)| <= |1 - t| rho + t hq <= rho + t w.  A sphere can give the ray a root only if its ball padded by
// the verified walk's cone margin (a computed root lies within r + 2^-9 |o - c|_1 of the centre, rt_body.h) meets
// K (a moving sphere: the ball around its mid-time centre holding the sweep).  With z the axial coordinate along
// a^ = a / |a| from C and s = w / |a| < 1, K is the union of the balls B(C + z a^, rho + z s), z >= 0; for a ball
// B(c, R) with v = c - C, zc = v.a^, q = |v - zc a^|:
//   min over z >= 0 of |v - z a^| - z s = q sqrt(1 - s^2) - zc s   (at z* = zc + s q / sqrt(1 - s^2) >= 0)
//                                        = |v|                      (z* < 0),
// and B meets K iff that minimum <= R + rho (evaluated in double with an extra relative margin).  BVH boxes are
// culled against a square frustum holding K (prim_cone_box_out).  The kept spheres are sorted by a lower bound of
// their axial coordinate, zc - R (rounded down to float), then by index: the ray's axial coordinate below tmax is
// at most rho + tmax |d|, so a sphere whose bound exceeds that cannot yield a root below tmax, and neither can the
// rest of the list (AccelTraceK's list loop).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "rt_layout.h"

namespace rt {

struct PrimListGeom {
  double p00[3], du[3], dv[3], c[3];   // camera: pixel (0,0) centre, pixel steps, centre (rt_camera)
  double rho;                          // bound on |ray origin - centre| (defocus disc + rounding)
  double eps;                          // absolute widening of the footprint (rounding of the ray arithmetic)
  double half_motion;                  // max over spheres of |motion| / 2 (0: none moves)
  int32_t width, rows, row_offset, row_stride;
  uint32_t tiles_x;
  uint32_t tile_shift;                 // tiles of 64 pixels, 1 << tile_shift wide (RenderArgs::tile_shift)
};

constexpr uint32_t kPrimListNone = 0xffffffffu;   // count of a tile without a list (overflow / degenerate cone)
constexpr double kPrimPad = 1.0 / 512.0;          // kAccelKappa: the walk's cone margin per unit of |o - c|_1
constexpr double kSqrt3 = 1.7320508075688772;

__host__ __device__ inline double pl_len(const double v[3]) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
__host__ __device__ inline float pl_f(uint32_t b) { return __builtin_bit_cast(float, b); }
__host__ __device__ inline uint32_t pl_u(float f) { return __builtin_bit_cast(uint32_t, f); }

// one tile's cone: axis a^, slope s, and the frustum planes n_k.(X - C) <= hplane
struct PrimCone {
  double c[3], ah[3], rho, s, cs, hplane, pn[4][3];
};

// the cone of tile `tile` of the shard; false: no list (past the shard, degenerate or wide cone)
__host__ __device__ inline bool prim_cone(const PrimListGeom &g, uint32_t tile, PrimCone *k) {
  const uint32_t ty = tile / g.tiles_x, tx = tile - ty * g.tiles_x;
  const int32_t tw = 1 << g.tile_shift, th = 64 >> g.tile_shift;
  const int32_t lr0 = static_cast<int32_t>(ty) * th, lr1 = lr0 + th - 1 < g.rows - 1 ? lr0 + th - 1 : g.rows - 1;
  const int32_t j0 = static_cast<int32_t>(tx) * tw, j1 = j0 + tw - 1 < g.width - 1 ? j0 + tw - 1 : g.width - 1;
  if (lr0 >= g.rows || j0 >= g.width) return false;
  const double y0 = g.row_offset + static_cast<double>(lr0) * g.row_stride - 0.5;
  const double y1 = g.row_offset + static_cast<double>(lr1) * g.row_stride + 0.5;
  const double x0 = j0 - 0.5, x1 = j1 + 0.5;
  double qc[3], a[3];
  for (int i = 0; i < 3; ++i) qc[i] = g.p00[i] + 0.5 * (y0 + y1) * g.dv[i] + 0.5 * (x0 + x1) * g.du[i];
  double hq = 0.0;
  for (int cy = 0; cy < 2; ++cy)
    for (int cx = 0; cx < 2; ++cx) {
      double d[3];
      for (int i = 0; i < 3; ++i) d[i] = g.p00[i] + (cy ? y1 : y0) * g.dv[i] + (cx ? x1 : x0) * g.du[i] - qc[i];
      const double l = pl_len(d);
      hq = l > hq ? l : hq;
    }
  hq += g.eps;
  for (int i = 0; i < 3; ++i) { a[i] = qc[i] - g.c[i]; k->c[i] = g.c[i]; }
  const double la = pl_len(a);
  const double w = g.rho + hq;
  if (!(la > 0.0) || !(w < 0.5 * la)) return false;
  k->rho = g.rho;
  k->s = w / la;
  k->cs = sqrt(1.0 - k->s * k->s);
  for (int i = 0; i < 3; ++i) k->ah[i] = a[i] / la;
  // frustum: n = +-e_k - s' a^ with s' = s / sqrt(1 - s^2) keeps every ball B(C + z a^, rho + z s), z >= 0, below
  // n.(X - C) <= rho / sqrt(1 - s^2) (n.(z a^) + (rho + z s) |n| = rho / sqrt(1 - s^2) for every z)
  const double *ah = k->ah;
  const int m = (fabs(ah[0]) <= fabs(ah[1]) && fabs(ah[0]) <= fabs(ah[2])) ? 0 : (fabs(ah[1]) <= fabs(ah[2]) ? 1 : 2);
  double ax[3] = {0.0, 0.0, 0.0};
  ax[m] = 1.0;
  double e1[3] = {ah[1] * ax[2] - ah[2] * ax[1], ah[2] * ax[0] - ah[0] * ax[2], ah[0] * ax[1] - ah[1] * ax[0]};
  const double l1 = pl_len(e1);
  for (int i = 0; i < 3; ++i) e1[i] /= l1;
  const double e2[3] = {ah[1] * e1[2] - ah[2] * e1[1], ah[2] * e1[0] - ah[0] * e1[2], ah[0] * e1[1] - ah[1] * e1[0]};
  const double sp = k->s / k->cs;
  k->hplane = g.rho / k->cs;
  for (int i = 0; i < 3; ++i) {
    k->pn[0][i] = e1[i] - sp * ah[i]; k->pn[1][i] = -e1[i] - sp * ah[i];
    k->pn[2][i] = e2[i] - sp * ah[i]; k->pn[3][i] = -e2[i] - sp * ah[i];
  }
  return true;
}

// does the ball (c, R) meet the cone?  *axial: the ball's axial lower bound
__host__ __device__ inline bool prim_cone_meets(const PrimCone &k, const double c[3], double R, double *axial) {
  const double v[3] = {c[0] - k.c[0], c[1] - k.c[1], c[2] - k.c[2]};
  const double zc = v[0] * k.ah[0] + v[1] * k.ah[1] + v[2] * k.ah[2];
  const double p[3] = {v[0] - zc * k.ah[0], v[1] - zc * k.ah[1], v[2] - zc * k.ah[2]};
  const double q = pl_len(p), lv = pl_len(v);
  const double rr = (R + k.rho) * (1.0 + 1.0e-9) + 1.0e-12 * lv;
  *axial = zc - R;
  if (zc + k.s * q / k.cs >= 0.0) return q * k.cs - zc * k.s <= rr;
  return lv <= rr;
}

// is the box (centre bc, half-extents hd) wholly outside the frustum or behind the near plane a^.(X - C) >= -rho?
__host__ __device__ inline bool prim_cone_box_out(const PrimCone &k, const double bc[3], const double hd[3]) {
  const double v[3] = {bc[0] - k.c[0], bc[1] - k.c[1], bc[2] - k.c[2]};
  const double tol = 1.0e-9 * (fabs(v[0]) + fabs(v[1]) + fabs(v[2]) + hd[0] + hd[1] + hd[2] + k.rho);
  if (v[0] * k.ah[0] + v[1] * k.ah[1] + v[2] * k.ah[2] + fabs(k.ah[0]) * hd[0] + fabs(k.ah[1]) * hd[1] +
          fabs(k.ah[2]) * hd[2] < -k.rho - tol)
    return true;
  for (int i = 0; i < 4; ++i) {
    const double d = k.pn[i][0] * v[0] + k.pn[i][1] * v[1] + k.pn[i][2] * v[2] -
                     (fabs(k.pn[i][0]) * hd[0] + fabs(k.pn[i][1]) * hd[1] + fabs(k.pn[i][2]) * hd[2]);
    if (d > k.hplane + tol) return true;
  }
  return false;
}

// child ch of BVH node nd: may a sphere below it meet the cone?  Every sphere below has B(c, r) inside the box
// (c = its mid-time centre, on the swept sphere's axis) and is tested as B(c, r + |mv|/2 + margin): within the box
// widened by the half-motion bound and the largest margin of a sphere inside.
__host__ __device__ inline bool prim_cone_child(const PrimCone &k, const PrimListGeom &g, const uint32_t *nd, int ch) {
  const uint32_t *b = nd + 6 * ch;
  double bc[3], hd[3];
  for (int i = 0; i < 3; ++i) {
    const double lo = pl_f(b[2 * i]), hi = pl_f(b[2 * i + 1]);
    bc[i] = 0.5 * (lo + hi);
    hd[i] = 0.5 * (hi - lo);
  }
  if (!(hd[0] >= 0.0 && hd[1] >= 0.0 && hd[2] >= 0.0)) return false;
  const double m = g.half_motion + kPrimPad * (fabs(bc[0] - g.c[0]) + fabs(bc[1] - g.c[1]) + fabs(bc[2] - g.c[2]) +
                                               hd[0] + hd[1] + hd[2] + kSqrt3 * (pl_len(hd) + g.half_motion) + kSqrt3 * g.rho);
  const double hw[3] = {hd[0] + m, hd[1] + m, hd[2] + m};
  return !prim_cone_box_out(k, bc, hw);
}

// SAH prim pi: does its padded ball meet the cone?  *key: its axial lower bound as float bits (rounded down)
__host__ __device__ inline bool prim_cone_sphere(const PrimCone &k, const PrimListGeom &g, const uint32_t *prims, uint32_t pi,
                                                 uint32_t *key) {
  const uint32_t *pw = prims + static_cast<size_t>(pi) * kAccelPrimWords;
  double c[3], mv[3];
  for (int i = 0; i < 3; ++i) { mv[i] = pl_f(pw[AP_MOTION + i]); c[i] = pl_f(pw[AP_CENTER + i]) + 0.5 * mv[i]; }
  const double R0 = sqrt(static_cast<double>(pl_f(pw[AP_RADIUS2]))) + 0.5 * pl_len(mv);
  const double R = R0 + kPrimPad * (fabs(c[0] - g.c[0]) + fabs(c[1] - g.c[1]) + fabs(c[2] - g.c[2]) + kSqrt3 * R0 + kSqrt3 * g.rho);
  double ax;
  if (!prim_cone_meets(k, c, R, &ax)) return false;
  float fb = static_cast<float>(ax);
  if (static_cast<double>(fb) > ax) fb = nextafterf(fb, -__builtin_huge_valf());
  *key = pl_u(fb);
  return true;
}

// list order: ascending bound, then index
__host__ __device__ inline bool prim_before(uint2 a, uint2 b) {
  const float fa = pl_f(a.y), fb = pl_f(b.y);
  return fa < fb || (fa == fb && a.x < b.x);
}

// Host form (rt_prim_lists; the device builds the same set breadth-first, prim_list_kernel): the list of tile
// `tile` into out (cap entries), returns its count or kPrimListNone.
inline uint32_t prim_list_build_host(const PrimListGeom &g, const uint32_t *nodes, uint32_t root, const uint32_t *prims,
                                     uint32_t tile, uint32_t cap, uint2 *out) {
  PrimCone k;
  if (!prim_cone(g, tile, &k)) return kPrimListNone;
  uint32_t n = 0;
  uint32_t stack[64];
  int sp = 0;
  stack[sp++] = root;
  while (sp > 0) {
    const uint32_t *nd = nodes + static_cast<size_t>(stack[--sp]) * kAccelNodeWords;
    for (int ch = 0; ch < 2; ++ch) {
      if (!prim_cone_child(k, g, nd, ch)) continue;
      const uint32_t ref = nd[12 + ch];
      if (!(ref & kAccelLeaf)) {
        if (sp >= 64) return kPrimListNone;
        stack[sp++] = ref;
        continue;
      }
      const uint32_t first = ref & 0xffffffu, cnt = ((ref >> 24) & 0x7fu) + 1u;
      for (uint32_t i = 0; i < cnt; ++i) {
        uint32_t key;
        if (!prim_cone_sphere(k, g, prims, first + i, &key)) continue;
        if (n >= cap) return kPrimListNone;
        const uint2 e = make_uint2(first + i, key);
        uint32_t j = n++;
        while (j > 0 && prim_before(e, out[j - 1])) { out[j] = out[j - 1]; --j; }
        out[j] = e;
      }
    }
  }
  return n;
}

}  // namespace rt
