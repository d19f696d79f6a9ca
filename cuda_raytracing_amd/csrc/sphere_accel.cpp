// sphere_accel.cpp — SAH BVH over the spheres of an all-sphere world, for the verified traversal.
//
// The reference builds its BVH by median splits on a random axis (raytracing.cu:842-871) and walks it
// depth-first, left child first (:1124-1130): on the 10k-sphere scene a ray visits ~70 nodes.  The
// closest hit does not depend on the tree (see AccelTraceK in device/rt_body.h for why, and for the
// exact conditions under which it can): this file builds a second, better tree over the same
// spheres — binned SAH, child boxes stored in the parent — plus, per sphere, the box the reference's
// own traversal must pass to reach it (its deepest BVH ancestor), which the kernel uses to prove that
// the reference would have reached the hit the fast tree found.
//
// Eligibility: every record reachable from the root is a BVH node, a group or a sphere, and every
// sphere is reached once (a span-1 leaf names it twice from one parent, :858-859: still one sphere).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "gpu_scene.h"

namespace rt {
namespace {

inline float fl(uint32_t b) { float f; std::memcpy(&f, &b, 4); return f; }
inline uint32_t fb(float f) { uint32_t b; std::memcpy(&b, &f, 4); return b; }

struct Prim {
  double lo[3], hi[3], c[3];   // padded bounds over the motion, centroid
  double m;                    // |c0| + |mv| + r: bounds |centre(t)| + r
  uint32_t node;               // reference record
  float vbox[6];               // deepest reference BVH ancestor box (x0 x1 y0 y1 z0 z1)
};

struct Box {
  double lo[3] = {std::numeric_limits<double>::infinity(), std::numeric_limits<double>::infinity(),
                  std::numeric_limits<double>::infinity()};
  double hi[3] = {-std::numeric_limits<double>::infinity(), -std::numeric_limits<double>::infinity(),
                  -std::numeric_limits<double>::infinity()};
  void grow(const double *l, const double *h) {
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], l[a]); hi[a] = std::max(hi[a], h[a]); }
  }
  double area() const {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

// float bounds that contain the double box (rounded outward)
inline float down(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
  return f;
}
inline float up(double x) {
  float f = static_cast<float>(x);
  if (static_cast<double>(f) < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
  return f;
}

struct Builder {
  std::vector<Prim> prims;
  std::vector<uint32_t> nodes;   // kAccelNodeWords per node
  std::vector<uint32_t> order;   // prim order of the leaves
  uint32_t max_depth = 0;

  static constexpr int kBins = 16;
  // SAH constants (A/B knobs RT_ACCEL_LEAF = max spheres per leaf, RT_ACCEL_ISECT = sphere test cost
  // relative to a node visit)
  uint32_t kMaxLeaf = 4;
  double kTravCost = 1.0, kIsectCost = 1.5;

  // returns the child reference; fills its box and M
  uint32_t build(uint32_t b, uint32_t e, uint32_t depth, Box *box_out, double *m_out) {
    max_depth = std::max(max_depth, depth);
    Box bb, cb;
    double m = 0.0;
    for (uint32_t i = b; i < e; ++i) {
      bb.grow(prims[i].lo, prims[i].hi);
      cb.grow(prims[i].c, prims[i].c);
      m = std::max(m, prims[i].m);
    }
    *box_out = bb;
    *m_out = m;
    const uint32_t n = e - b;
    auto leaf = [&]() {
      const uint32_t first = static_cast<uint32_t>(order.size());
      for (uint32_t i = b; i < e; ++i) order.push_back(i);
      return kAccelLeaf | ((n - 1) << 24) | first;
    };
    if (n <= 1) return leaf();
    // binned SAH over centroids
    int best_axis = -1, best_split = -1;
    double best_cost = std::numeric_limits<double>::infinity();
    for (int a = 0; a < 3; ++a) {
      const double ext = cb.hi[a] - cb.lo[a];
      if (!(ext > 0)) continue;
      Box bin[kBins];
      uint32_t cnt[kBins] = {0};
      for (uint32_t i = b; i < e; ++i) {
        int k = static_cast<int>((prims[i].c[a] - cb.lo[a]) / ext * kBins);
        k = std::min(std::max(k, 0), kBins - 1);
        bin[k].grow(prims[i].lo, prims[i].hi);
        cnt[k]++;
      }
      double right_area[kBins];
      uint32_t right_cnt[kBins];
      Box acc;
      uint32_t c = 0;
      for (int k = kBins - 1; k > 0; --k) {
        if (cnt[k]) acc.grow(bin[k].lo, bin[k].hi);
        c += cnt[k];
        right_area[k] = acc.area();
        right_cnt[k] = c;
      }
      Box lacc;
      uint32_t lc = 0;
      for (int k = 0; k < kBins - 1; ++k) {
        if (cnt[k]) lacc.grow(bin[k].lo, bin[k].hi);
        lc += cnt[k];
        if (lc == 0 || right_cnt[k + 1] == 0) continue;
        const double cost = lacc.area() * lc + right_area[k + 1] * right_cnt[k + 1];
        if (cost < best_cost) { best_cost = cost; best_axis = a; best_split = k; }
      }
    }
    const double parent_area = std::max(bb.area(), 1e-30);
    const double split_cost = kTravCost + kIsectCost * best_cost / parent_area;
    const double leaf_cost = kIsectCost * n;
    if (n <= kMaxLeaf && (best_axis < 0 || leaf_cost <= split_cost)) return leaf();
    uint32_t mid;
    if (best_axis >= 0) {
      const int a = best_axis;
      const double ext = cb.hi[a] - cb.lo[a];
      auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim &p) {
        int k = static_cast<int>((p.c[a] - cb.lo[a]) / ext * kBins);
        k = std::min(std::max(k, 0), kBins - 1);
        return k <= best_split;
      });
      mid = static_cast<uint32_t>(it - prims.begin());
    } else {
      mid = b + n / 2;   // coincident centroids: split the list
    }
    if (mid == b || mid == e) mid = b + n / 2;
    const uint32_t idx = static_cast<uint32_t>(nodes.size() / kAccelNodeWords);
    nodes.resize(nodes.size() + kAccelNodeWords, 0);
    Box lb, rb;
    double lm, rm;
    const uint32_t l = build(b, mid, depth + 1, &lb, &lm);
    const uint32_t r = build(mid, e, depth + 1, &rb, &rm);
    uint32_t *w = &nodes[static_cast<size_t>(idx) * kAccelNodeWords];
    const Box *cbx[2] = {&lb, &rb};
    const double mm[2] = {lm, rm};
    for (int c = 0; c < 2; ++c) {
      // stored pre-padded by the subtree's share of the cone padding, kAccelKappa * M (the ray's
      // share, kAccelKappa * |o|_1, is applied in t by the kernel)
      const double pad = static_cast<double>(kAccelKappa) * mm[c];
      uint32_t *o = w + 6 * c;
      o[0] = fb(down(cbx[c]->lo[0] - pad)); o[1] = fb(up(cbx[c]->hi[0] + pad));
      o[2] = fb(down(cbx[c]->lo[1] - pad)); o[3] = fb(up(cbx[c]->hi[1] + pad));
      o[4] = fb(down(cbx[c]->lo[2] - pad)); o[5] = fb(up(cbx[c]->hi[2] + pad));
    }
    w[12] = l;
    w[13] = r;
    w[14] = fb(up(lm));
    w[15] = fb(up(rm));
    return idx;
  }
};

struct Walker {
  const SceneImage &img;
  std::vector<int> seen_parent;   // sphere record -> parent BVH record that reached it (-2: none yet)
  std::vector<Prim> *prims;
  bool ok = true;

  const uint32_t *node(uint32_t i) const { return &img.words[static_cast<size_t>(i) * kNodeWords]; }

  void walk(uint32_t i, int bvh_parent, int depth) {
    if (!ok) return;
    if (depth > 256 || i >= img.node_count) { ok = false; return; }
    const uint32_t *w = node(i);
    switch (w[W_KIND]) {
      case K_BVH: {
        const uint32_t l = w[W_AUX] & 0xffffu, r = w[W_AUX] >> 16;
        // a span-1 leaf names its child twice (:858-859); the second walk of the same subtree can
        // never change the record (every sphere re-test meets root >= tmax), so it is walked once
        walk(l, static_cast<int>(i), depth + 1);
        if (r != l) walk(r, static_cast<int>(i), depth + 1);
      } break;
      case K_GROUP:
        for (uint32_t k = 0; k < w[W_COUNT]; ++k) walk(static_cast<uint16_t>(w[W_AUX] + k), bvh_parent, depth + 1);
        break;
      case K_SPHERE: {
        if (seen_parent[i] != -2) { ok = false; return; }   // reachable twice: keep the reference walk
        seen_parent[i] = bvh_parent;
        Prim p{};
        p.node = i;
        double c0[3], mv[3];
        for (int a = 0; a < 3; ++a) {
          c0[a] = fl(w[W_CENTER + a]);
          mv[a] = fl(w[W_MOTION + a]);
        }
        const double rad = std::sqrt(static_cast<double>(fl(w[W_RADIUS2])));
        double cn = 0, mn = 0;
        for (int a = 0; a < 3; ++a) {
          const double e0 = c0[a], e1 = c0[a] + mv[a];
          // centre(t) = c0 + t*mv is rounded per component: pad by a few ulps of the magnitudes
          const double slack = 1e-6 * (std::fabs(e0) + std::fabs(mv[a]) + rad) + 1e-30;
          p.lo[a] = std::min(e0, e1) - rad - slack;
          p.hi[a] = std::max(e0, e1) + rad + slack;
          p.c[a] = 0.5 * (p.lo[a] + p.hi[a]);
          cn += c0[a] * c0[a];
          mn += mv[a] * mv[a];
        }
        p.m = std::sqrt(cn) + std::sqrt(mn) + rad;
        if (!std::isfinite(p.m) || !(rad > 0)) { ok = false; return; }
        if (bvh_parent >= 0) {
          const uint32_t *pw = node(static_cast<uint32_t>(bvh_parent));
          for (int k = 0; k < 6; ++k) p.vbox[k] = fl(pw[W_BOX + k]);
        } else {
          for (int k = 0; k < 6; ++k)
            p.vbox[k] = (k & 1) ? std::numeric_limits<float>::infinity() : -std::numeric_limits<float>::infinity();
        }
        prims->push_back(p);
      } break;
      default:
        ok = false;
    }
  }
};

}  // namespace

bool build_sphere_accel(const SceneImage &img, uint32_t min_spheres, SphereAccel *out, std::string *why) {
  *out = SphereAccel();
  std::vector<Prim> prims;
  Walker wk{img, std::vector<int>(img.node_count, -2), &prims};
  wk.walk(img.root, -1, 0);
  if (!wk.ok) { if (why) *why = "world is not an all-sphere BVH/group tree"; return false; }
  if (prims.size() < min_spheres) { if (why) *why = "too few spheres"; return false; }
  if (prims.size() >= (1u << 24)) { if (why) *why = "too many spheres"; return false; }
  Builder bd;
  if (const char *e = std::getenv("RT_ACCEL_LEAF")) bd.kMaxLeaf = static_cast<uint32_t>(std::max(1, std::min(64, std::atoi(e))));
  if (const char *e = std::getenv("RT_ACCEL_ISECT")) bd.kIsectCost = std::max(0.05, std::atof(e));
  bd.prims = std::move(prims);
  Box rb;
  double rm;
  const uint32_t root = bd.build(0, static_cast<uint32_t>(bd.prims.size()), 1, &rb, &rm);
  if (root & kAccelLeaf) { if (why) *why = "degenerate tree"; return false; }
  if (bd.nodes.size() / kAccelNodeWords >= 65536) { if (why) *why = "tree too large for u16 stack entries"; return false; }
  out->root = root;
  out->depth = bd.max_depth;
  out->spheres = static_cast<uint32_t>(bd.order.size());
  out->node_words = bd.nodes;
  out->prim_words.assign(static_cast<size_t>(bd.order.size()) * kAccelPrimWords, 0);
  for (size_t k = 0; k < bd.order.size(); ++k) {
    const Prim &p = bd.prims[bd.order[k]];
    const uint32_t *w = &img.words[static_cast<size_t>(p.node) * kNodeWords];
    uint32_t *o = &out->prim_words[k * kAccelPrimWords];
    for (int a = 0; a < 3; ++a) { o[AP_CENTER + a] = w[W_CENTER + a]; o[AP_MOTION + a] = w[W_MOTION + a]; }
    o[AP_RADIUS2] = w[W_RADIUS2];
    o[AP_INV_RADIUS] = w[W_INV_RADIUS];
    o[AP_MAT] = w[W_AUX];
    o[AP_NODE] = p.node;
    for (int j = 0; j < 6; ++j) o[AP_VBOX + j] = fb(p.vbox[j]);
  }
  return true;
}

}  // namespace rt
