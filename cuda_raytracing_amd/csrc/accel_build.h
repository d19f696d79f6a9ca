// accel_build.h — binned-SAH BVH2 builder shared by the verified traversals (sphere_accel.cpp,
// mixed_accel.cpp).  Node layout: device/rt_layout.h kAccel*: child boxes pre-padded by the subtree's
// share of the conservative padding (kAccelKappa * M), child refs, per-child M.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "device/rt_layout.h"

namespace rt {
namespace accel {

inline float fl(uint32_t b) { float f; std::memcpy(&f, &b, 4); return f; }
inline uint32_t fb(float f) { uint32_t b; std::memcpy(&b, &f, 4); return b; }

struct Prim {
  double lo[3], hi[3], c[3];   // padded bounds (over the motion for spheres), centroid
  double m;                    // bounds |point| over the primitive (sphere: |c0| + |mv| + r)
  uint32_t node;               // reference record
  float vbox[6];               // deepest reference BVH ancestor box (x0 x1 y0 y1 z0 z1)
  uint32_t group = 0xffffffffu;   // that ancestor's record (mixed walk), ~0u: none below the macro root
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

  // renumber the internal nodes breadth-first from `root` (which becomes node 0), so that the top levels
  // of the tree are the first nodes: a prefix of the array is a complete top of the tree (the part a
  // kernel can stage in LDS); leaf references are unchanged
  uint32_t bfs_order(uint32_t root) {
    const uint32_t count = static_cast<uint32_t>(nodes.size() / kAccelNodeWords);
    std::vector<uint32_t> order_bfs, new_id(count, 0xffffffffu);
    order_bfs.reserve(count);
    order_bfs.push_back(root);
    new_id[root] = 0;
    for (size_t i = 0; i < order_bfs.size(); ++i) {
      const uint32_t *w = &nodes[static_cast<size_t>(order_bfs[i]) * kAccelNodeWords];
      for (int c = 0; c < 2; ++c) {
        const uint32_t ch = w[12 + c];
        if (ch & kAccelLeaf) continue;
        new_id[ch] = static_cast<uint32_t>(order_bfs.size());
        order_bfs.push_back(ch);
      }
    }
    std::vector<uint32_t> out(nodes.size());
    for (size_t i = 0; i < order_bfs.size(); ++i) {
      uint32_t *o = &out[i * kAccelNodeWords];
      std::memcpy(o, &nodes[static_cast<size_t>(order_bfs[i]) * kAccelNodeWords], kAccelNodeWords * 4);
      for (int c = 0; c < 2; ++c)
        if (!(o[12 + c] & kAccelLeaf)) o[12 + c] = new_id[o[12 + c]];
    }
    out.resize(order_bfs.size() * kAccelNodeWords);
    nodes.swap(out);
    return 0;
  }
};

// 4-wide nodes from a (breadth-first) BVH2 in the kAccelNodeWords layout: each wide node holds the subtrees
// reached from a BVH2 node by opening, twice, the internal child with the largest padded box surface.  The
// child boxes are the BVH2's own padded boxes (the culling of every sphere is unchanged: a wide child box is
// exactly the box the BVH2 walk would test at that subtree).  Wide nodes are numbered breadth-first from the
// root (node 0).  depth_out: levels of the wide tree.
inline std::vector<uint32_t> collapse_wide(const std::vector<uint32_t> &nodes, uint32_t root, uint32_t *depth_out) {
  auto area = [](const uint32_t *b) {
    const double dx = fl(b[1]) - fl(b[0]), dy = fl(b[3]) - fl(b[2]), dz = fl(b[5]) - fl(b[4]);
    return (dx >= 0 && dy >= 0 && dz >= 0) ? 2.0 * (dx * dy + dy * dz + dz * dx) : 0.0;
  };
  struct Kid { const uint32_t *box; uint32_t ref; };
  std::vector<uint32_t> out;
  std::vector<uint32_t> queue{root}, level{1};
  uint32_t depth = 0;
  for (size_t qi = 0; qi < queue.size(); ++qi) {
    const uint32_t *w = &nodes[static_cast<size_t>(queue[qi]) * kAccelNodeWords];
    depth = std::max(depth, level[qi]);
    std::vector<Kid> kids{{w, w[12]}, {w + 6, w[13]}};
    while (kids.size() < 4) {
      int open = -1;
      double best = -1.0;
      for (size_t i = 0; i < kids.size(); ++i)
        if (!(kids[i].ref & kAccelLeaf) && area(kids[i].box) > best) { best = area(kids[i].box); open = static_cast<int>(i); }
      if (open < 0) break;
      const uint32_t *cw = &nodes[static_cast<size_t>(kids[open].ref) * kAccelNodeWords];
      kids.erase(kids.begin() + open);
      kids.push_back({cw, cw[12]});
      kids.push_back({cw + 6, cw[13]});
    }
    const size_t base = out.size();
    out.resize(base + kAccel4NodeWords, 0);
    uint32_t *o = &out[base];
    for (int c = 0; c < 4; ++c) {
      for (int k = 0; k < 6; ++k)
        o[4 * k + c] = (k & 1) ? fb(-std::numeric_limits<float>::infinity()) : fb(std::numeric_limits<float>::infinity());
      o[kAccel4Ref + c] = 0;
    }
    for (size_t c = 0; c < kids.size(); ++c) {
      for (int k = 0; k < 6; ++k) o[4 * k + c] = kids[c].box[k];
      if (kids[c].ref & kAccelLeaf) {
        o[kAccel4Ref + c] = kids[c].ref;
      } else {
        o[kAccel4Ref + c] = static_cast<uint32_t>(queue.size());   // breadth-first numbering
        queue.push_back(kids[c].ref);
        level.push_back(level[qi] + 1);
      }
    }
  }
  *depth_out = depth;
  return out;
}

// Quantised 4-wide nodes (rt_layout.h kAccel4Q*) from collapse_wide's nodes, same numbering.  Per node and axis:
// the origin o = the valid children's lowest plane minus the rounding pad ep (= 2^-20 of the node's largest
// |plane| on the axis), rounded down to a float; the step 2^e the smallest power of two whose 255 steps reach the
// highest plane plus ep; each child plane rounded outward to a step (q_lo = floor, q_hi = ceil, checked in exact
// double arithmetic), so every decoded box contains its float box widened by ep.  Returns false (out cleared)
// when a step would leave the exponent range the kernel's scale 2^e / d tolerates (|e| <= 40).
inline bool quantize_wide(const std::vector<uint32_t> &wide, std::vector<uint32_t> *out) {
  const size_t n = wide.size() / kAccel4NodeWords;
  out->assign(n * kAccel4QNodeWords, 0u);
  for (size_t i = 0; i < n; ++i) {
    const uint32_t *w = &wide[i * kAccel4NodeWords];
    uint32_t *o = &(*out)[i * kAccel4QNodeWords];
    uint32_t valid = 0;
    for (int c = 0; c < 4; ++c) {
      bool ok = true;
      for (int a = 0; a < 3; ++a) ok = ok && fl(w[(2 * a) * 4 + c]) <= fl(w[(2 * a + 1) * 4 + c]);
      if (ok) valid |= 1u << c;
    }
    uint32_t meta = valid << 24;
    for (int a = 0; a < 3; ++a) {
      double lo = std::numeric_limits<double>::infinity(), hi = -lo;
      for (int c = 0; c < 4; ++c)
        if (valid >> c & 1u) { lo = std::min(lo, static_cast<double>(fl(w[(2 * a) * 4 + c]))); hi = std::max(hi, static_cast<double>(fl(w[(2 * a + 1) * 4 + c]))); }
      if (!valid) lo = hi = 0.0;
      if (!std::isfinite(lo) || !std::isfinite(hi)) { out->clear(); return false; }
      const double ep = std::max(std::fabs(lo), std::fabs(hi)) * 0x1p-20;
      float org = static_cast<float>(lo - ep);
      while (static_cast<double>(org) > lo - ep) org = std::nextafter(org, -std::numeric_limits<float>::infinity());
      const double ext = (hi + ep) - static_cast<double>(org);
      int e = ext > 0 ? static_cast<int>(std::ceil(std::log2(ext / 255.0))) : -40;
      e = std::max(e, -40);
      uint32_t qlo = 0, qhi = 0;
      for (;; ++e) {
        if (e > 40) { out->clear(); return false; }
        const double step = std::ldexp(1.0, e);
        bool fits = true;
        qlo = qhi = 0;
        for (int c = 0; c < 4 && fits; ++c) {
          uint32_t l = 255, h = 0;   // empty slot: never tested (valid mask)
          if (valid >> c & 1u) {
            const double clo = static_cast<double>(fl(w[(2 * a) * 4 + c])) - ep, chi = static_cast<double>(fl(w[(2 * a + 1) * 4 + c])) + ep;
            double ql = std::floor((clo - org) / step), qh = std::ceil((chi - org) / step);
            while (ql > 0 && org + ql * step > clo) ql -= 1;
            while (org + qh * step < chi) qh += 1;
            if (ql < 0 || qh > 255) { fits = false; break; }
            l = static_cast<uint32_t>(ql);
            h = static_cast<uint32_t>(qh);
          }
          qlo |= l << (8 * c);
          qhi |= h << (8 * c);
        }
        if (fits) break;
      }
      o[a] = fb(org);
      meta |= static_cast<uint32_t>(e + 127) << (8 * a);
      o[4 + 2 * a] = qlo;
      o[5 + 2 * a] = qhi;
    }
    o[3] = meta;
    for (int c = 0; c < 4; ++c) o[kAccel4QRef + c] = w[kAccel4Ref + c];
  }
  return true;
}

}  // namespace accel
}  // namespace rt
