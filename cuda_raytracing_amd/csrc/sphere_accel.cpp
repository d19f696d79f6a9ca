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

#include "accel_build.h"
#include "gpu_scene.h"

namespace rt {
namespace {

using accel::Box;
using accel::Builder;
using accel::Prim;
using accel::fb;
using accel::fl;

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
  uint32_t root = bd.build(0, static_cast<uint32_t>(bd.prims.size()), 1, &rb, &rm);
  if (root & kAccelLeaf) { if (why) *why = "degenerate tree"; return false; }
  // breadth-first node order (the top levels first: what RT_ACCEL_LDS_NODES stages in LDS);
  // RT_ACCEL_BFS=0 keeps the builder's depth-first order
  if (!(std::getenv("RT_ACCEL_BFS") && std::getenv("RT_ACCEL_BFS")[0] == '0')) root = bd.bfs_order(root);
  if (bd.nodes.size() / kAccelNodeWords >= 65536) { if (why) *why = "tree too large for u16 stack entries"; return false; }
  out->root = root;
  out->depth = bd.max_depth;
  out->wide_words = accel::collapse_wide(bd.nodes, root, &out->wide_depth);
  out->wide_stack = 3 * out->wide_depth + 1;
  if (out->wide_words.size() / kAccel4NodeWords >= 65536) out->wide_words.clear();   // u16 stack entries
  if (!out->wide_words.empty()) accel::quantize_wide(out->wide_words, &out->wide_q_words);
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
