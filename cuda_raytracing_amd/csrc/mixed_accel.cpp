// mixed_accel.cpp — SAH trees for the verified traversal of mixed worlds (MixedTraceK, device/rt_body.h).
//
// hit() (raytracing.cu:1079-1251) rotates and translates the ray IN PLACE when it enters a transform and
// back when it leaves (:1176-1237); the round trip is not exact, so every test after the first transform
// the walk enters sees a drifted ray, and which transforms the walk enters depends on the reference tree
// and its visit order.  A different tree cannot reproduce that.  But a subtree that holds no transform,
// or that the ray provably enters no transform of, leaves the ray untouched: there the record hit()
// returns is the closest acceptable primitive the reference walk reaches (ties aside), whatever the order.
// This file marks such subtrees ("macro roots") and builds a binned-SAH tree over each one's primitives:
//   static macro   a BVH / group node whose subtree holds no translate / rotate, below a node that does
//                  (or the root): every ray may take its SAH walk;
//   dynamic macro  a node with transforms below and at least kDynMinPrims transform-free primitives: a ray
//                  may take the SAH walk only if the reference's own slab test on the union of the boxes
//                  of the BVH nodes with a transform child below (W_XFBOX) fails — those nodes are then
//                  missed at their visit too (smaller box, smaller tmax, same ray), so no transform below
//                  is entered and the ray stays untouched throughout the subtree.
// Per primitive the SAH prim record keeps the box of its deepest reference BVH ancestor below the macro
// root, with which the kernel proves that the reference walk reaches the hit it found (MixedTraceK).
// The walk above the macro roots stays the reference's own DFS, transforms included.
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

constexpr uint32_t kDynMinPrims = 64;   // dynamic macros only where the SAH walk replaces a large subtree

struct Analysis {
  const SceneImage &img;
  std::vector<int8_t> tf;          // 1 = no translate / rotate below (memo; -1 unknown)
  std::vector<uint32_t> nprims;    // transform-free primitives below (chains excluded)
  std::vector<uint8_t> has_xf;     // a BVH node with a transform child below
  std::vector<float> xfbox;        // 6 per record
  bool ok = true;

  explicit Analysis(const SceneImage &i)
      : img(i), tf(i.node_count, -1), nprims(i.node_count, 0), has_xf(i.node_count, 0), xfbox(6 * i.node_count, 0.0f) {}
  const uint32_t *node(uint32_t r) const { return &img.words[static_cast<size_t>(r) * kNodeWords]; }
  static bool is_prim(uint32_t k) { return k == K_SPHERE || k == K_QUAD || k == K_TRIANGLE; }

  void grow_box(uint32_t r, const float *b) {
    float *x = &xfbox[6 * static_cast<size_t>(r)];
    if (!has_xf[r]) { std::memcpy(x, b, 6 * sizeof(float)); has_xf[r] = 1; return; }
    for (int a = 0; a < 3; ++a) { x[2 * a] = std::min(x[2 * a], b[2 * a]); x[2 * a + 1] = std::max(x[2 * a + 1], b[2 * a + 1]); }
  }

  // children of a BVH / group node as the reference pushes them (a span-1 leaf names one child twice)
  void children(uint32_t r, std::vector<uint32_t> *out) const {
    const uint32_t *w = node(r);
    out->clear();
    if (w[W_KIND] == K_BVH) {
      const uint32_t l = w[W_AUX] & 0xffffu, rr = w[W_AUX] >> 16;
      out->push_back(l);
      if (rr != l) out->push_back(rr);
    } else if (w[W_KIND] == K_GROUP) {
      for (uint32_t k = 0; k < w[W_COUNT]; ++k) out->push_back(static_cast<uint16_t>(w[W_AUX] + k));
    }
  }

  // post-order over the reachable records (iterative: the reference tree can be deep)
  void analyse(uint32_t root) {
    std::vector<std::pair<uint32_t, bool>> st{{root, false}};
    std::vector<uint32_t> ch;
    std::vector<uint8_t> done(img.node_count, 0);
    size_t guard = 0;
    while (!st.empty()) {
      if (++guard > 64u * img.node_count + 1024) { ok = false; return; }
      auto [r, expanded] = st.back();
      st.pop_back();
      if (done[r]) continue;
      const uint32_t k = node(r)[W_KIND];
      if (k == K_TRANSLATE || k == K_YROTATE) {   // a transform chain: never part of a macro
        tf[r] = 0; nprims[r] = 0; done[r] = 1;
        continue;
      }
      if (is_prim(k)) { tf[r] = 1; nprims[r] = 1; done[r] = 1; continue; }
      if (k != K_BVH && k != K_GROUP) { ok = false; return; }
      children(r, &ch);
      if (!expanded) {
        st.push_back({r, true});
        for (uint32_t c : ch) if (!done[c]) st.push_back({c, false});
        continue;
      }
      bool t = true;
      uint64_t n = 0;
      for (uint32_t c : ch) {
        t = t && tf[c] == 1;
        n += nprims[c];
        if (has_xf[c]) grow_box(r, &xfbox[6 * static_cast<size_t>(c)]);
        const uint32_t ck = node(c)[W_KIND];
        if (k == K_BVH && (ck == K_TRANSLATE || ck == K_YROTATE)) {
          float b[6];
          for (int q = 0; q < 6; ++q) b[q] = fl(node(r)[W_BOX + q]);
          grow_box(r, b);
        }
      }
      tf[r] = t ? 1 : 0;
      nprims[r] = static_cast<uint32_t>(std::min<uint64_t>(n, 0xffffffffu));
      done[r] = 1;
    }
  }
};

// the transform-free primitives of a macro root's subtree (transform chains skipped), each with its deepest
// BVH ancestor below the root; false if a primitive is reached twice (other than a span-1 leaf's double
// name) or has non-finite geometry
bool collect(const Analysis &an, uint32_t root, std::vector<Prim> *out) {
  struct Item { uint32_t r; uint32_t anc; };
  std::vector<Item> st;
  std::vector<uint32_t> ch;
  std::vector<uint32_t> seen;
  an.children(root, &ch);
  for (uint32_t c : ch) st.push_back({c, kMixNoGroup});
  while (!st.empty()) {
    const Item it = st.back();
    st.pop_back();
    const uint32_t *w = an.node(it.r);
    const uint32_t k = w[W_KIND];
    if (k == K_TRANSLATE || k == K_YROTATE) continue;
    if (k == K_BVH || k == K_GROUP) {
      an.children(it.r, &ch);
      const uint32_t anc = k == K_BVH ? it.r : it.anc;
      for (uint32_t c : ch) st.push_back({c, anc});
      if (st.size() > 4u * an.img.node_count + 64) return false;
      continue;
    }
    if (!Analysis::is_prim(k)) return false;
    seen.push_back(it.r);
    Prim p{};
    p.node = it.r;
    p.group = it.anc;
    if (it.anc != kMixNoGroup) {
      for (int q = 0; q < 6; ++q) p.vbox[q] = fl(an.node(it.anc)[W_BOX + q]);
    } else {
      for (int q = 0; q < 6; ++q) p.vbox[q] = (q & 1) ? std::numeric_limits<float>::infinity() : -std::numeric_limits<float>::infinity();
    }
    if (k == K_SPHERE) {
      double c0[3], mv[3], cn = 0, mn = 0;
      const double rad = std::sqrt(static_cast<double>(fl(w[W_RADIUS2])));
      for (int a = 0; a < 3; ++a) {
        c0[a] = fl(w[W_CENTER + a]);
        mv[a] = fl(w[W_MOTION + a]);
        const double e0 = c0[a], e1 = c0[a] + mv[a];
        const double slack = 1e-6 * (std::fabs(e0) + std::fabs(mv[a]) + rad) + 1e-30;
        p.lo[a] = std::min(e0, e1) - rad - slack;
        p.hi[a] = std::max(e0, e1) + rad + slack;
        cn += c0[a] * c0[a];
        mn += mv[a] * mv[a];
      }
      p.m = std::sqrt(cn) + std::sqrt(mn) + rad;
      if (!(rad > 0)) return false;
    } else {   // quad: q, q+u, q+v, q+u+v; triangle: q, q+u, q+v
      double q[3], u[3], v[3], qn = 0, un = 0, vn = 0;
      for (int a = 0; a < 3; ++a) {
        q[a] = fl(w[W_Q + a]); u[a] = fl(w[W_U + a]); v[a] = fl(w[W_V + a]);
        qn += q[a] * q[a]; un += u[a] * u[a]; vn += v[a] * v[a];
      }
      for (int a = 0; a < 3; ++a) {
        double lo = std::min({q[a], q[a] + u[a], q[a] + v[a]}), hi = std::max({q[a], q[a] + u[a], q[a] + v[a]});
        if (k == K_QUAD) { lo = std::min(lo, q[a] + u[a] + v[a]); hi = std::max(hi, q[a] + u[a] + v[a]); }
        const double slack = 1e-6 * (std::fabs(q[a]) + std::fabs(u[a]) + std::fabs(v[a])) + 1e-30;
        p.lo[a] = lo - slack;
        p.hi[a] = hi + slack;
      }
      p.m = std::sqrt(qn) + std::sqrt(un) + std::sqrt(vn);
    }
    for (int a = 0; a < 3; ++a) p.c[a] = 0.5 * (p.lo[a] + p.hi[a]);
    if (!std::isfinite(p.m)) return false;
    for (int a = 0; a < 3; ++a) if (!std::isfinite(p.lo[a]) || !std::isfinite(p.hi[a])) return false;
    out->push_back(p);
  }
  std::sort(seen.begin(), seen.end());
  return std::adjacent_find(seen.begin(), seen.end()) == seen.end();
}

}  // namespace

bool build_mixed_accel(SceneImage *img, MixedAccel *out, std::string *why) {
  *out = MixedAccel();
  Analysis an(*img);
  an.analyse(img->root);
  if (!an.ok) { if (why) *why = "unexpected record kind"; return false; }
  // macro roots: static (transform-free node below a node with transforms, or the root) and dynamic
  uint32_t dyn_min = kDynMinPrims;   // RT_MIX_DYN_MIN (A/B): primitives below a node for a dynamic macro
  if (const char *e = std::getenv("RT_MIX_DYN_MIN")) dyn_min = static_cast<uint32_t>(std::max(1, std::atoi(e)));
  std::vector<uint32_t> roots;
  std::vector<uint8_t> dyn;
  {
    std::vector<uint32_t> st{img->root}, ch;
    std::vector<uint8_t> vis(img->node_count, 0);
    while (!st.empty()) {
      const uint32_t r = st.back();
      st.pop_back();
      if (vis[r]) continue;
      vis[r] = 1;
      const uint32_t k = an.node(r)[W_KIND];
      if (k == K_TRANSLATE || k == K_YROTATE) { st.push_back(an.node(r)[W_AUX]); continue; }
      if (k != K_BVH && k != K_GROUP) continue;
      if (an.tf[r] == 1) { roots.push_back(r); dyn.push_back(0); continue; }   // static: whole subtree
      if (an.nprims[r] >= dyn_min && an.has_xf[r]) { roots.push_back(r); dyn.push_back(1); }
      an.children(r, &ch);
      for (uint32_t c : ch) st.push_back(c);
    }
  }
  Builder bd;
  bd.kMaxLeaf = 4;
  if (const char *e = std::getenv("RT_MIX_LEAF")) bd.kMaxLeaf = static_cast<uint32_t>(std::max(1, std::min(64, std::atoi(e))));
  std::vector<uint32_t> macro_word(img->node_count, 0);
  for (size_t m = 0; m < roots.size(); ++m) {
    std::vector<Prim> prims;
    if (!collect(an, roots[m], &prims) || prims.empty()) continue;
    if (bd.prims.size() + prims.size() >= (1u << 24)) break;
    const uint32_t b = static_cast<uint32_t>(bd.prims.size());
    bd.prims.insert(bd.prims.end(), prims.begin(), prims.end());
    Box box;
    double mm;
    uint32_t ref = bd.build(b, static_cast<uint32_t>(bd.prims.size()), 1, &box, &mm);
    if (ref & kAccelLeaf) {   // one leaf: wrap it in a node whose second child is an empty box
      const uint32_t idx = static_cast<uint32_t>(bd.nodes.size() / kAccelNodeWords);
      bd.nodes.resize(bd.nodes.size() + kAccelNodeWords, 0);
      uint32_t *w = &bd.nodes[static_cast<size_t>(idx) * kAccelNodeWords];
      const double pad = static_cast<double>(kAccelKappa) * mm;
      w[0] = fb(accel::down(box.lo[0] - pad)); w[1] = fb(accel::up(box.hi[0] + pad));
      w[2] = fb(accel::down(box.lo[1] - pad)); w[3] = fb(accel::up(box.hi[1] + pad));
      w[4] = fb(accel::down(box.lo[2] - pad)); w[5] = fb(accel::up(box.hi[2] + pad));
      const float inf = std::numeric_limits<float>::infinity();
      w[6] = fb(inf); w[7] = fb(-inf); w[8] = fb(inf); w[9] = fb(-inf); w[10] = fb(inf); w[11] = fb(-inf);
      w[12] = ref;
      w[13] = ref;   // never entered: its box is empty
      w[14] = fb(accel::up(mm));
      w[15] = 0;
      ref = idx;
    }
    if (ref > kMacroRootMask) break;
    macro_word[roots[m]] = (dyn[m] ? kMacroDynamic : kMacroStatic) | ref;
    out->macros++;
    out->dynamic += dyn[m];
  }
  if (out->macros == 0) { if (why) *why = "no transform-free subtree"; return false; }
  if (bd.nodes.size() / kAccelNodeWords >= 65536) { if (why) *why = "SAH trees too large for u16 stack entries"; return false; }
  // transform chains ending in a primitive: one fused step in the kernel (W_MACRO of the chain's head); a
  // chain ending in a sphere also carries the sphere's words (and the rotation's sin / cos) in the head's
  // unused words 5..11 and 13..19 (kChainPacked, rt_layout.h).  RT_MIX_PACK=0 (A/B) keeps the loads.
  const char *pk_env = std::getenv("RT_MIX_PACK");
  const bool pack = !(pk_env && pk_env[0] == '0');
  for (uint32_t r = 0; r < img->node_count; ++r) {
    uint32_t *w = &img->words[static_cast<size_t>(r) * kNodeWords];
    if (w[W_KIND] != K_TRANSLATE && w[W_KIND] != K_YROTATE) continue;   // words 5..19 unused by both
    const uint32_t c = w[W_AUX];
    if (c >= img->node_count) continue;
    const uint32_t ck = an.node(c)[W_KIND];
    uint32_t prim = ~0u, rot = ~0u;
    if (Analysis::is_prim(ck)) {
      prim = c;
      if (w[W_KIND] == K_YROTATE) rot = r;
    } else if (w[W_KIND] == K_TRANSLATE && ck == K_YROTATE) {
      const uint32_t g = an.node(c)[W_AUX];
      if (g < img->node_count && Analysis::is_prim(an.node(g)[W_KIND])) { prim = g; rot = c; }
    }
    if (prim == ~0u || prim > kChainPrimMask) continue;
    uint32_t mw = kChainFused | (w[W_KIND] == K_TRANSLATE && rot != ~0u ? kChainRotate : 0u) | prim;
    const uint32_t *pw = an.node(prim);
    if (pack && pw[W_KIND] == K_SPHERE) {
      for (int j = 0; j < 3; ++j) w[W_PK_SPHERE0 + j] = pw[1 + j];
      for (int j = 0; j < 4; ++j) w[W_PK_SPHERE4 + j] = pw[4 + j];
      for (int j = 0; j < 4; ++j) w[W_PK_SPHERE8 + j] = pw[8 + j];
      if (rot != ~0u) { w[W_PK_SIN] = an.node(rot)[W_SIN]; w[W_PK_COS] = an.node(rot)[W_COS]; }
      mw |= kChainPacked;
      out->packed++;
    }
    w[W_MACRO] = mw;
  }
  for (uint32_t r = 0; r < img->node_count; ++r) {
    uint32_t *w = &img->words[static_cast<size_t>(r) * kNodeWords];
    if (w[W_KIND] != K_BVH && w[W_KIND] != K_GROUP) continue;   // primitives use words 12..19
    w[W_MACRO] = macro_word[r];
    if (macro_word[r] & kMacroDynamic)
      for (int q = 0; q < 6; ++q) w[W_XFBOX + q] = fb(an.xfbox[6 * static_cast<size_t>(r) + q]);
  }
  out->node_words = bd.nodes;
  out->depth = bd.max_depth + 1;
  out->prims = static_cast<uint32_t>(bd.order.size());
  out->prim_words.assign(static_cast<size_t>(bd.order.size()) * kMixPrimWords, 0);
  for (size_t k = 0; k < bd.order.size(); ++k) {
    const Prim &p = bd.prims[bd.order[k]];
    const uint32_t *w = &img->words[static_cast<size_t>(p.node) * kNodeWords];
    uint32_t *o = &out->prim_words[k * kMixPrimWords];
    for (int j = 0; j < kNodeWords; ++j) o[j] = w[j];
    o[MP_GROUP] = p.group;
    for (int j = 0; j < 6; ++j) o[MP_GBOX + j] = fb(p.vbox[j]);
    o[MP_RECORD] = p.node;
  }
  return true;
}

}  // namespace rt
