// scene_codegen.cpp — expand one scene's hit() DFS into straight-line HIP (the StaticTrace policy).
//
// hit() (raytracing.cu:1079-1251) runs a stack machine whose push order is fixed by the scene: a hit
// BVH node pushes right then left, a group pushes its children in index order, a transform pushes
// itself (cleanup marker) then its child.  With no transform nested inside a transform of the same
// kind (compile_scene rejects that: the reference itself loops forever there), every pop sequence is
// the pre-order walk
//     BVH  : if (box hit with the current tmax) { walk(left); walk(right); }
//     group: walk(child n-1) ... walk(child 0)
//     T / R: enter (was_last = 0, move the ray); walk(child); cleanup (move back, fix the record)
//     leaf : primitive test (sets was_last when inside a transform)
// so the whole traversal of a small scene can be emitted as nested ifs with every node constant as an
// immediate: no stack, no node loads, no kind dispatch, and per-visit work identical to the generic
// kernels (the same planar_hit / sphere_hit / box_hit / transform helpers of device/rt_body.h).
//
// Exact constant folding (the "folded" copy of the traversal).  With node data known, many products
// in the quad/triangle test multiply by +-0 or +-1 (axis-aligned normals, edges, origins).  Only
// rewrites that give bit-identical results are applied:
//   x * 1 -> x,  x * -1 -> -x,  x - (+0) -> x          exact for every x;
//   a + x*(+-0), a - x*(+-0) -> a                      exact for FINITE x, up to the sign of a zero
//                                                      result (a left-to-right sum that drops +-0
//                                                      terms equals the original except that a zero
//                                                      result may differ in sign);
// and every folded value only feeds zero-sign-insensitive consumers: |denom| >= eps, t = num/denom
// (a zero num gives t = +-0 < tmin either way), the inside compares, front = denom < 0, and — only
// when no image texture reads u,v — alpha/beta stored as h.u/h.v.  Sphere centres with zero motion
// fold to constants (time is in (0,1], so mv*time == mv for mv = +-0).  Finiteness: the folded copy
// is used only when every ray has |o|,|d| <= 1e9 at traversal start; with the scene's constants bounded by 1e6 (checked here, else no folding) every
// dropped factor (d, o, p - q, the edge cross products) stays finite through <= 2 transform levels.
// The host decides per render whether every ray is bounded (rt_capi.cpp ray_bound()); the kernel
// double-checks each traversal and flags violations (the frame is then re-rendered unfolded).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gpu_scene.h"

namespace rt {
namespace {

// an emitted scalar expression; zero = the value is +-0 (sign unknown, only in folded code)
struct E {
  std::string s;
  bool zero = false;
};

struct Gen {
  const SceneImage &img;
  uint32_t budget;
  bool fold = false;          // emit the folded copy
  bool fold_uv = false;       // alpha/beta may be folded too (no image texture reads u,v)
  std::string out;
  uint32_t visits = 0;
  int indent = 4;
  bool ok = true;
  uint32_t uid = 0;
  // lazy 1/dir: the reference recomputes 1/dir in every aabb_hit from the current ray; the kernels
  // cache it in T.inv.  Here it is (re)computed only before a box test that follows a direction change
  // (start, y-rotation enter/exit), instead of at every rotation — same values, fewer divisions.
  bool inv_fresh = false;
  // per-axis reciprocals (T.rcp) of the current direction: a folded axis-aligned plane needs only its
  // own, so after a rotation the planes refresh one axis each (3 ops) instead of the whole dir_rcp
  // (three reciprocals, three 1/dir divisions and the exactness check); inv_fresh implies all three
  bool rcp_fresh[3] = {false, false, false};
  // A/B knobs: RT_JIT_FASTDIV=0 keeps the compiler's division in the folded copy; RT_JIT_SHARE_RCP=0
  // gives every axis-aligned plane its own reciprocal instead of the direction's shared one
  bool fast_div = !(std::getenv("RT_JIT_FASTDIV") && std::getenv("RT_JIT_FASTDIV")[0] == '0');
  bool share_rcp = fast_div && !(std::getenv("RT_JIT_SHARE_RCP") && std::getenv("RT_JIT_SHARE_RCP")[0] == '0');
  std::vector<uint32_t> boxes_after;   // boxes_after[k]: visits reading 1/dir after pre-order visit k (pass 1)
  std::vector<uint8_t> kinds;          // pass 1: 1 if pre-order visit k (1-based) reads 1/dir
  bool collect = false;

  bool span1_primitive(const uint32_t *w) const {
    if ((w[W_AUX] & 0xffffu) != (w[W_AUX] >> 16) || (w[W_AUX] & 0xffffu) >= img.node_count) return false;
    const uint32_t ck = node(w[W_AUX] & 0xffffu)[W_KIND];
    return ck == K_SPHERE || ck == K_QUAD || ck == K_TRIANGLE;
  }
  void need_inv() {
    if (inv_fresh) return;
    // folded copy: 1/dir and the per-axis reciprocals the axis-aligned planes divide by (exact under
    // the folded copy's ray bound, see rcp_ref / div_ref in device/rt_body.h)
    line(fold && fast_div ? "dir_rcp(T, r);" : "T.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);");
    inv_fresh = true;
    for (bool &b : rcp_fresh) b = fold && fast_div;
  }
  void need_rcp(int axis) {   // folded copy only (share_rcp): T.rcp.<axis> of the current direction
    if (rcp_fresh[axis]) return;
    const char *axn[3] = {"x", "y", "z"};
    line(std::string("T.rcp.") + axn[axis] + " = rcp_ref(r.d." + axn[axis] + ");");
    rcp_fresh[axis] = true;
  }
  void dir_changed() {
    inv_fresh = false;
    for (bool &b : rcp_fresh) b = false;
  }
  // folded copy: a plane whose normal is +-(unit axis) has denominator +-r.d.<axis>; returns the axis
  // (0..2, -1 otherwise) and whether the denominator is negated
  static int axis_den(const E &den, bool *neg) {
    const char *names[3] = {"r.d.x", "r.d.y", "r.d.z"};
    for (int a = 0; a < 3; ++a) {
      if (den.s == names[a]) { *neg = false; return a; }
      if (den.s == std::string("(-") + names[a] + ")") { *neg = true; return a; }
    }
    return -1;
  }
  bool needs_dir(const uint32_t *w) const {   // visit reads T.inv / T.rcp
    if (w[W_KIND] == K_BVH) return true;
    if (!fold || (w[W_KIND] != K_QUAD && w[W_KIND] != K_TRIANGLE)) return false;
    const E d[3] = {{"r.d.x"}, {"r.d.y"}, {"r.d.z"}};
    bool neg;
    return share_rcp && axis_den(dotc(w + W_NORMAL, d, true), &neg) >= 0;
  }
  bool boxes_later() const { return visits < boxes_after.size() && boxes_after[visits] > 0; }

  static bool is_zero(uint32_t b) { return (b & 0x7fffffffu) == 0; }
  // c * x (x a runtime value, finite in folded code)
  E term(const E &x, uint32_t cbits, bool fold_here) const {
    if (x.zero && fold_here) return E{"", true};
    if (fold_here && is_zero(cbits)) return E{"", true};
    if (fold_here && cbits == 0x3f800000u) return x;
    if (fold_here && cbits == 0xbf800000u) return E{"(-" + x.s + ")", false};
    return E{"(" + x.s + " * " + f(cbits) + ")", false};
  }
  static E sum(const E &a, const E &b) {
    if (a.zero) return b;
    if (b.zero) return a;
    return E{"(" + a.s + " + " + b.s + ")", false};
  }
  static E diff(const E &a, const E &b) {
    if (b.zero) return a;
    if (a.zero) return E{"(-" + b.s + ")", false};
    return E{"(" + a.s + " - " + b.s + ")", false};
  }
  static std::string val(const E &e) { return e.zero ? std::string("0.0f") : e.s; }
  // dot(c, x) = (c.x*x.x + c.y*x.y) + c.z*x.z with constant c (product order is immaterial)
  E dotc(const uint32_t *c, const E x[3], bool fold_here) const {
    return sum(sum(term(x[0], c[0], fold_here), term(x[1], c[1], fold_here)), term(x[2], c[2], fold_here));
  }

  // quad / triangle test (planar_hit in device/rt_body.h) with exact folding
  void planar_folded(const uint32_t *w, bool tri, bool in_xf, uint32_t i) {
    const std::string k = std::to_string(uid++);
    const E d[3] = {{"r.d.x"}, {"r.d.y"}, {"r.d.z"}}, o[3] = {{"r.o.x"}, {"r.o.y"}, {"r.o.z"}};
    const E den = dotc(w + W_NORMAL, d, true);
    const E non = dotc(w + W_NORMAL, o, true);
    line("{   // node " + u(i) + (tri ? " (triangle, folded)" : " (quad, folded)"));
    indent += 2;
    line("const float den" + k + " = " + val(den) + ";");
    // t for every lane (a tiny denominator only yields inf/NaN there), one branch for both tests
    // dd - x with dd = +-0 is -x up to the sign of a zero t (which fails the tmin test either way)
    const std::string num = is_zero(w[W_D]) ? "(-" + val(non) + ")" : "(" + f(w[W_D]) + " - " + val(non) + ")";
    // num / den without div_scale / div_fixup: in every lane where t matters (|den| >= 1e-8, t in
    // [tmin, tmax]) the folded copy's bounds (|o|, |d| <= 1e9, constants <= 1e6) put |den| in
    // [2^-27, 2^52] and |num| in [2^-37, 2^52], where that sequence is a/b bit for bit; elsewhere a
    // tiny numerator still gives |t| < tmin and a tiny denominator fails the |den| test, so every
    // predicate is unchanged.  Axis-aligned planes reuse the direction's reciprocal (x/(-b) == -(x/b)).
    bool neg = false;
    const int ax_d = axis_den(den, &neg);
    const char *axn[3] = {"x", "y", "z"};
    if (ax_d >= 0 && share_rcp) {
      need_rcp(ax_d);
      line("const float t" + k + " = " + (neg ? "-" : "") + "div_ref(" + num + ", r.d." + axn[ax_d] + ", T.rcp." +
           axn[ax_d] + ");");
    } else if (fast_div) {
      line("const float t" + k + " = div_ref(" + num + ", den" + k + ", rcp_ref(den" + k + "));");
    } else {
      line("const float t" + k + " = " + num + " / den" + k + ";");
    }
    line("if ((fabsf(den" + k + ") >= kDenomEps) & (kTmin <= t" + k + ") & (t" + k + " <= T.tmax)) {");
    indent += 2;
    line("const f3 p" + k + " = mk(r.o.x + r.d.x * t" + k + ", r.o.y + r.d.y * t" + k + ", r.o.z + r.d.z * t" + k + ");");
    const char *ax[3] = {"x", "y", "z"};
    E pq[3];
    for (int a = 0; a < 3; ++a) {
      const uint32_t qb = w[W_Q + a];
      pq[a] = E{qb == 0u ? "p" + k + "." + ax[a] : "(p" + k + "." + ax[a] + " - " + f(qb) + ")", false};
    }
    for (int a = 0; a < 3; ++a) line("const float q" + k + ax[a] + " = " + pq[a].s + ";");
    const E qv[3] = {{"q" + k + "x"}, {"q" + k + "y"}, {"q" + k + "z"}};
    const uint32_t *vv = w + W_V, *uu = w + W_U, *ww = w + W_W;
    const bool fa = fold_uv;
    // cross(pq, vv) and cross(uu, pq) as in rt_body.h cross()
    const E c1[3] = {diff(term(qv[1], vv[2], fa), term(qv[2], vv[1], fa)),
                     diff(term(qv[2], vv[0], fa), term(qv[0], vv[2], fa)),
                     diff(term(qv[0], vv[1], fa), term(qv[1], vv[0], fa))};
    const E c2[3] = {diff(term(qv[2], uu[1], fa), term(qv[1], uu[2], fa)),
                     diff(term(qv[0], uu[2], fa), term(qv[2], uu[0], fa)),
                     diff(term(qv[1], uu[0], fa), term(qv[0], uu[1], fa))};
    // the reference forms uu.y*pq.z - uu.z*pq.y: term() writes (pq.z * uu.y), the same product
    for (int a = 0; a < 3; ++a) {
      if (!c1[a].zero) line("const float a" + k + ax[a] + " = " + c1[a].s + ";");
      if (!c2[a].zero) line("const float b" + k + ax[a] + " = " + c2[a].s + ";");
    }
    E ca[3], cb[3];
    for (int a = 0; a < 3; ++a) {
      ca[a] = c1[a].zero ? E{"", true} : E{std::string("a") + k + ax[a], false};
      cb[a] = c2[a].zero ? E{"", true} : E{std::string("b") + k + ax[a], false};
    }
    const E al = dotc(ww, ca, fa), be = dotc(ww, cb, fa);
    line("const float al" + k + " = " + val(al) + ", be" + k + " = " + val(be) + ";");
    std::string in = "(0.0f <= al" + k + ") & (al" + k + " <= 1.0f) & (0.0f <= be" + k + ") & (be" + k + " <= 1.0f)";
    if (tri) in += " & (al" + k + " + be" + k + " <= 1.0f)";
    line("if (" + in + ") {");
    indent += 2;
    line("h.u = al" + k + "; h.v = be" + k + "; h.t = t" + k + "; h.p = p" + k + "; h.mat = " + u(w[W_AUX]) + ";");
    line("h.fd = den" + k + "; h.n = " + v3(w, W_NORMAL) + ";   // dot(dir, n) == denom bitwise (same products)");
    line(std::string("T.tmax = t") + k + ";" + (in_xf ? " T.was_last = 1;" : ""));
    indent -= 2;
    line("}");
    indent -= 2;
    line("}");
    indent -= 2;
    line("}");
  }

  const uint32_t *node(uint32_t i) const { return &img.words[static_cast<size_t>(i) * kNodeWords]; }
  static std::string f(uint32_t bits) {
    char b[48];
    std::snprintf(b, sizeof b, "__uint_as_float(0x%08xu)", bits);
    return b;
  }
  static std::string v3(const uint32_t *w, int k) { return "mk(" + f(w[k]) + ", " + f(w[k + 1]) + ", " + f(w[k + 2]) + ")"; }
  static std::string u(uint32_t x) { return std::to_string(x) + "u"; }
  void line(const std::string &s) {
    out.append(static_cast<size_t>(indent), ' ');
    out += s;
    out += '\n';
  }

  void walk(uint32_t i, bool in_t, bool in_r, int depth) {
    if (!ok) return;
    if (++visits > budget || depth > 256 || i >= img.node_count) { ok = false; return; }
    const uint32_t *w = node(i);
    if (collect) {
      if (kinds.size() <= visits) kinds.resize(visits + 1, 0);
      kinds[visits] = needs_dir(w) ? 1 : 0;
    }
    const std::string xf = (in_t || in_r) ? "true" : "false";
    switch (w[W_KIND]) {
      case K_BVH:
        if (span1_primitive(w)) {
          // span-1 leaf (both children the same sphere/quad/triangle, raytracing.cu:858-859): the second
          // test can never change the record (a sphere re-test rejects root1 == tmax and root2 >= root1;
          // a planar re-test rewrites identical values), so it is emitted once and counted twice
          line("if (COUNT) vc.k[" + u(K_BVH) + "]++;");
          need_inv();
          line("if (box_hit(T, r, " + f(w[W_BOX]) + ", " + f(w[W_BOX + 1]) + ", " + f(w[W_BOX + 2]) + ", " +
               f(w[W_BOX + 3]) + ", " + f(w[W_BOX + 4]) + ", " + f(w[W_BOX + 5]) + ")) {   // node " + u(i) +
               " (span 1)");
          indent += 2;
          line("if (COUNT) vc.k[" + u(node(w[W_AUX] & 0xffffu)[W_KIND]) + "]++;");
          walk(w[W_AUX] & 0xffffu, in_t, in_r, depth + 1);
          if (!inv_fresh && boxes_later()) need_inv();
          indent -= 2;
          line("}");
          break;
        }
        line("if (COUNT) vc.k[" + u(K_BVH) + "]++;");
        need_inv();
        line("if (box_hit(T, r, " + f(w[W_BOX]) + ", " + f(w[W_BOX + 1]) + ", " + f(w[W_BOX + 2]) + ", " +
             f(w[W_BOX + 3]) + ", " + f(w[W_BOX + 4]) + ", " + f(w[W_BOX + 5]) + ")) {   // node " + u(i));
        indent += 2;
        walk(w[W_AUX] & 0xffffu, in_t, in_r, depth + 1);
        walk(w[W_AUX] >> 16, in_t, in_r, depth + 1);
        if (!inv_fresh && boxes_later()) need_inv();   // leave the block with a valid 1/dir
        indent -= 2;
        line("}");
        break;
      case K_QUAD:
      case K_TRIANGLE:
        line("if (COUNT) vc.k[" + u(w[W_KIND]) + "]++;");
        if (fold) { planar_folded(w, w[W_KIND] == K_TRIANGLE, in_t || in_r, i); break; }
        line(std::string("planar_hit(T, r, h, ") + (w[W_KIND] == K_TRIANGLE ? "true" : "false") + ", " + u(w[W_AUX]) +
             ", " + v3(w, W_NORMAL) + ", " + f(w[W_D]) + ", " + v3(w, W_Q) + ", " + v3(w, W_U) + ", " + v3(w, W_V) +
             ", " + v3(w, W_W) + ", " + xf + ");   // node " + u(i));
        break;
      case K_SPHERE: {
        line("if (COUNT) vc.k[" + u(K_SPHERE) + "]++;");
        const uint32_t *mv = w + W_MOTION;
        if (fold && is_zero(mv[0]) && is_zero(mv[1]) && is_zero(mv[2])) {
          // centre(t) = c + mv*t with mv = +-0 and t in (0,1]: exactly c + mv (float add, sign rules)
          uint32_t cb[3];
          for (int a = 0; a < 3; ++a) {
            float c, m, r;
            std::memcpy(&c, &w[W_CENTER + a], 4);
            std::memcpy(&m, &mv[a], 4);
            r = c + m;
            std::memcpy(&cb[a], &r, 4);
          }
          line("sphere_hit_static<UV>(T, r, h, " + u(w[W_AUX]) + ", mk(" + f(cb[0]) + ", " + f(cb[1]) + ", " + f(cb[2]) +
               "), " + f(w[W_RADIUS2]) + ", " + f(w[W_INV_RADIUS]) + ", " + xf + ");   // node " + u(i) + " (folded)");
          break;
        }
        line("sphere_hit<UV>(T, r, h, " + u(w[W_AUX]) + ", " + v3(w, W_CENTER) + ", " + v3(w, W_MOTION) + ", " +
             f(w[W_RADIUS2]) + ", " + f(w[W_INV_RADIUS]) + ", " + xf + ");   // node " + u(i));
        break;
      }
      case K_TRANSLATE:
        if (in_t) { ok = false; return; }
        line("if (COUNT) vc.k[" + u(K_TRANSLATE) + "]++;");
        line("translate_enter(T, r, " + v3(w, W_OFFSET) + ");   // node " + u(i));
        walk(w[W_AUX], true, in_r, depth + 1);
        line("if (COUNT) vc.k[" + u(K_TRANSLATE) + "]++;");
        line("translate_exit(T, r, h, " + v3(w, W_OFFSET) + ");");
        break;
      case K_YROTATE:
        if (in_r) { ok = false; return; }
        line("if (COUNT) vc.k[" + u(K_YROTATE) + "]++;");
        line("rotate_enter_dir(T, r, " + f(w[W_SIN]) + ", " + f(w[W_COS]) + ");   // node " + u(i));
        dir_changed();
        walk(w[W_AUX], in_t, true, depth + 1);
        line("if (COUNT) vc.k[" + u(K_YROTATE) + "]++;");
        line("rotate_exit_dir(T, r, h, " + f(w[W_SIN]) + ", " + f(w[W_COS]) + ");");
        dir_changed();
        break;
      case K_GROUP:
        line("if (COUNT) vc.k[" + u(K_GROUP) + "]++;");
        for (uint32_t k = w[W_COUNT]; k-- > 0;) walk(static_cast<uint16_t>(w[W_AUX] + k), in_t, in_r, depth + 1);
        break;
      default:
        ok = false;
    }
  }
};

}  // namespace

// Scene constants small enough for the finiteness argument of the folded copy (header comment).
bool foldable(const SceneImage &img) {
  auto small = [](uint32_t b) {
    float x;
    std::memcpy(&x, &b, 4);
    return std::fabs(x) <= 1.0e6f;   // false for inf / NaN
  };
  for (uint32_t i = 0; i < img.node_count; ++i) {
    const uint32_t *w = &img.words[static_cast<size_t>(i) * kNodeWords];
    if (w[W_KIND] == K_QUAD || w[W_KIND] == K_TRIANGLE) {
      for (int k = W_NORMAL; k < W_W; ++k) if (!small(w[k])) return false;
      for (int k = W_W; k < W_W + 3; ++k) {
        float x;
        std::memcpy(&x, &w[k], 4);
        if (!std::isfinite(x)) return false;
      }
    } else if (w[W_KIND] == K_TRANSLATE) {
      for (int k = 0; k < 3; ++k) if (!small(w[W_OFFSET + k])) return false;
    }
  }
  return true;
}

bool generate_static_trace(const SceneImage &img, uint32_t max_visits, bool fold, std::string *src, uint32_t *visits,
                           bool *folded) {
  fold = fold && foldable(img);
  Gen g1{img, max_visits};   // pass 1: pre-order visits that read 1/dir (for the lazy 1/dir)
  g1.collect = true;
  g1.fold = fold;
  g1.walk(img.root, false, false, 0);
  if (!g1.ok) {
    if (visits) *visits = g1.visits;
    return false;
  }
  Gen g{img, max_visits};
  g.boxes_after.assign(g1.kinds.size() + 1, 0);
  for (size_t k = g1.kinds.size(); k-- > 0;)
    g.boxes_after[k] = g.boxes_after[k + 1] + (k + 1 < g1.kinds.size() && g1.kinds[k + 1] ? 1u : 0u);
  g.fold = fold;
  g.fold_uv = fold && !img.needs_uv;
  g.walk(img.root, false, false, 0);
  if (visits) *visits = g.visits;
  if (folded) *folded = fold;
  if (!g.ok) return false;
  src->clear();
  *src += "struct StaticTrace {\n";
  *src += "  static constexpr bool kCarryPoint = true;   // render_body keeps the viewport point per pixel\n";
  *src += "  template <bool LDS, bool COUNT, bool UV>\n";
  *src += "  __device__ __forceinline__ static void run(const Mem<LDS> &, const RenderArgs &A, bool busy, uint64_t,\n";
  *src += "                                             uint32_t, uint16_t *, Trav &T, Ray &r, Hit &h, Visits &vc) {\n";
  *src += "    if (!busy) return;\n";
  *src += "    trav_reset_dir(T);\n";
  if (fold) {
    // the host enables folding only when it can bound every ray by 1e6 (camera + scene box + materials);
    // a lane that ever sees a larger or non-finite ray flags the frame, which the host then re-renders
    // without folding (rt_context_timing), so a wrong bound can cost time but never change a frame
    // RT_FOLD_CHECK_BOUND (tests only) lowers the flag threshold so that a violation can be forced
    std::string kb = "1.0e9f";
    if (const char *e = std::getenv("RT_FOLD_CHECK_BOUND")) {
      char buf[64];
      std::snprintf(buf, sizeof buf, "%.9gf", std::atof(e));
      kb = buf;
    }
    *src += "    const float kB = " + kb + ";\n";
    *src += "    const bool small = (fabsf(r.o.x) <= kB) & (fabsf(r.o.y) <= kB) & (fabsf(r.o.z) <= kB) &\n";
    *src += "                       (fabsf(r.d.x) <= kB) & (fabsf(r.d.y) <= kB) & (fabsf(r.d.z) <= kB);\n";
    *src += "    if (!small) atomicOr(A.fold_violation, 1u);\n";
  }
  *src += g.out;
  // every accepted hit has a finite t (planar: |denom| >= 1e-8, finite numerator; sphere: root < tmax),
  // so "some hit" is exactly "tmax left +inf" — no per-hit flag to merge across the nested ifs
  *src += "    T.result = T.tmax != __builtin_huge_valf();\n";
  *src += "  }\n};\n";
  return true;
}

}  // namespace rt
