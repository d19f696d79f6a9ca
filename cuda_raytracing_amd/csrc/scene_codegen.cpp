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
#include <cstdio>
#include <string>

#include "gpu_scene.h"

namespace rt {
namespace {

struct Gen {
  const SceneImage &img;
  uint32_t budget;
  std::string out;
  uint32_t visits = 0;
  int indent = 4;
  bool ok = true;

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
    const std::string xf = (in_t || in_r) ? "true" : "false";
    switch (w[W_KIND]) {
      case K_BVH:
        line("if (COUNT) vc.k[" + u(K_BVH) + "]++;");
        line("if (box_hit(T, r, " + f(w[W_BOX]) + ", " + f(w[W_BOX + 1]) + ", " + f(w[W_BOX + 2]) + ", " +
             f(w[W_BOX + 3]) + ", " + f(w[W_BOX + 4]) + ", " + f(w[W_BOX + 5]) + ")) {   // node " + u(i));
        indent += 2;
        walk(w[W_AUX] & 0xffffu, in_t, in_r, depth + 1);
        walk(w[W_AUX] >> 16, in_t, in_r, depth + 1);
        indent -= 2;
        line("}");
        break;
      case K_QUAD:
      case K_TRIANGLE:
        line("if (COUNT) vc.k[" + u(w[W_KIND]) + "]++;");
        line(std::string("planar_hit(T, r, h, ") + (w[W_KIND] == K_TRIANGLE ? "true" : "false") + ", " + u(w[W_AUX]) +
             ", " + v3(w, W_NORMAL) + ", " + f(w[W_D]) + ", " + v3(w, W_Q) + ", " + v3(w, W_U) + ", " + v3(w, W_V) +
             ", " + v3(w, W_W) + ", " + xf + ");   // node " + u(i));
        break;
      case K_SPHERE:
        line("if (COUNT) vc.k[" + u(K_SPHERE) + "]++;");
        line("sphere_hit<UV>(T, r, h, " + u(w[W_AUX]) + ", " + v3(w, W_CENTER) + ", " + v3(w, W_MOTION) + ", " +
             f(w[W_RADIUS2]) + ", " + f(w[W_INV_RADIUS]) + ", " + xf + ");   // node " + u(i));
        break;
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
        line("rotate_enter(T, r, " + f(w[W_SIN]) + ", " + f(w[W_COS]) + ");   // node " + u(i));
        walk(w[W_AUX], in_t, true, depth + 1);
        line("if (COUNT) vc.k[" + u(K_YROTATE) + "]++;");
        line("rotate_exit(T, r, h, " + f(w[W_SIN]) + ", " + f(w[W_COS]) + ");");
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

bool generate_static_trace(const SceneImage &img, uint32_t max_visits, std::string *src, uint32_t *visits) {
  Gen g{img, max_visits};
  g.walk(img.root, false, false, 0);
  if (visits) *visits = g.visits;
  if (!g.ok) return false;
  src->clear();
  *src += "struct StaticTrace {\n";
  *src += "  template <bool LDS, bool COUNT, bool UV>\n";
  *src += "  __device__ __forceinline__ static void run(const Mem<LDS> &, const RenderArgs &, bool busy, uint64_t,\n";
  *src += "                                             uint32_t, uint16_t *, Trav &T, Ray &r, Hit &h, Visits &vc) {\n";
  *src += "    if (!busy) return;\n";
  *src += "    trav_reset(T, r);\n";
  *src += g.out;
  *src += "  }\n};\n";
  return true;
}

}  // namespace rt
