// scene_compile.cpp — reference scene bytes -> SceneImage (gpu_scene.h).
//
// Input contract: rt_scene (rt_render.h) = the reference's Hittable[] records, u16 WorldRef list
// and texture arena exactly as render() copies them to the GPU (raytracing.cu:1699-1733).
// Validation replaces the reference's unchecked accesses: every record kind, child index, WorldRef,
// texture offset and group range is checked, so malformed bytes are RT_ERR_SCENE instead of a
// device fault.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_map>

#include "gpu_scene.h"
#include "rt_render.h"

namespace rt {
namespace {

inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

struct Compiler {
  const rt_scene *sc;
  SceneImage *img;
  std::vector<uint32_t> nodes, mats, texs, perlin, pixels;
  std::map<std::vector<uint32_t>, uint32_t> mat_index;
  std::unordered_map<uint64_t, uint32_t> tex_index;       // arena offset -> texture index
  std::unordered_map<uint64_t, uint32_t> perlin_index;    // arena offset -> table index
  std::vector<int32_t> need_memo;
  int status = RT_OK;

  bool read_tex(uint64_t off, rtr_texture *t) {
    if (off > sc->texture_bytes || sc->texture_bytes - off < sizeof(rtr_texture)) return false;
    std::memcpy(t, sc->textures + off, sizeof *t);
    return true;
  }

  // texture at arena offset -> index (checker children first; cycles rejected)
  int64_t texture(uint64_t off, int depth) {
    auto it = tex_index.find(off);
    if (it != tex_index.end()) return it->second;
    if (depth > 32) return -1;
    rtr_texture t;
    if (!read_tex(off, &t)) return -1;
    uint32_t w[kTexWords] = {0};
    w[T_KIND] = t.kind;
    switch (t.kind) {
      case RTR_TEX_SOLID:
        w[T_RGB] = fbits(t.u.solid.x); w[T_RGB + 1] = fbits(t.u.solid.y); w[T_RGB + 2] = fbits(t.u.solid.z);
        break;
      case RTR_TEX_CHECKER: {
        int64_t e = texture(t.u.checker.even.offset, depth + 1);
        int64_t o = texture(t.u.checker.odd.offset, depth + 1);
        if (e < 0 || o < 0) return -1;
        w[T_EVEN] = static_cast<uint32_t>(e); w[T_ODD] = static_cast<uint32_t>(o);
        w[T_INV_SCALE] = fbits(t.u.checker.inv_scale);
      } break;
      case RTR_TEX_IMAGE: {
        w[T_WIDTH] = static_cast<uint32_t>(t.u.image.width);
        w[T_HEIGHT] = static_cast<uint32_t>(t.u.image.height);
        w[T_HAS_PIXELS] = t.u.image.host_pixels != 0;
        if (w[T_HAS_PIXELS]) {
          // the reference indexes the arena from pixels_offset with a clamp that admits x==width,
          // y==height (raytracing.cu:349-351); keep every arena byte from there on so such reads
          // see the same bytes, and zero past the arena end (as the oracle does).
          uint64_t po = t.u.image.pixels_offset;
          if (po > sc->texture_bytes) return -1;
          uint64_t n = (sc->texture_bytes - po) / 4;
          w[T_PIXELS] = static_cast<uint32_t>(pixels.size());
          size_t base = pixels.size();
          pixels.resize(base + n);
          if (n) std::memcpy(pixels.data() + base, sc->textures + po, n * 4);
          img->needs_uv = true;
        }
      } break;
      case RTR_TEX_NOISE: {
        uint64_t po = t.u.noise.table_offset;
        if (po > sc->texture_bytes || sc->texture_bytes - po < sizeof(rtr_perlin)) return -1;
        auto pit = perlin_index.find(po);
        uint32_t pidx;
        if (pit != perlin_index.end()) {
          pidx = pit->second;
        } else {
          rtr_perlin p;
          std::memcpy(&p, sc->textures + po, sizeof p);
          pidx = static_cast<uint32_t>(perlin.size() / kPerlinWords);
          size_t base = perlin.size();
          perlin.resize(base + kPerlinWords, 0);
          for (int i = 0; i < RTR_PERLIN_POINTS; ++i) {
            perlin[base + 4 * i + 0] = fbits(p.gradients[i].x);
            perlin[base + 4 * i + 1] = fbits(p.gradients[i].y);
            perlin[base + 4 * i + 2] = fbits(p.gradients[i].z);
          }
          uint8_t *perm = reinterpret_cast<uint8_t *>(perlin.data() + base + kPerlinPermWord);
          uint16_t *perm2 = reinterpret_cast<uint16_t *>(perlin.data() + base + kPerlinPerm2Word);
          for (int i = 0; i < RTR_PERLIN_POINTS; ++i) {
            if (p.perm_x[i] < 0 || p.perm_x[i] > 255) return -1;   // the gather index must stay in the table
            perm[i] = static_cast<uint8_t>(p.perm_x[i]);
          }
          for (int i = 0; i < RTR_PERLIN_POINTS; ++i)
            perm2[i] = static_cast<uint16_t>(perm[i] | (perm[(i + 1) & 255] << 8));
          perlin_index[po] = pidx;
        }
        w[T_PERLIN] = pidx;
        w[T_NOISE_SCALE] = fbits(t.u.noise.scale);
        img->has_noise = true;
      } break;
      default:
        return -1;
    }
    uint32_t idx = static_cast<uint32_t>(texs.size() / kTexWords);
    texs.insert(texs.end(), w, w + kTexWords);
    tex_index[off] = idx;
    return idx;
  }

  int64_t material(const rtr_material &m) {
    uint32_t w[kMatWords] = {0};
    w[M_KIND] = m.kind;
    switch (m.kind) {
      case RTR_MAT_LAMBERTIAN:
      case RTR_MAT_DIFFUSE_LIGHT: {
        int64_t t = texture(m.u.lambert_tex.offset, 0);
        if (t < 0) return -1;
        w[M_TEX] = static_cast<uint32_t>(t);
      } break;
      case RTR_MAT_METAL:
        w[M_ALBEDO] = fbits(m.u.metal.albedo.x); w[M_ALBEDO + 1] = fbits(m.u.metal.albedo.y);
        w[M_ALBEDO + 2] = fbits(m.u.metal.albedo.z); w[M_FUZZ] = fbits(m.u.metal.fuzz);
        break;
      case RTR_MAT_DIELECTRIC:
        w[M_IOR] = fbits(m.u.dielectric.ior);
        break;
      default:
        // unknown kinds neither emit nor scatter in the reference (switch without default case)
        break;
    }
    std::vector<uint32_t> key(w, w + kMatWords);
    auto it = mat_index.find(key);
    if (it != mat_index.end()) return it->second;
    uint32_t idx = static_cast<uint32_t>(mats.size() / kMatWords);
    mats.insert(mats.end(), w, w + kMatWords);
    mat_index.emplace(std::move(key), idx);
    return idx;
  }

  bool href_of(uint16_t wref, uint32_t *out) const {   // wref_to_href (raytracing.cu:243-246)
    if (wref >= sc->ref_count) return false;
    uint16_t h = sc->refs[wref];
    if (h >= sc->hittable_count) return false;
    *out = h;
    return true;
  }

  bool node(uint32_t i) {
    const rtr_hittable &h = sc->hittables[i];
    uint32_t *w = &nodes[static_cast<size_t>(i) * kNodeWords];
    w[W_KIND] = h.kind;
    switch (h.kind) {
      case RTR_OBJ_SPHERE: {
        const rtr_sphere &s = h.u.sphere;
        int64_t m = material(s.mat);
        if (m < 0) return false;
        w[W_AUX] = static_cast<uint32_t>(m);
        w[W_CENTER] = fbits(s.center.x); w[W_CENTER + 1] = fbits(s.center.y); w[W_CENTER + 2] = fbits(s.center.z);
        w[W_MOTION] = fbits(s.motion.x); w[W_MOTION + 1] = fbits(s.motion.y); w[W_MOTION + 2] = fbits(s.motion.z);
        w[W_RADIUS] = fbits(s.radius);
        w[W_RADIUS2] = fbits(s.radius * s.radius);          // raytracing.cu:1099
        w[W_INV_RADIUS] = fbits(1.0f / s.radius);           // raytracing.cu:1112
      } break;
      case RTR_OBJ_BVH: {
        uint32_t l, r;
        if (!href_of(h.u.bvh.left, &l) || !href_of(h.u.bvh.right, &r)) return false;
        w[W_AUX] = l | (r << 16);
        const rtr_aabb &b = h.u.bvh.box;
        w[W_BOX + 0] = fbits(b.x0); w[W_BOX + 1] = fbits(b.x1); w[W_BOX + 2] = fbits(b.y0);
        w[W_BOX + 3] = fbits(b.y1); w[W_BOX + 4] = fbits(b.z0); w[W_BOX + 5] = fbits(b.z1);
      } break;
      case RTR_OBJ_TRIANGLE:
      case RTR_OBJ_QUAD: {
        const rtr_plane &g = h.u.planar.geom;
        int64_t m = material(h.u.planar.mat);
        if (m < 0) return false;
        w[W_AUX] = static_cast<uint32_t>(m);
        w[W_NORMAL] = fbits(g.normal.x); w[W_NORMAL + 1] = fbits(g.normal.y); w[W_NORMAL + 2] = fbits(g.normal.z);
        w[W_D] = fbits(g.d);
        w[W_Q] = fbits(g.q.x); w[W_Q + 1] = fbits(g.q.y); w[W_Q + 2] = fbits(g.q.z);
        w[W_U] = fbits(g.u.x); w[W_U + 1] = fbits(g.u.y); w[W_U + 2] = fbits(g.u.z);
        w[W_V] = fbits(g.v.x); w[W_V + 1] = fbits(g.v.y); w[W_V + 2] = fbits(g.v.z);
        w[W_W] = fbits(g.w.x); w[W_W + 1] = fbits(g.w.y); w[W_W + 2] = fbits(g.w.z);
      } break;
      case RTR_OBJ_TRANSLATE: {
        if (h.u.translate.child >= sc->hittable_count) return false;
        w[W_AUX] = h.u.translate.child;
        const rtr_vec3 &o = h.u.translate.offset;
        w[W_OFFSET] = fbits(o.x); w[W_OFFSET + 1] = fbits(o.y); w[W_OFFSET + 2] = fbits(o.z);
      } break;
      case RTR_OBJ_YROTATE: {
        if (h.u.yrotate.child >= sc->hittable_count) return false;
        w[W_AUX] = h.u.yrotate.child;
        w[W_SIN] = fbits(h.u.yrotate.sin_theta);
        w[W_COS] = fbits(h.u.yrotate.cos_theta);
      } break;
      case RTR_OBJ_GROUP: {
        const rtr_group &g = h.u.group;
        // children are pushed as u16 (first + i) (raytracing.cu:1243-1245)
        if (g.count > 65535u) return false;
        for (uint64_t k = 0; k < g.count; ++k)
          if (static_cast<uint16_t>(g.first + k) >= sc->hittable_count) return false;
        w[W_AUX] = g.first;
        w[W_COUNT] = static_cast<uint32_t>(g.count);
      } break;
      default:
        return false;
    }
    return true;
  }

  // No translation below a translation, no y-rotation below a y-rotation (see compile_scene).
  bool transforms_well_nested(uint32_t root) {
    // state per record: bit0 = reached under a translation, bit1 = under a rotation
    std::vector<uint8_t> seen(sc->hittable_count, 0xff);
    std::vector<std::pair<uint32_t, uint8_t>> work{{root, 0}};
    while (!work.empty()) {
      auto [i, ctx] = work.back();
      work.pop_back();
      if (seen[i] != 0xff && (seen[i] & ctx) == ctx) continue;
      seen[i] = seen[i] == 0xff ? ctx : static_cast<uint8_t>(seen[i] | ctx);
      const uint32_t *w = &nodes[static_cast<size_t>(i) * kNodeWords];
      switch (w[W_KIND]) {
        case K_BVH:
          work.push_back({w[W_AUX] & 0xffff, ctx});
          work.push_back({w[W_AUX] >> 16, ctx});
          break;
        case K_TRANSLATE:
          if (ctx & 1) return false;
          work.push_back({w[W_AUX], static_cast<uint8_t>(ctx | 1)});
          break;
        case K_YROTATE:
          if (ctx & 2) return false;
          work.push_back({w[W_AUX], static_cast<uint8_t>(ctx | 2)});
          break;
        case K_GROUP:
          for (uint32_t k = 0; k < w[W_COUNT]; ++k) work.push_back({static_cast<uint16_t>(w[W_AUX] + k), ctx});
          break;
        default:
          break;
      }
    }
    return true;
  }

  // Exact worst-case hit-stack depth of the DFS of raytracing.cu:1079-1251 starting at record i
  // (the record's own slot included).  -1 on a cycle / runaway depth.
  int32_t need(uint32_t i, int depth) {
    if (depth > 512) return -1;
    if (need_memo[i] == -2) return -1;         // on the current path: cycle
    if (need_memo[i] >= 0) return need_memo[i];
    need_memo[i] = -2;
    const uint32_t *w = &nodes[static_cast<size_t>(i) * kNodeWords];
    int32_t r = 1;
    switch (w[W_KIND]) {
      case K_BVH: {
        int32_t nl = need(w[W_AUX] & 0xffff, depth + 1), nr = need(w[W_AUX] >> 16, depth + 1);
        if (nl < 0 || nr < 0) { r = -1; break; }
        r = std::max(2, std::max(1 + nl, nr));
      } break;
      case K_TRANSLATE:
      case K_YROTATE: {
        int32_t nc = need(w[W_AUX], depth + 1);
        r = nc < 0 ? -1 : std::max(2, 1 + nc);
      } break;
      case K_GROUP: {
        uint32_t n = w[W_COUNT];
        r = std::max<int32_t>(1, static_cast<int32_t>(n));
        for (uint32_t k = 0; k < n && r >= 0; ++k) {
          int32_t nc = need(static_cast<uint16_t>(w[W_AUX] + k), depth + 1);
          if (nc < 0) r = -1;
          else r = std::max<int32_t>(r, static_cast<int32_t>(k) + nc);
        }
      } break;
      default:
        break;
    }
    need_memo[i] = r;
    return r;
  }
};

}  // namespace

int compile_scene(const void *scene_ptr, SceneImage *img) {
  const rt_scene *sc = static_cast<const rt_scene *>(scene_ptr);
  if (!sc || !img || !sc->hittables || !sc->refs || sc->hittable_count == 0 || sc->ref_count == 0 ||
      sc->hittable_count > 65536u || (sc->texture_bytes && !sc->textures))
    return RT_ERR_SCENE;
  *img = SceneImage();
  Compiler c;
  c.sc = sc;
  c.img = img;
  c.nodes.assign(static_cast<size_t>(sc->hittable_count) * kNodeWords, 0);
  for (uint32_t i = 0; i < sc->hittable_count; ++i)
    if (!c.node(i)) return RT_ERR_SCENE;
  uint32_t root;
  if (!c.href_of(sc->root, &root)) return RT_ERR_SCENE;
  c.need_memo.assign(sc->hittable_count, -1);
  int32_t need = c.need(root, 0);
  if (need < 0) return RT_ERR_SCENE;
  // hit() keeps ONE translation and ONE y-rotation cleanup counter per ray (raytracing.cu:1084-1085):
  // a translation reachable inside another translation's subtree (or a rotation inside a rotation)
  // is taken for the outer one's cleanup marker and the outer one re-enters forever.  The reference
  // hangs on such scenes; reject them instead of launching a kernel that never finishes.
  if (!c.transforms_well_nested(root)) return RT_ERR_UNSUPPORTED;

  img->node_count = sc->hittable_count;
  img->mat_count = static_cast<uint32_t>(c.mats.size() / kMatWords);
  img->tex_count = static_cast<uint32_t>(c.texs.size() / kTexWords);
  img->perlin_count = static_cast<uint32_t>(c.perlin.size() / kPerlinWords);
  img->root = root;
  img->stack_need = static_cast<uint32_t>(need);
  auto &W = img->words;
  W = c.nodes;
  // spheres whose material reads u,v (an image texture, raytracing.cu:332-351): the walk computes the
  // sphere's u,v only for these (get_sphere_uv's values are read by nothing else); RT_LAZY_UV=0 (A/B): all
  const char *lz = std::getenv("RT_LAZY_UV");
  const bool lazy_uv = !(lz && lz[0] == '0');
  // a texture reads u,v if it is an image or a checker with such a child anywhere below it (texture_color
  // follows the checker recursion down to the image, :366-384); depth-bounded like texture() (cycles were
  // rejected there, so the recursion ends)
  std::vector<int8_t> reads_uv(img->tex_count, -1);
  auto tex_reads_uv = [&](auto &&self, uint32_t ti, int depth) -> bool {
    if (ti >= img->tex_count || depth > 64) return true;   // conservative
    if (reads_uv[ti] >= 0) return reads_uv[ti] != 0;
    const uint32_t *t = &c.texs[static_cast<size_t>(ti) * kTexWords];
    bool r = t[T_KIND] == T_IMAGE;
    if (t[T_KIND] == T_CHECKER) r = self(self, t[T_EVEN], depth + 1) || self(self, t[T_ODD], depth + 1);
    reads_uv[ti] = r ? 1 : 0;
    return r;
  };
  for (uint32_t i = 0; i < sc->hittable_count; ++i) {
    uint32_t *w = &W[static_cast<size_t>(i) * kNodeWords];
    if (w[W_KIND] != K_SPHERE) continue;
    const uint32_t *m = &c.mats[static_cast<size_t>(w[W_AUX]) * kMatWords];
    const bool textured = m[M_KIND] == MAT_LAMBERTIAN || m[M_KIND] == MAT_DIFFUSE_LIGHT;
    w[W_SPHERE_UV] = !lazy_uv || (textured && tex_reads_uv(tex_reads_uv, m[M_TEX], 0)) ? 1u : 0u;
  }
  img->off_mats = static_cast<uint32_t>(W.size());
  W.insert(W.end(), c.mats.begin(), c.mats.end());
  img->off_texs = static_cast<uint32_t>(W.size());
  W.insert(W.end(), c.texs.begin(), c.texs.end());
  // constant colour records (rt_layout.h kRcConsts): magenta, black, NaN grey at words 1..3
  img->rec_consts = img->mat_count + img->tex_count;
  {
    const float nan = std::nanf("");
    const float rgb[kRcConsts][3] = {{1.0f, 0.0f, 1.0f}, {0.0f, 0.0f, 0.0f}, {nan, nan, nan}};
    for (uint32_t k = 0; k < kRcConsts; ++k) {
      uint32_t w[kRecWords] = {0xffffffffu};
      for (int ch = 0; ch < 3; ++ch) w[1 + ch] = fbits(rgb[k][ch]);
      W.insert(W.end(), w, w + kRecWords);
    }
  }
  while (W.size() % 4) W.push_back(0);   // float4 alignment for the gradient table
  img->off_perlin = static_cast<uint32_t>(W.size());
  W.insert(W.end(), c.perlin.begin(), c.perlin.end());
  img->off_pixels = static_cast<uint32_t>(W.size());
  W.insert(W.end(), c.pixels.begin(), c.pixels.end());
  return RT_OK;
}

}  // namespace rt
