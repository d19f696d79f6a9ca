// rt_host.cpp — host side of the render path: scene records, BVH, scene catalog, camera, PPM.
//
// Clean-room restatement of luk-zm/cuda_raytracing's host pre-pass.  The
// arithmetic follows the reference statement by statement (float ops in source order, no FP
// contraction: build with -ffp-contract=off) and consumes glibc rand() in the order g++ evaluates
// the reference's calls (function arguments right-to-left, braced initialisers left-to-right;
// SURVEY §7 "Argument-evaluation order").  Output: rt_ref_layout.h bytes.
#include "rt_host.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "glibc_rand.h"

namespace {

constexpr float kPi = 3.1415926535897932385f;   // utility.h:24

inline float inf_f32() { return INFINITY; }      // utility.h:100-105
inline float neg_inf_f32() { return -INFINITY; } // utility.h:107-112

// utility.h:6-8 — ternary semantics (NaN falls through to the second operand)
inline float tmin(float a, float b) { return (a < b) ? a : b; }
inline float tmax(float a, float b) { return (a < b) ? b : a; }

inline rtr_vec3 V(float x, float y, float z) { return rtr_vec3{x, y, z}; }
// Scene literals are written as doubles in the reference and converted to f32 at the call.
inline rtr_vec3 Vd(double x, double y, double z) {
  return rtr_vec3{static_cast<float>(x), static_cast<float>(y), static_cast<float>(z)};
}
inline rtr_vec3 add(rtr_vec3 a, rtr_vec3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
inline rtr_vec3 sub(rtr_vec3 a, rtr_vec3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
inline rtr_vec3 scale(float s, rtr_vec3 v) { return V(v.x * s, v.y * s, v.z * s); }
inline rtr_vec3 neg(rtr_vec3 v) { return V(-v.x, -v.y, -v.z); }
inline float dot(rtr_vec3 a, rtr_vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline rtr_vec3 cross(rtr_vec3 a, rtr_vec3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline float length(rtr_vec3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
inline rtr_vec3 unit(rtr_vec3 v) {   // vec3.h:106-114
  float l = length(v);
  if (l == 0.0f) return V(0.0f, 0.0f, 0.0f);
  return V(v.x / l, v.y / l, v.z / l);
}
inline rtr_vec3 comp_scale(rtr_vec3 a, rtr_vec3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
inline rtr_vec3 line_at(rtr_vec3 o, float t, rtr_vec3 d) { return add(o, scale(t, d)); }

// ---- AABB (raytracing.cu:538-581) ----
inline void pad_to_minimums(rtr_aabb *b) {
  const float delta = 0.0001f;
  auto expand = [&](float *lo, float *hi) { float p = delta / 2; *lo -= p; *hi += p; };
  if ((b->x1 - b->x0) < delta) expand(&b->x0, &b->x1);
  if ((b->y1 - b->y0) < delta) expand(&b->y0, &b->y1);
  if ((b->z1 - b->z0) < delta) expand(&b->z0, &b->z1);
}
inline rtr_aabb make_aabb(rtr_vec3 p1, rtr_vec3 p2) {
  rtr_aabb r;
  r.x0 = tmin(p1.x, p2.x); r.x1 = tmax(p1.x, p2.x);
  r.y0 = tmin(p1.y, p2.y); r.y1 = tmax(p1.y, p2.y);
  r.z0 = tmin(p1.z, p2.z); r.z1 = tmax(p1.z, p2.z);
  pad_to_minimums(&r);
  return r;
}
inline rtr_aabb merge(const rtr_aabb &a, const rtr_aabb &b) {
  rtr_aabb r;
  r.x0 = tmin(a.x0, b.x0); r.x1 = tmax(a.x1, b.x1);
  r.y0 = tmin(a.y0, b.y0); r.y1 = tmax(a.y1, b.y1);
  r.z0 = tmin(a.z0, b.z0); r.z1 = tmax(a.z1, b.z1);
  pad_to_minimums(&r);
  return r;
}
inline rtr_aabb add_offset(rtr_aabb b, rtr_vec3 o) {
  b.x0 += o.x; b.x1 += o.x; b.y0 += o.y; b.y1 += o.y; b.z0 += o.z; b.z1 += o.z;
  return b;
}

rtr_hittable zero_record() { rtr_hittable h; std::memset(&h, 0, sizeof h); return h; }

// raytracing.cu:683-709
const rtr_aabb *bbox_of(const rtr_hittable &h) {
  switch (h.kind) {
    case RTR_OBJ_SPHERE: return &h.u.sphere.box;
    case RTR_OBJ_BVH: return &h.u.bvh.box;
    case RTR_OBJ_TRIANGLE:
    case RTR_OBJ_QUAD: return &h.u.planar.box;
    case RTR_OBJ_TRANSLATE: return &h.u.translate.box;
    case RTR_OBJ_YROTATE: return &h.u.yrotate.box;
    case RTR_OBJ_GROUP: return &h.u.group.box;
  }
  return nullptr;
}

rtr_plane make_plane(rtr_vec3 q, rtr_vec3 u, rtr_vec3 v) {   // raytracing.cu:607-611,625-629
  rtr_plane g;
  std::memset(&g, 0, sizeof g);
  g.q = q; g.u = u; g.v = v;
  rtr_vec3 n = cross(u, v);
  g.w = scale(1.0f / dot(n, n), n);
  g.normal = unit(n);
  g.d = dot(g.normal, q);
  return g;
}

rtr_hittable make_quad(rtr_vec3 q, rtr_vec3 u, rtr_vec3 v, rtr_material m) {   // :604-620,654-658
  rtr_hittable h = zero_record();
  h.kind = RTR_OBJ_QUAD;
  h.u.planar.geom = make_plane(q, u, v);
  h.u.planar.mat = m;
  rtr_aabb b1 = make_aabb(q, add(q, add(u, v)));
  rtr_aabb b2 = make_aabb(add(q, u), add(q, v));
  h.u.planar.box = merge(b1, b2);
  return h;
}

rtr_hittable make_triangle(rtr_vec3 q, rtr_vec3 u, rtr_vec3 v, rtr_material m) {  // :622-652,660-664
  rtr_hittable h = zero_record();
  h.kind = RTR_OBJ_TRIANGLE;
  h.u.planar.geom = make_plane(q, u, v);
  h.u.planar.mat = m;
  rtr_vec3 p1 = add(q, v), p2 = add(q, u);
  rtr_aabb b;
  b.x0 = tmin(q.x, tmin(p1.x, p2.x)); b.x1 = tmax(q.x, tmax(p1.x, p2.x));
  b.y0 = tmin(q.y, tmin(p1.y, p2.y)); b.y1 = tmax(q.y, tmax(p1.y, p2.y));
  b.z0 = tmin(q.z, tmin(p1.z, p2.z)); b.z1 = tmax(q.z, tmax(p1.z, p2.z));
  const float eps = 1e-3f;
  b.x0 -= eps; b.x1 += eps; b.y0 -= eps; b.y1 += eps; b.z0 -= eps; b.z1 += eps;
  h.u.planar.box = b;
  return h;
}

rtr_hittable make_sphere(rtr_vec3 c, float r, rtr_material m) {   // :592-602
  rtr_hittable h = zero_record();
  h.kind = RTR_OBJ_SPHERE;
  h.u.sphere.center = c;
  h.u.sphere.motion = V(0.0f, 0.0f, 0.0f);
  h.u.sphere.radius = r;
  h.u.sphere.mat = m;
  rtr_vec3 rv = V(r, r, r);
  h.u.sphere.box = make_aabb(sub(c, rv), add(c, rv));
  return h;
}

rtr_hittable make_moving_sphere(rtr_vec3 c, rtr_vec3 motion, float r, rtr_material m) {  // :666-681
  rtr_hittable h = zero_record();
  h.kind = RTR_OBJ_SPHERE;
  h.u.sphere.center = c;
  h.u.sphere.motion = motion;
  h.u.sphere.radius = r;
  h.u.sphere.mat = m;
  rtr_vec3 rv = V(r, r, r);
  rtr_vec3 p0 = line_at(c, 0.0f, motion), p1 = line_at(c, 1.0f, motion);
  rtr_aabb b1 = make_aabb(sub(p0, rv), add(p0, rv));
  rtr_aabb b2 = make_aabb(sub(p1, rv), add(p1, rv));
  h.u.sphere.box = merge(b1, b2);
  return h;
}

}  // namespace

// ============================================================================================
struct rt_world {
  uint32_t capacity;
  std::vector<rtr_hittable> objs;
  std::vector<uint16_t> refs;
  std::vector<uint8_t> arena;
  uint64_t arena_cap;
  rt::GlibcRand rng;
  bool failed = false;
  bool unsupported = false;   // an image file exists in a format this build does not decode

  // utility.h:26-41
  float random_f32() { return static_cast<float>(rng.next()) / (2147483647 + 1.0f); }
  float random_bound(float lo, float hi) { return lo + (hi - lo) * random_f32(); }
  int32_t random_i32_bound(int32_t lo, int32_t hi) {
    return static_cast<int32_t>(random_bound(static_cast<float>(lo), static_cast<float>(hi + 1)));
  }
  // vec3.h:122-128 — Vec3(f(), f(), f()) evaluated right-to-left by g++: z, then y, then x
  rtr_vec3 random_vec() { float z = random_f32(); float y = random_f32(); float x = random_f32(); return V(x, y, z); }
  rtr_vec3 random_vec_bound(float lo, float hi) {
    float z = random_bound(lo, hi); float y = random_bound(lo, hi); float x = random_bound(lo, hi);
    return V(x, y, z);
  }

  // raytracing.cu:833-842 (asserts capacity)
  uint32_t list_add(const rtr_hittable &h) {
    if (objs.size() >= capacity || objs.size() >= 65535u) { failed = true; return 0; }
    objs.push_back(h);
    return static_cast<uint32_t>(objs.size() - 1);
  }
  // raytracing.cu:256-261 (we reject the silent drop instead of returning a dangling ref)
  uint16_t ref_add(uint32_t idx) {
    if (refs.size() >= capacity || refs.size() >= 65535u) { failed = true; return 0; }
    refs.push_back(static_cast<uint16_t>(idx));
    return static_cast<uint16_t>(refs.size() - 1);
  }
  uint8_t *arena_push(uint64_t size) {   // memory.h:30-38 (no alignment)
    if (arena.size() + size > arena_cap) { failed = true; return nullptr; }
    arena.resize(arena.size() + size);
    return arena.data() + arena.size() - size;
  }

  // raytracing.cu:263-291
  rtr_texref texture_add(const rtr_texture &tex, const rtr_perlin *perlin,
                         const float *pixels, uint64_t pixel_count) {
    rtr_texref ref{arena.size()};
    rtr_texture t = tex;
    uint8_t *slot = arena_push(sizeof(rtr_texture));
    if (!slot) return ref;
    if (t.kind == RTR_TEX_IMAGE) {
      t.u.image.pixels_offset = arena.size();
      std::memcpy(arena.data() + ref.offset, &t, sizeof t);
      uint64_t bytes = sizeof(float) * 3 * pixel_count;
      uint8_t *dst = arena_push(bytes);
      if (dst && bytes) std::memcpy(dst, pixels, bytes);
    } else if (t.kind == RTR_TEX_NOISE) {
      t.u.noise.table_offset = arena.size();
      std::memcpy(arena.data() + ref.offset, &t, sizeof t);
      uint8_t *dst = arena_push(sizeof(rtr_perlin));
      if (dst) std::memcpy(dst, perlin, sizeof(rtr_perlin));
    } else {
      std::memcpy(slot, &t, sizeof t);
    }
    return ref;
  }

  rtr_texref solid_texture(rtr_vec3 c) {
    rtr_texture t; std::memset(&t, 0, sizeof t);
    t.kind = RTR_TEX_SOLID; t.u.solid = c;
    return texture_add(t, nullptr, nullptr, 0);
  }

  // perlin_noise.cpp:48-70
  void perlin_permutation(int32_t *arr) {
    for (int32_t i = 0; i < RTR_PERLIN_POINTS; ++i) arr[i] = i;
    for (int32_t i = RTR_PERLIN_POINTS - 1; i > 0; --i) {
      int32_t target = random_i32_bound(0, i);
      int32_t tmp = arr[i]; arr[i] = arr[target]; arr[target] = tmp;
    }
  }
  void make_perlin(rtr_perlin *p) {
    std::memset(p, 0, sizeof *p);
    for (int i = 0; i < RTR_PERLIN_POINTS; ++i) p->gradients[i] = unit(random_vec_bound(-1, 1));
    perlin_permutation(p->perm_x);
    perlin_permutation(p->perm_y);
    perlin_permutation(p->perm_z);
  }

  // raytracing.cu:787-794
  rtr_hittable make_translation(uint32_t child, rtr_vec3 offset) {
    rtr_hittable h = zero_record();
    h.kind = RTR_OBJ_TRANSLATE;
    h.u.translate.child = static_cast<uint16_t>(child);
    h.u.translate.offset = offset;
    h.u.translate.box = add_offset(*bbox_of(objs[child]), offset);
    return h;
  }
  // raytracing.cu:796-831
  rtr_hittable make_y_rotation(uint32_t child, float angle) {
    rtr_hittable h = zero_record();
    h.kind = RTR_OBJ_YROTATE;
    rtr_yrotate &y = h.u.yrotate;
    y.child = static_cast<uint16_t>(child);
    float radians = angle * (kPi / 180);
    y.sin_theta = sinf(radians);
    y.cos_theta = cosf(radians);
    y.box = *bbox_of(objs[child]);
    rtr_vec3 mn = V(inf_f32(), inf_f32(), inf_f32());
    rtr_vec3 mx = V(neg_inf_f32(), neg_inf_f32(), neg_inf_f32());
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j)
        for (int k = 0; k < 2; ++k) {
          float x = i * y.box.x1 + (1 - i) * y.box.x0;
          float yy = j * y.box.y1 + (1 - j) * y.box.y0;
          float z = k * y.box.z1 + (1 - k) * y.box.z0;
          float nx = y.cos_theta * x + y.sin_theta * z;
          float nz = -y.sin_theta * x + y.cos_theta * z;
          mn.x = tmin(mn.x, nx); mx.x = tmax(mx.x, nx);
          mn.y = tmin(mn.y, yy); mx.y = tmax(mx.y, yy);
          mn.z = tmin(mn.z, nz); mx.z = tmax(mx.z, nz);
        }
    y.box = make_aabb(mn, mx);
    return h;
  }

  // raytracing.cu:908-927 — reserves `size` zeroed slots, returns the (not yet added) group record
  rtr_hittable make_group(uint64_t size) {
    rtr_hittable g = zero_record();
    g.kind = RTR_OBJ_GROUP;
    g.u.group.first = static_cast<uint16_t>(objs.size());
    g.u.group.size = size;
    for (uint64_t i = 0; i < size; ++i) list_add(zero_record());
    return g;
  }
  void group_add(rtr_hittable *g, const rtr_hittable &h) {
    rtr_group &s = g->u.group;
    if (s.count <= s.size) {
      uint64_t idx = s.first + s.count;
      if (idx < objs.size()) objs[idx] = h;
      s.box = merge(s.box, *bbox_of(h));
      s.count += 1;
    }
  }
  // raytracing.cu:929-952
  rtr_hittable make_box(rtr_vec3 a, rtr_vec3 b, rtr_material m) {
    rtr_hittable box = make_group(6);
    rtr_vec3 mn = V(tmin(a.x, b.x), tmin(a.y, b.y), tmin(a.z, b.z));
    rtr_vec3 mx = V(tmax(a.x, b.x), tmax(a.y, b.y), tmax(a.z, b.z));
    rtr_vec3 dx = V(mx.x - mn.x, 0, 0), dy = V(0, mx.y - mn.y, 0), dz = V(0, 0, mx.z - mn.z);
    group_add(&box, make_quad(V(mn.x, mn.y, mx.z), dx, dy, m));
    group_add(&box, make_quad(V(mx.x, mn.y, mx.z), neg(dz), dy, m));
    group_add(&box, make_quad(V(mx.x, mn.y, mn.z), neg(dx), dy, m));
    group_add(&box, make_quad(V(mn.x, mn.y, mn.z), dz, dy, m));
    group_add(&box, make_quad(V(mn.x, mx.y, mx.z), dx, neg(dz), m));
    group_add(&box, make_quad(V(mn.x, mn.y, mn.z), dx, dz, m));
    return box;
  }
  // raytracing.cu:954-980
  rtr_hittable make_pyramid(rtr_vec3 a, rtr_vec3 b, rtr_vec3 tip, rtr_material m) {
    rtr_hittable p = make_group(5);
    rtr_vec3 mn = V(tmin(a.x, b.x), tmin(a.y, b.y), tmin(a.z, b.z));
    rtr_vec3 mx = V(tmax(a.x, b.x), tmax(a.y, b.y), tmax(a.z, b.z));
    rtr_vec3 dx = V(mx.x - mn.x, 0, 0), dz = V(0, 0, mx.z - mn.z);
    rtr_vec3 p1 = V(mn.x, mn.y, mn.z), p2 = V(mx.x, mn.y, mn.z);
    rtr_vec3 p3 = V(mx.x, mn.y, mx.z), p4 = V(mn.x, mn.y, mx.z);
    group_add(&p, make_quad(V(mn.x, mn.y, mn.z), dx, dz, m));
    group_add(&p, make_triangle(p1, dx, sub(tip, p1), m));
    group_add(&p, make_triangle(p2, dz, sub(tip, p2), m));
    group_add(&p, make_triangle(p3, neg(dx), sub(tip, p3), m));
    group_add(&p, make_triangle(p4, neg(dz), sub(tip, p4), m));
    return p;
  }

  // world_add / world_add_translated / world_add_rotated / world_add_rotated_translated (:1775-1803)
  int add(int xf, float angle, rtr_vec3 offset, const rtr_hittable &h) {
    uint32_t idx;
    switch (xf) {
      case RT_XF_NONE: return ref_add(list_add(h));
      case RT_XF_TRANSLATE: idx = list_add(h); return ref_add(list_add(make_translation(idx, offset)));
      case RT_XF_YROTATE: idx = list_add(h); return ref_add(list_add(make_y_rotation(idx, angle)));
      case RT_XF_YROTATE_TRANSLATE:
        idx = list_add(h);
        idx = list_add(make_y_rotation(idx, angle));
        idx = list_add(make_translation(idx, offset));
        return ref_add(idx);
    }
    failed = true;
    return -1;
  }

  // ---- BVH (raytracing.cu:711-785, 850-906) ----
  bool less_on_axis(uint16_t a, uint16_t b, int axis) const {
    const rtr_aabb *ba = bbox_of(objs[a]), *bb = bbox_of(objs[b]);
    switch (axis) {
      case 0: return ba->x0 < bb->x0;
      case 1: return ba->y0 < bb->y0;
      case 2: return ba->z0 < bb->z0;
    }
    return false;   // axis 3 (random_f32()==1.0): every comparison false
  }
  // top-down merge sort of refs[lo..hi] (inclusive); mid = (lo+hi)/2; ties take the right run
  void merge_sort(std::vector<uint16_t> &tmp, uint64_t lo, uint64_t hi, int axis) {
    if (hi <= lo) return;
    uint64_t mid = (hi + lo) / 2;
    merge_sort(tmp, lo, mid, axis);
    merge_sort(tmp, mid + 1, hi, axis);
    uint64_t a = lo, b = mid + 1, o = lo;
    while (a <= mid && b <= hi) {
      if (less_on_axis(refs[a], refs[b], axis)) tmp[o++] = refs[a++];
      else tmp[o++] = refs[b++];
    }
    while (a <= mid) tmp[o++] = refs[a++];
    while (b <= hi) tmp[o++] = refs[b++];
    for (uint64_t i = lo; i <= hi; ++i) refs[i] = tmp[i];
  }
  uint16_t build_bvh(uint64_t start, uint64_t end) {
    rtr_hittable node = zero_record();
    node.kind = RTR_OBJ_BVH;
    uint64_t span = end - start;
    uint16_t left, right;
    if (span == 1) {
      left = right = static_cast<uint16_t>(start);
    } else if (span == 2) {
      left = static_cast<uint16_t>(start);
      right = static_cast<uint16_t>(start + 1);
    } else {
      int axis = random_i32_bound(0, 2);
      std::vector<uint16_t> tmp(refs);
      merge_sort(tmp, start, end - 1, axis);
      uint64_t mid = start + span / 2;
      left = build_bvh(start, mid);
      right = build_bvh(mid, end);
    }
    node.u.bvh.left = left;
    node.u.bvh.right = right;
    node.u.bvh.box = merge(*bbox_of(objs[refs[left]]), *bbox_of(objs[refs[right]]));
    return ref_add(list_add(node));
  }
};

// ============================================================================================
namespace {

rtr_material mat_with_tex(uint32_t kind, rtr_texref t) {
  rtr_material m; std::memset(&m, 0, sizeof m);
  m.kind = kind;
  m.u.lambert_tex = t;   // light_tex aliases the same bytes
  return m;
}

}  // namespace

extern "C" {

rt_world *rt_world_create(uint32_t capacity, uint64_t arena_bytes) {
  rt_world *w = new (std::nothrow) rt_world();
  if (!w) return nullptr;
  w->capacity = capacity ? capacity : 8000;
  w->arena_cap = arena_bytes ? arena_bytes : (10ull << 20);
  w->objs.reserve(w->capacity);
  w->refs.reserve(w->capacity);
  return w;
}

void rt_world_destroy(rt_world *w) { delete w; }

int32_t rt_world_rand(rt_world *w) { return w->rng.next(); }
uint32_t rt_world_hittable_count(const rt_world *w) { return static_cast<uint32_t>(w->objs.size()); }
uint32_t rt_world_ref_count(const rt_world *w) { return static_cast<uint32_t>(w->refs.size()); }
uint64_t rt_world_texture_bytes(const rt_world *w) { return w->arena.size(); }

rtr_material rt_mat_lambert_solid(rt_world *w, rtr_vec3 albedo) {
  return mat_with_tex(RTR_MAT_LAMBERTIAN, w->solid_texture(albedo));
}
rtr_material rt_mat_light_solid(rt_world *w, rtr_vec3 color) {
  return mat_with_tex(RTR_MAT_DIFFUSE_LIGHT, w->solid_texture(color));
}
rtr_material rt_mat_lambert_image(rt_world *w, const char *file_name) {
  // raytracing.cu:332-341 via stbi_loadf (image_load.cpp).  A missing or undecodable file is the
  // reference's failed load: pixels == NULL, width = height = 0, the texture renders magenta (:346-347) —
  // the catalog's earthmap.jpg is not in the reference repository, so that is what every reference run
  // sees.  (An RT_ERR_UNSUPPORTED from the loader, which no format stb decodes returns any more, is the world's status.)
  float *rgb = nullptr;
  int32_t width = 0, height = 0;
  const int st = rt_image_load(file_name, &rgb, &width, &height);
  if (st == RT_OK) {
    rtr_material m = rt_mat_lambert_image_pixels(w, rgb, width, height);
    rt_image_free(rgb);
    return m;
  }
  if (st != RT_IMAGE_MISSING) w->unsupported = true;
  rtr_texture t; std::memset(&t, 0, sizeof t);
  t.kind = RTR_TEX_IMAGE;
  return mat_with_tex(RTR_MAT_LAMBERTIAN, w->texture_add(t, nullptr, nullptr, 0));
}
int rt_world_status(const rt_world *w) {
  if (!w) return RT_ERR_INVALID_ARG;
  return w->failed ? RT_ERR_SCENE : (w->unsupported ? RT_ERR_UNSUPPORTED : RT_OK);
}
rtr_material rt_mat_lambert_image_pixels(rt_world *w, const float *rgb, int32_t width, int32_t height) {
  // what make_image_texture (:332-341) builds when stbi_loadf succeeds: float RGB texels copied into
  // the arena behind the Texture record (texture_list_add, :270-279)
  rtr_texture t; std::memset(&t, 0, sizeof t);
  t.kind = RTR_TEX_IMAGE;
  if (!rgb || width <= 0 || height <= 0) return mat_with_tex(RTR_MAT_LAMBERTIAN, w->texture_add(t, nullptr, nullptr, 0));
  t.u.image.host_pixels = reinterpret_cast<uint64_t>(rgb);
  t.u.image.width = width;
  t.u.image.height = height;
  return mat_with_tex(RTR_MAT_LAMBERTIAN,
                      w->texture_add(t, nullptr, rgb, static_cast<uint64_t>(width) * static_cast<uint64_t>(height)));
}
rtr_material rt_mat_lambert_noise(rt_world *w, float scale) {
  rtr_perlin p;
  w->make_perlin(&p);
  rtr_texture t; std::memset(&t, 0, sizeof t);
  t.kind = RTR_TEX_NOISE;
  t.u.noise.host_table = 1;   // the reference stores a host pointer here; only non-NULL matters
  t.u.noise.scale = scale;
  return mat_with_tex(RTR_MAT_LAMBERTIAN, w->texture_add(t, &p, nullptr, 0));
}
rtr_material rt_mat_metal(rtr_vec3 albedo, float fuzz) {
  rtr_material m; std::memset(&m, 0, sizeof m);
  m.kind = RTR_MAT_METAL; m.u.metal.albedo = albedo; m.u.metal.fuzz = fuzz;
  return m;
}
rtr_material rt_mat_dielectric(float ior) {
  rtr_material m; std::memset(&m, 0, sizeof m);
  m.kind = RTR_MAT_DIELECTRIC; m.u.dielectric.ior = ior;
  return m;
}
rtr_material rt_mat_lambert_checker(rt_world *w, float scale, rtr_vec3 even, rtr_vec3 odd) {
  rtr_texref re = w->solid_texture(even);
  rtr_texref ro = w->solid_texture(odd);
  rtr_texture t; std::memset(&t, 0, sizeof t);
  t.kind = RTR_TEX_CHECKER;
  t.u.checker.inv_scale = 1.0f / scale;
  t.u.checker.even = re; t.u.checker.odd = ro;
  return mat_with_tex(RTR_MAT_LAMBERTIAN, w->texture_add(t, nullptr, nullptr, 0));
}

int rt_add_sphere(rt_world *w, int xf, float angle, rtr_vec3 offset, rtr_vec3 c, float r, rtr_material m) {
  return w->add(xf, angle, offset, make_sphere(c, r, m));
}
int rt_add_moving_sphere(rt_world *w, int xf, float angle, rtr_vec3 offset, rtr_vec3 c, rtr_vec3 motion,
                         float r, rtr_material m) {
  return w->add(xf, angle, offset, make_moving_sphere(c, motion, r, m));
}
int rt_add_quad(rt_world *w, int xf, float angle, rtr_vec3 offset, rtr_vec3 q, rtr_vec3 u, rtr_vec3 v,
                rtr_material m) {
  return w->add(xf, angle, offset, make_quad(q, u, v, m));
}
int rt_add_triangle(rt_world *w, int xf, float angle, rtr_vec3 offset, rtr_vec3 q, rtr_vec3 u, rtr_vec3 v,
                    rtr_material m) {
  return w->add(xf, angle, offset, make_triangle(q, u, v, m));
}
int rt_add_box(rt_world *w, int xf, float angle, rtr_vec3 offset, rtr_vec3 a, rtr_vec3 b, rtr_material m) {
  rtr_hittable box = w->make_box(a, b, m);
  return w->add(xf, angle, offset, box);
}
int rt_add_pyramid(rt_world *w, int xf, float angle, rtr_vec3 offset, rtr_vec3 a, rtr_vec3 b, rtr_vec3 tip,
                   rtr_material m) {
  rtr_hittable p = w->make_pyramid(a, b, tip, m);
  return w->add(xf, angle, offset, p);
}

int rt_world_build_bvh(rt_world *w, uint16_t *root) {
  if (!w || !root || w->refs.empty()) return RT_ERR_INVALID_ARG;
  uint16_t r = w->build_bvh(0, w->refs.size());
  if (w->failed) return RT_ERR_SCENE;
  *root = r;
  return RT_OK;
}

int rt_world_scene(const rt_world *w, uint16_t root, rt_scene *out) {
  if (!w || !out) return RT_ERR_INVALID_ARG;
  std::memset(out, 0, sizeof *out);
  out->hittables = w->objs.data();
  out->hittable_count = static_cast<uint32_t>(w->objs.size());
  out->refs = w->refs.data();
  out->ref_count = static_cast<uint32_t>(w->refs.size());
  out->root = root;
  out->textures = w->arena.data();
  out->texture_bytes = w->arena.size();
  return w->failed ? RT_ERR_SCENE : RT_OK;
}

// ---- settings + catalog (raytracing.cu:1523-1529, 1979-2320; main.cu:52-117) ----
static void set_name(rt_settings *s, const char *n) {
  std::snprintf(s->img_name, sizeof s->img_name, "%s", n);
}

void rt_settings_default(rt_settings *s) {
  std::memset(s, 0, sizeof *s);
  s->img_ratio = 1; s->img_width = 800; s->samples_per_pixel = 100; s->max_bounces = 50; s->vfov = 90;
  s->lookfrom = V(0, 0, 0); s->lookat = V(0, 0, -1); s->view_up = V(0, 1, 0);
  s->defocus_angle = 0.0f; s->background = V(0.7f, 0.8f, 1.0f);
  set_name(s, "image.ppm");
}

static void bouncing_settings(rt_settings *s) {   // g_bouncing_spheres_settings, :1523-1525
  std::memset(s, 0, sizeof *s);
  s->img_ratio = 16.0f / 9.0f; s->img_width = 1200; s->samples_per_pixel = 100; s->max_bounces = 50;
  s->vfov = 20.0f; s->lookfrom = V(13.0f, 2.0f, 3.0f); s->lookat = V(0, 0, 0); s->view_up = V(0, 1, 0);
  s->defocus_angle = 0.6f; s->background = V(0.7f, 0.8f, 1.0f);
  set_name(s, "image.ppm");
}

static const rtr_vec3 kZero = {0.0f, 0.0f, 0.0f};

// bouncing_spheres_scene (:1979-2020); `half` = 11 in the reference, 50 for the 10k scene
static void scene_bouncing(rt_world *w, rt_settings *s, int half) {
  rtr_material default_mat = rt_mat_lambert_solid(w, Vd(0.5, 0.5, 0.5));
  (void)default_mat;
  rtr_material ground = rt_mat_lambert_checker(w, static_cast<float>(0.32), Vd(0.2, 0.3, 0.1), Vd(0.9, 0.9, 0.9));
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, -1000, 0), 1000, ground);
  for (int32_t a = -half; a < half; ++a) {
    for (int32_t b = -half; b < half; ++b) {
      float choice = w->random_f32();
      float cx = a + 0.9f * w->random_f32();          // braced initialiser: left to right
      float cz = b + 0.9f * w->random_f32();
      rtr_vec3 center = V(cx, 0.2f, cz);
      if (length(sub(center, V(4.0f, 0.2f, 0.0f))) > 0.9f) {
        rtr_material m;
        if (choice < 0.8f) {
          rtr_vec3 rb = w->random_vec();                // vec3_comp_scale(r(), r()): right arg first
          rtr_vec3 ra = w->random_vec();
          m = rt_mat_lambert_solid(w, comp_scale(ra, rb));
          rtr_vec3 dir = V(0.0f, w->random_bound(0.0f, 0.5f), 0.0f);
          rt_add_moving_sphere(w, RT_XF_NONE, 0, kZero, center, dir, static_cast<float>(0.2), m);
        } else {
          if (choice < 0.95f) {
            rtr_vec3 albedo = w->random_vec_bound(0.5f, 1.0f);
            float fuzz = w->random_bound(0.0f, 0.5f);
            m = rt_mat_metal(albedo, fuzz);
          } else {
            m = rt_mat_dielectric(1.5f);
          }
          rt_add_sphere(w, RT_XF_NONE, 0, kZero, center, static_cast<float>(0.2), m);
        }
      }
    }
  }
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 1, 0), 1, rt_mat_dielectric(1.5f));
  rtr_material m2 = rt_mat_lambert_solid(w, Vd(0.4, 0.2, 0.1));
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(-4, 1, 0), 1, m2);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(4, 1, 0), 1, rt_mat_metal(V(0.7f, 0.6f, 0.5f), 0.0f));
  bouncing_settings(s);
}

static void scene_checkered(rt_world *w, rt_settings *s) {   // :2022-2040
  rtr_material m = rt_mat_lambert_checker(w, static_cast<float>(0.32), Vd(0.2, 0.3, 0.1), Vd(0.9, 0.9, 0.9));
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, -10, 0), 10, m);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 10, 0), 10, m);
  s->img_ratio = 16.0f / 9.0f; s->img_width = 400; s->samples_per_pixel = 100; s->max_bounces = 50;
  s->vfov = 20.0f; s->lookfrom = V(13.0f, 2.0f, 3.0f); s->lookat = V(0, 0, 0);
  s->view_up = V(0.0f, 0.1f, 0.0f); s->defocus_angle = 0.0f; s->background = V(0.7f, 0.8f, 1.0f);
  set_name(s, "checkered_spheres.ppm");
}

static void scene_earth(rt_world *w, rt_settings *s) {   // :2042-2052
  rtr_material m = rt_mat_lambert_image(w, "earthmap.jpg");
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 0, 0), 2, m);
  s->img_width = 400; s->samples_per_pixel = 100; s->lookfrom = V(0, 0, 12); s->lookat = V(0, 0, 0);
  s->defocus_angle = 0; set_name(s, "earth.ppm");
}

static void scene_perlin(rt_world *w, rt_settings *s) {   // :2054-2065
  rtr_material m = rt_mat_lambert_noise(w, 4);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, -1000, 0), 1000, m);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 2, 0), 2, m);
  s->img_width = 400; s->samples_per_pixel = 100; s->lookfrom = V(13, 2, 3); s->lookat = V(0, 0, 0);
  s->defocus_angle = 0; set_name(s, "perlin_spheres.ppm");
}

static void scene_quads(rt_world *w, rt_settings *s) {   // :2067-2091
  rtr_material left = rt_mat_lambert_solid(w, V(1.0f, 0.2f, 0.2f));
  rtr_material back = rt_mat_lambert_solid(w, V(0.2f, 1.0f, 0.2f));
  rtr_material right = rt_mat_lambert_solid(w, V(0.2f, 0.2f, 1.0f));
  rtr_material upper = rt_mat_lambert_solid(w, V(1.0f, 0.5f, 0.0f));
  rtr_material lower = rt_mat_lambert_solid(w, V(0.2f, 0.8f, 0.8f));
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(-3, -2, 5), V(0, 0, -4), V(0, 4, 0), left);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(-2, -2, 0), V(4, 0, 0), V(0, 4, 0), back);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(3, -2, 1), V(0, 0, 4), V(0, 4, 0), right);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(-2, 3, 1), V(4, 0, 0), V(0, 0, 4), upper);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(-2, -3, 5), V(4, 0, 0), V(0, 0, -4), lower);
  s->img_ratio = 1.0f; s->img_width = 400; s->samples_per_pixel = 100; s->max_bounces = 50; s->vfov = 80;
  s->lookfrom = V(0, 0, 9); s->lookat = V(0, 0, 0); s->view_up = V(0, 1, 0); s->defocus_angle = 0;
  s->background = V(0.7f, 0.8f, 1.0f); set_name(s, "quads.ppm");
}

static void scene_simple_light(rt_world *w, rt_settings *s) {   // :2093-2111
  rtr_material noise = rt_mat_lambert_noise(w, 4);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, -1000, 0), 1000, noise);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 2, 0), 2, noise);
  rtr_material light = rt_mat_light_solid(w, V(4, 4, 4));
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(3, 1, -2), V(2, 0, 0), V(0, 2, 0), light);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 7, 0), 2, light);
  s->img_ratio = 16.0f / 9.0f; s->img_width = 1080; s->samples_per_pixel = 1000; s->max_bounces = 50;
  s->vfov = 20; s->lookfrom = V(26, 3, 6); s->lookat = V(0, 2, 0); s->view_up = V(0, 1, 0);
  set_name(s, "simple_light.ppm");
}

static void scene_cornell(rt_world *w, rt_settings *s) {   // :2113-2149
  rtr_material red = rt_mat_lambert_solid(w, Vd(0.65, 0.05, 0.05));
  rtr_material white = rt_mat_lambert_solid(w, Vd(0.73, 0.73, 0.73));
  rtr_material green = rt_mat_lambert_solid(w, Vd(0.12, 0.45, 0.15));
  rtr_material light = rt_mat_light_solid(w, V(15, 15, 15));
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(555, 0, 0), V(0, 555, 0), V(0, 0, 555), green);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(0, 0, 0), V(0, 555, 0), V(0, 0, 555), red);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(343, 554, 332), V(-130, 0, 0), V(0, 0, -105), light);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(0, 0, 0), V(555, 0, 0), V(0, 0, 555), white);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(555, 555, 555), V(-555, 0, 0), V(0, 0, -555), white);
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(0, 0, 555), V(555, 0, 0), V(0, 555, 0), white);
  rt_add_box(w, RT_XF_YROTATE_TRANSLATE, 15, V(265, 0, 295), V(0, 0, 0), V(165, 330, 165), white);
  rt_add_box(w, RT_XF_YROTATE_TRANSLATE, -18, V(130, 0, 100), V(0, 0, 0), V(165, 165, 165), white);
  s->img_ratio = 1.0f; s->img_width = 600; s->samples_per_pixel = 200; s->max_bounces = 40; s->vfov = 40;
  s->lookfrom = V(278, 278, -800); s->lookat = V(278, 278, 0); s->view_up = V(0, 1, 0);
  s->defocus_angle = 0; s->background = V(0, 0, 0); set_name(s, "cornell_box.ppm");
}

static void scene_final(rt_world *w, rt_settings *s) {   // :2151-2202
  rtr_material ground = rt_mat_lambert_solid(w, V(0.48f, 0.83f, 0.53f));
  const int32_t per_side = 20;
  for (int32_t i = 0; i < per_side; ++i) {
    for (int32_t j = 0; j < per_side; ++j) {
      float wd = 100;
      float x0 = -1000.0f + i * wd, z0 = -1000.0f + j * wd, y0 = 0;
      float x1 = x0 + wd;
      float y1 = w->random_bound(1, 101);
      float z1 = z0 + wd;
      rt_add_box(w, RT_XF_NONE, 0, kZero, V(x0, y0, z0), V(x1, y1, z1), ground);
    }
  }
  rtr_material light = rt_mat_light_solid(w, V(7, 7, 7));
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(123, 554, 147), V(300, 0, 0), V(0, 0, 265), light);
  rtr_material sm = rt_mat_lambert_solid(w, V(0.7f, 0.3f, 0.1f));
  rt_add_moving_sphere(w, RT_XF_NONE, 0, kZero, V(400, 400, 200), V(30, 0, 0), 50, sm);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(260, 150, 45), 50, rt_mat_dielectric(1.5f));
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(0, 150, 145), 50, rt_mat_metal(V(0.8f, 0.8f, 0.9f), 1.0f));
  rtr_material earth = rt_mat_lambert_image(w, "earthmap.jpg");
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(400, 200, 400), 100, earth);
  rtr_material perlin = rt_mat_lambert_noise(w, 0.2f);
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, V(220, 280, 300), 80, perlin);
  rtr_material white = rt_mat_lambert_solid(w, V(0.73f, 0.73f, 0.73f));
  for (int32_t i = 0; i < 1000; ++i) {
    rtr_vec3 c = w->random_vec_bound(0, 165);
    rt_add_sphere(w, RT_XF_YROTATE_TRANSLATE, 15, V(-100, 270, 395), c, 10, white);
  }
  s->img_ratio = 1.0f; s->img_width = 800; s->samples_per_pixel = 10000; s->max_bounces = 40;
  s->vfov = 40.0f; s->lookfrom = V(478, 278, -600); s->lookat = V(278, 278, 0);
  s->view_up = V(0.0f, 0.1f, 0.0f); s->defocus_angle = 0.0f; s->background = kZero;
  set_name(s, "feature_test.ppm");
}

// fv1 / metal_test_scene / refract_test_scene share the box + pyramid set (:2206-2269)
static void box_and_pyramid(rt_world *w) {
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(-5, 0, 1), V(10, 0, 0), V(0, 0, -5),
              rt_mat_lambert_solid(w, Vd(0.73, 0.73, 0.73)));
  rt_add_box(w, RT_XF_TRANSLATE, 0, Vd(-1.5, 0, -1), kZero, Vd(0.7, 0.7, 0.7),
             rt_mat_lambert_solid(w, Vd(0.5, 0, 0)));
  rt_add_pyramid(w, RT_XF_YROTATE_TRANSLATE, 30, V(1, 0, -1), kZero, Vd(0.7, 0, 0.7), Vd(0.35, 1.5, 0.35),
                 rt_mat_lambert_solid(w, Vd(0, 0, 0.5)));
}

static void scene_fv1(rt_world *w, rt_settings *s) {
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, Vd(0, 0.5, -1), 0.5f, rt_mat_lambert_solid(w, Vd(0, 0.5, 0)));
  box_and_pyramid(w);
  s->img_width = 800; s->img_ratio = static_cast<float>(16.0 / 9.0); s->samples_per_pixel = 100;
  s->max_bounces = 40; s->lookfrom = Vd(0, 0.9, 0.75); s->lookat = Vd(0, 0.5, -1);
  set_name(s, "fv1.ppm");
}

static void scene_metal(rt_world *w, rt_settings *s, float fuzz, const char *name) {
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, Vd(0, 0.5, -1), 0.5f, rt_mat_metal(Vd(0.8, 0.8, 0.8), fuzz));
  box_and_pyramid(w);
  s->img_width = 800; s->img_ratio = static_cast<float>(16.0 / 9.0); s->samples_per_pixel = 100;
  s->max_bounces = 40; s->lookfrom = Vd(0, 0.9, 0); s->lookat = Vd(0, 0.5, -1);
  set_name(s, name);
}

static void scene_refract(rt_world *w, rt_settings *s, float ior, const char *name) {
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, Vd(-0.4, 0.5, -2), 0.5f, rt_mat_lambert_solid(w, Vd(0.5, 0.5, 0)));
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, Vd(0, 0.5, -1), 0.5f, rt_mat_dielectric(ior));
  box_and_pyramid(w);
  s->img_width = 800; s->img_ratio = static_cast<float>(16.0 / 9.0); s->samples_per_pixel = 100;
  s->max_bounces = 40; s->lookfrom = Vd(0, 0.9, 0); s->lookat = Vd(0, 0.5, -1);
  set_name(s, name);
}

static void scene_motion_blur(rt_world *w, rt_settings *s) {   // :2291-2303
  rt_add_moving_sphere(w, RT_XF_NONE, 0, kZero, Vd(-1, 0.5, -1), V(0, 1, 0), 0.5f,
                       rt_mat_lambert_solid(w, Vd(0.5, 0.5, 0)));
  rt_add_moving_sphere(w, RT_XF_NONE, 0, kZero, Vd(1, 0.5, -1), Vd(0, 0.5, 0), 0.5f,
                       rt_mat_lambert_solid(w, Vd(0.5, 0.5, 0.5)));
  rt_add_quad(w, RT_XF_NONE, 0, kZero, V(-5, 0, 1), V(10, 0, 0), V(0, 0, -5),
              rt_mat_lambert_solid(w, Vd(0.73, 0.73, 0.73)));
  s->img_width = 800; s->img_ratio = static_cast<float>(16.0 / 9.0); s->samples_per_pixel = 100;
  s->max_bounces = 40; s->lookfrom = Vd(0, 0.9, 0.5); s->lookat = Vd(0, 0.5, -1);
  set_name(s, "mblur.ppm");
}

static void scene_light_test(rt_world *w, rt_settings *s) {   // :2305-2320
  rt_add_sphere(w, RT_XF_NONE, 0, kZero, Vd(0, 0.5, -1), 0.5f, rt_mat_light_solid(w, V(15, 15, 15)));
  box_and_pyramid(w);
  s->img_width = 800; s->img_ratio = static_cast<float>(16.0 / 9.0); s->samples_per_pixel = 100;
  s->max_bounces = 40; s->lookfrom = Vd(0, 0.9, 0.75); s->lookat = Vd(0, 0.5, -1);
  s->background = V(0, 0, 0);
  set_name(s, "lighttest.ppm");
}

static const char *kSceneNames[RT_SCENE_COUNT] = {
    "fv1", "cornell_box", "bouncing_spheres", "final", "fv2", "fv3", "fv4", "fv5",
    "refract1", "refract2", "refract3", "refract4", "refract5", "motion_blur", "light_test",
    "checkered_spheres", "earth", "perlin_spheres", "quads", "simple_light", "random_10k"};

const char *rt_scene_name(int index) {
  return (index >= 0 && index < RT_SCENE_COUNT) ? kSceneNames[index] : nullptr;
}

int rt_world_build_scene(rt_world *w, int index, rt_settings *s) {
  if (!w || !s) return RT_ERR_INVALID_ARG;
  rt_settings_default(s);
  switch (index) {
    case 0: scene_fv1(w, s); break;
    case 1: scene_cornell(w, s); break;
    case 2: scene_bouncing(w, s, 11); break;
    case 3: scene_final(w, s); break;
    case 4: scene_metal(w, s, 0.0f, "fv2.ppm"); break;
    case 5: scene_metal(w, s, static_cast<float>(0.2), "fv3.ppm"); break;
    case 6: scene_metal(w, s, static_cast<float>(0.5), "fv4.ppm"); break;
    case 7: scene_metal(w, s, 1.0f, "fv5.ppm"); break;
    case 8: scene_refract(w, s, 1.0f, "refract1.ppm"); break;
    case 9: scene_refract(w, s, static_cast<float>(1.05), "refract2.ppm"); break;
    case 10: scene_refract(w, s, static_cast<float>(1.333), "refract3.ppm"); break;
    case 11: scene_refract(w, s, static_cast<float>(1.5), "refract4.ppm"); break;
    case 12: scene_refract(w, s, static_cast<float>(2.417), "refract5.ppm"); break;
    case 13: scene_motion_blur(w, s); break;
    case 14: scene_light_test(w, s); break;
    case 15: scene_checkered(w, s); break;
    case 16: scene_earth(w, s); break;
    case 17: scene_perlin(w, s); break;
    case 18: scene_quads(w, s); break;
    case 19: scene_simple_light(w, s); break;
    case RT_SCENE_RANDOM_10K:
      scene_bouncing(w, s, 50);
      set_name(s, "random_10k.ppm");
      break;
    default: return RT_ERR_INVALID_ARG;
  }
  return rt_world_status(w);
}

// ---- camera (raytracing.cu:1657-1692) ----
int rt_camera_from_settings(const rt_settings *s, int32_t width, int32_t height, rt_camera *cam,
                            int32_t *out_w, int32_t *out_h) {
  if (!s || !cam) return RT_ERR_INVALID_ARG;
  int32_t W = width > 0 ? width : s->img_width;
  int32_t H = height > 0 ? height : static_cast<int32_t>(W / s->img_ratio);
  if (W <= 0 || H <= 0) return RT_ERR_INVALID_ARG;
  float focus_dist = 10.0f;
  float theta = s->vfov * (kPi / 180.0f);
  float h = tanf(theta / 2.0f);
  float viewport_height = 2.0f * h * focus_dist;
  float viewport_ratio = static_cast<float>(W) / static_cast<float>(H);
  float viewport_width = viewport_height * viewport_ratio;
  rtr_vec3 camera_pos = s->lookfrom;
  rtr_vec3 cam_w = unit(sub(s->lookfrom, s->lookat));
  rtr_vec3 cam_u = unit(cross(s->view_up, cam_w));
  rtr_vec3 cam_v = cross(cam_w, cam_u);
  rtr_vec3 viewport_v = scale(viewport_height, neg(cam_v));
  rtr_vec3 viewport_u = scale(viewport_width, cam_u);
  rtr_vec3 pdv = scale(1.0f / static_cast<float>(H), viewport_v);
  rtr_vec3 pdu = scale(1.0f / static_cast<float>(W), viewport_u);
  rtr_vec3 ulc = camera_pos;
  ulc = sub(ulc, scale(focus_dist, cam_w));
  ulc = sub(ulc, scale(0.5f, viewport_u));
  ulc = sub(ulc, scale(0.5f, viewport_v));
  float defocus_radius = focus_dist * tanf((s->defocus_angle / 2.0f) * kPi / 180.0f);
  rtr_vec3 pc = ulc;
  pc = add(pc, scale(0.5f, pdv));
  pc = add(pc, scale(0.5f, pdu));
  cam->pixel00 = pc;
  cam->delta_u = pdu;
  cam->delta_v = pdv;
  cam->center = camera_pos;
  cam->defocus_u = scale(defocus_radius, cam_u);
  cam->defocus_v = scale(defocus_radius, cam_v);
  cam->defocus_angle = s->defocus_angle;
  if (out_w) *out_w = W;
  if (out_h) *out_h = H;
  return RT_OK;
}

// ---- hit-stack size the reference allocates (raytracing.cu:1614-1647, 1735-1737) ----
static int32_t ref_depth(const rt_scene *sc, uint32_t href, int guard) {
  if (href >= sc->hittable_count || guard > 64) return 0;
  const rtr_hittable &h = sc->hittables[href];
  switch (h.kind) {
    case RTR_OBJ_SPHERE: case RTR_OBJ_TRIANGLE: case RTR_OBJ_QUAD: return 1;
    case RTR_OBJ_TRANSLATE: return 2 + ref_depth(sc, h.u.translate.child, guard + 1);
    case RTR_OBJ_YROTATE: return 2 + ref_depth(sc, h.u.yrotate.child, guard + 1);
    case RTR_OBJ_GROUP: return static_cast<int32_t>(h.u.group.size);
  }
  return 0;
}

int rt_reference_stack_depth(const rt_scene *sc, uint32_t *depth) {
  if (!sc || !depth || sc->ref_count == 0) return RT_ERR_INVALID_ARG;
  uint64_t d = static_cast<uint64_t>(logf(static_cast<float>(sc->ref_count)) / logf(2.0f) + 1);
  int32_t mx = 0;
  for (uint32_t i = 0; i < sc->ref_count; ++i) {
    int32_t c = ref_depth(sc, sc->refs[i], 0);
    if (c > mx) mx = c;
  }
  *depth = static_cast<uint32_t>(d + static_cast<uint64_t>(mx));
  return RT_OK;
}

// ---- tonemap + PPM (raytracing.cu:1391-1436, utility.h:43-49) ----
static inline float linear_to_gamma(float c) { return c > 0 ? sqrtf(c) : 0.0f; }
static inline float clampf(float v, float lo, float hi) { if (v < lo) return lo; if (v > hi) return hi; return v; }

void rt_tonemap(const float *rgb, size_t pixels, uint8_t *out) {
  for (size_t i = 0; i < 3 * pixels; ++i)
    out[i] = static_cast<uint8_t>(256 * clampf(linear_to_gamma(rgb[i]), 0.0f, 0.999f));
}

int rt_write_ppm(const char *path, const float *rgb, uint32_t width, uint32_t height) {
  if (!path || !rgb) return RT_ERR_INVALID_ARG;
  FILE *f = std::fopen(path, "wb");
  if (!f) return RT_ERR_INVALID_ARG;
  std::fprintf(f, "P6\n%u %u\n255\n", width, height);
  std::vector<uint8_t> bytes(static_cast<size_t>(width) * height * 3);
  rt_tonemap(rgb, static_cast<size_t>(width) * height, bytes.data());
  size_t n = std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
  return n == bytes.size() ? RT_OK : RT_ERR_INVALID_ARG;
}

#ifndef RT_SOURCE_HASH
#define RT_SOURCE_HASH "unstamped"
#define RT_SOURCE_FILES ""
#endif
// the sources this library was built from and the hash of their bytes (Makefile `stamp`; checked by _abi.py)
const char *rt_host_build_hash(void) { return RT_SOURCE_HASH; }
const char *rt_host_build_files(void) { return RT_SOURCE_FILES; }

int rt_abi_struct_sizes(uint32_t *out, int n) {
  const uint32_t v[8] = {sizeof(rt_scene), sizeof(rt_camera), sizeof(rt_params), sizeof(rt_stats),
                         sizeof(rt_settings), sizeof(rtr_hittable), sizeof(rtr_material), sizeof(rtr_texture)};
  if (!out || n < 0) return RT_ERR_INVALID_ARG;
  for (int i = 0; i < n && i < 8; ++i) out[i] = v[i];
  return 8;
}

}  // extern "C"
