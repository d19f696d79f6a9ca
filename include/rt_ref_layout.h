/*
 * rt_ref_layout.h — the reference renderer's scene bytes, described as a wire format.
 *
 * The hot path of luk-zm/cuda_raytracing reads three host-built arrays (copied H2D at
 * src/raytracing.cu:1699-1733):
 *   - a flat array of 120-byte tagged-union scene records  (`Hittable`, raytracing.cu:182-193)
 *   - a u16 indirection list WorldRef -> record index       (`HittableRefList`, raytracing.cu:1-7)
 *   - a byte arena of textures addressed by byte offset     (`TextureList`, raytracing.cu:56-59,263-302)
 *
 * These structs restate that layout (x86-64 natural alignment, as nvcc's host compiler lays it
 * out) so a caller can hand the reference's own buffers to rt_render() unchanged.  They are a
 * byte-level contract only; field names are ours.  Static asserts pin every size and offset.
 */
#ifndef RT_REF_LAYOUT_H
#define RT_REF_LAYOUT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* vec3.h:4-8 */
typedef struct { float x, y, z; } rtr_vec3;

/* raytracing.cu:61-65 */
typedef struct { float x0, x1, y0, y1, z0, z1; } rtr_aabb;

/* raytracing.cu:15-17 — byte offset of a texture record inside the arena */
typedef struct { uint64_t offset; } rtr_texref;

/* raytracing.cu:38-44 */
enum { RTR_TEX_SOLID = 0, RTR_TEX_CHECKER = 1, RTR_TEX_IMAGE = 2, RTR_TEX_NOISE = 3 };

/* raytracing.cu:46-54 (32 bytes; may sit at any byte offset of the arena, memory.h:30-38) */
typedef struct {
  uint32_t kind;
  uint32_t pad_;
  union {
    rtr_vec3 solid;                                          /* SolidColor   :9-11  */
    struct { float inv_scale; uint32_t pad_; rtr_texref even, odd; } checker;   /* :19-23 */
    struct { uint64_t host_pixels; uint64_t pixels_offset; int32_t width, height; } image; /* :25-30 */
    struct { uint64_t host_table; uint64_t table_offset; float scale; uint32_t pad_; } noise;  /* :32-36 */
  } u;
} rtr_texture;

/* perlin_noise.h:4-10 (6144 bytes, stored inline after its noise texture record, raytracing.cu:280-287) */
#define RTR_PERLIN_POINTS 256
typedef struct {
  rtr_vec3 gradients[RTR_PERLIN_POINTS];
  int32_t perm_x[RTR_PERLIN_POINTS];
  int32_t perm_y[RTR_PERLIN_POINTS];
  int32_t perm_z[RTR_PERLIN_POINTS];
} rtr_perlin;

/* raytracing.cu:78-84 */
enum { RTR_MAT_LAMBERTIAN = 0, RTR_MAT_METAL = 1, RTR_MAT_DIELECTRIC = 2, RTR_MAT_DIFFUSE_LIGHT = 3 };

/* raytracing.cu:86-99 (24 bytes) */
typedef struct {
  uint32_t kind;
  uint32_t pad_;
  union {
    rtr_texref lambert_tex;
    struct { rtr_vec3 albedo; float fuzz; } metal;
    struct { float ior; } dielectric;
    rtr_texref light_tex;
  } u;
} rtr_material;

/* raytracing.cu:107-112 (80 bytes) — centre(t) = centre + t * motion */
typedef struct {
  rtr_vec3 center;
  rtr_vec3 motion;
  float radius;
  uint32_t pad_;
  rtr_material mat;
  rtr_aabb box;
} rtr_sphere;

/* raytracing.cu:114-121 (64 bytes) */
typedef struct {
  rtr_vec3 q, u, v;
  float d;
  rtr_vec3 w;
  rtr_vec3 normal;
} rtr_plane;

/* raytracing.cu:123-133 (112 bytes; quads and triangles share it) */
typedef struct {
  rtr_plane geom;
  rtr_material mat;
  rtr_aabb box;
} rtr_planar;

/* raytracing.cu:138-142 — children are WorldRefs (indices into the u16 ref list) */
typedef struct { uint16_t left, right; rtr_aabb box; } rtr_bvh;

/* raytracing.cu:169-173 */
typedef struct { uint16_t child; uint16_t pad_; rtr_vec3 offset; rtr_aabb box; } rtr_translate;

/* raytracing.cu:175-180 */
typedef struct { uint16_t child; uint16_t pad_; float sin_theta, cos_theta; rtr_aabb box; } rtr_yrotate;

/* raytracing.cu:162-167 — `count` consecutive records starting at `first` */
typedef struct { uint16_t first; uint16_t pad_; rtr_aabb box; uint64_t size; uint64_t count; } rtr_group;

/* raytracing.cu:144-153 */
enum {
  RTR_OBJ_SPHERE = 0, RTR_OBJ_BVH = 1, RTR_OBJ_TRIANGLE = 2, RTR_OBJ_QUAD = 3,
  RTR_OBJ_TRANSLATE = 4, RTR_OBJ_YROTATE = 5, RTR_OBJ_GROUP = 6
};

/* raytracing.cu:182-193 (120 bytes) */
typedef struct {
  uint32_t kind;
  uint32_t pad_;
  union {
    rtr_sphere sphere;
    rtr_bvh bvh;
    rtr_planar planar;       /* triangle or quad */
    rtr_translate translate;
    rtr_yrotate yrotate;
    rtr_group group;
  } u;
} rtr_hittable;

#define RTR_STATIC_ASSERT(c, m) typedef char rtr_static_assert_##m[(c) ? 1 : -1]
RTR_STATIC_ASSERT(sizeof(rtr_texture) == 32, texture_size);
RTR_STATIC_ASSERT(sizeof(rtr_perlin) == 6144, perlin_size);
RTR_STATIC_ASSERT(sizeof(rtr_material) == 24, material_size);
RTR_STATIC_ASSERT(sizeof(rtr_sphere) == 80, sphere_size);
RTR_STATIC_ASSERT(offsetof(rtr_sphere, mat) == 32, sphere_mat_off);
RTR_STATIC_ASSERT(sizeof(rtr_plane) == 64, plane_size);
RTR_STATIC_ASSERT(offsetof(rtr_plane, w) == 40, plane_w_off);
RTR_STATIC_ASSERT(sizeof(rtr_planar) == 112, planar_size);
RTR_STATIC_ASSERT(offsetof(rtr_planar, box) == 88, planar_box_off);
RTR_STATIC_ASSERT(sizeof(rtr_bvh) == 28, bvh_size);
RTR_STATIC_ASSERT(sizeof(rtr_translate) == 40, translate_size);
RTR_STATIC_ASSERT(sizeof(rtr_yrotate) == 36, yrotate_size);
RTR_STATIC_ASSERT(sizeof(rtr_group) == 48, group_size);
RTR_STATIC_ASSERT(sizeof(rtr_hittable) == 120, hittable_size);
RTR_STATIC_ASSERT(offsetof(rtr_hittable, u) == 8, hittable_union_off);

#ifdef __cplusplus
}
#endif
#endif /* RT_REF_LAYOUT_H */
