/*
 * rt_host.h — host side of the path: scene builder, BVH, camera, tonemap/PPM.
 *
 * These stay on the CPU exactly as in luk-zm/cuda_raytracing; they produce
 * the scene bytes (rt_ref_layout.h) and camera values (rt_render.h) the device path consumes.
 * Everything here reproduces the reference's host arithmetic and its glibc rand() draw order
 * (utility.h:26-41, never srand-ed => seed 1) so scene bytes are identical to the reference's.
 */
#ifndef RT_HOST_H
#define RT_HOST_H

#include <stdint.h>
#include <stddef.h>
#include "rt_ref_layout.h"
#include "rt_render.h"

#ifdef __cplusplus
extern "C" {
#endif

/* RenderSettings (raytracing.cu:1509-1521); img_name is stored inline. */
typedef struct rt_settings {
  float img_ratio;
  int32_t img_width;
  int32_t samples_per_pixel;
  int32_t max_bounces;
  float vfov;
  rtr_vec3 lookfrom, lookat, view_up;
  float defocus_angle;
  rtr_vec3 background;
  char img_name[64];
} rt_settings;

/* Scene catalog indices: 0..19 as main.cu:52-117; 20 = the 10k-sphere scene (BASELINE config 4). */
#define RT_SCENE_COUNT 21
#define RT_SCENE_RANDOM_10K 20
const char *rt_scene_name(int index);

typedef struct rt_world rt_world;

/* capacity: max scene records and refs (reference WORLD_SIZE, main.cu:24; 8000 there).
 * arena_bytes: texture arena size (10 MB in the reference, main.cu:36).
 * Each world owns a fresh glibc-rand stream seeded with 1 (the reference never calls srand). */
rt_world *rt_world_create(uint32_t capacity, uint64_t arena_bytes);
void rt_world_destroy(rt_world *w);

/* settings <- g_default_render_settings (raytracing.cu:1527-1529) */
void rt_settings_default(rt_settings *s);
/* Build catalog scene `index` into an empty world and apply its settings (main.cu:50-117). */
int rt_world_build_scene(rt_world *w, int index, rt_settings *settings);
/* make_bvh (raytracing.cu:902-906) over the refs added so far; returns the root WorldRef. */
int rt_world_build_bvh(rt_world *w, uint16_t *root);
/* View of the world's buffers (valid until the world is modified or destroyed). */
int rt_world_scene(const rt_world *w, uint16_t root, rt_scene *out);
uint32_t rt_world_hittable_count(const rt_world *w);
uint32_t rt_world_ref_count(const rt_world *w);
uint64_t rt_world_texture_bytes(const rt_world *w);
/* RT_OK, RT_ERR_SCENE (capacity or arena exhausted) or RT_ERR_UNSUPPORTED (undecodable image file) */
int rt_world_status(const rt_world *w);
/* raw glibc rand() from the world's stream (tests) */
int32_t rt_world_rand(rt_world *w);

/* ---- scene builder API (raytracing.cu:1775-1977); materials are returned by value ---- */
rtr_material rt_mat_lambert_solid(rt_world *w, rtr_vec3 albedo);                 /* :1805 */
rtr_material rt_mat_light_solid(rt_world *w, rtr_vec3 color);                    /* :1813 */
/* :1821.  Loads the file like stbi_loadf(file, .., 3) (rt_image_load).  A missing, unknown or corrupt file
 * is the reference's failed load (magenta texture); should rt_image_load ever report RT_ERR_UNSUPPORTED,
 * the world's status says so (rt_world_status, returned by rt_world_build_scene). */
rtr_material rt_mat_lambert_image(rt_world *w, const char *file_name);
/* an image texture whose load succeeded: width*height float RGB texels (stbi_loadf layout, row 0 first) */
rtr_material rt_mat_lambert_image_pixels(rt_world *w, const float *rgb, int32_t width, int32_t height);
rtr_material rt_mat_lambert_noise(rt_world *w, float scale);                     /* :1829 */
rtr_material rt_mat_metal(rtr_vec3 albedo, float fuzz);                          /* :516 */
rtr_material rt_mat_dielectric(float ior);                                       /* :524 */
rtr_material rt_mat_lambert_checker(rt_world *w, float scale, rtr_vec3 even, rtr_vec3 odd); /* :1846 */

/* transform: 0 none, 1 translate, 2 y-rotate, 3 y-rotate then translate (world_add*, :1776-1803) */
enum { RT_XF_NONE = 0, RT_XF_TRANSLATE = 1, RT_XF_YROTATE = 2, RT_XF_YROTATE_TRANSLATE = 3 };
int rt_add_sphere(rt_world *w, int xf, float angle, rtr_vec3 offset,
                  rtr_vec3 center, float radius, rtr_material mat);
int rt_add_moving_sphere(rt_world *w, int xf, float angle, rtr_vec3 offset,
                         rtr_vec3 center, rtr_vec3 motion, float radius, rtr_material mat);
int rt_add_quad(rt_world *w, int xf, float angle, rtr_vec3 offset,
                rtr_vec3 q, rtr_vec3 u, rtr_vec3 v, rtr_material mat);
int rt_add_triangle(rt_world *w, int xf, float angle, rtr_vec3 offset,
                    rtr_vec3 q, rtr_vec3 u, rtr_vec3 v, rtr_material mat);
int rt_add_box(rt_world *w, int xf, float angle, rtr_vec3 offset,
               rtr_vec3 a, rtr_vec3 b, rtr_material mat);
int rt_add_pyramid(rt_world *w, int xf, float angle, rtr_vec3 offset,
                   rtr_vec3 base_a, rtr_vec3 base_b, rtr_vec3 tip, rtr_material mat);

/* ---- image files (make_image_texture's stbi_loadf, raytracing.cu:332-341) ----
 * *rgb = width*height float RGB texels, row 0 = top, as stb_image v2.30's stbi_loadf(path, .., 3) returns
 * them: JPEG (baseline + progressive), PNG, BMP, TGA, GIF (first image), Photoshop PSD (RGB), Softimage
 * PIC, binary PNM with 8-bit channels as powf(c/255, 2.2), Radiance HDR as stored; free with rt_image_free.
 * Returns RT_OK or RT_IMAGE_MISSING (no such file, or a file stb would fail to load: the reference's failed
 * load, a magenta texture). */
#define RT_IMAGE_MISSING 1
int rt_image_load(const char *path, float **rgb, int32_t *width, int32_t *height);
void rt_image_free(float *rgb);

/* ---- camera (raytracing.cu:1657-1692).  width/height <= 0 => reference rule
 * W = settings.img_width, H = (int)(W / img_ratio) (:1659-1660). ---- */
int rt_camera_from_settings(const rt_settings *s, int32_t width, int32_t height,
                            rt_camera *cam, int32_t *out_width, int32_t *out_height);

/* hit-stack size the reference allocates: (u64)(logf(refs)/logf(2)+1) + world_max_depth (:1735-1737) */
int rt_reference_stack_depth(const rt_scene *scene, uint32_t *depth);

/* ---- output (raytracing.cu:1391-1436) ---- */
void rt_tonemap(const float *rgb, size_t pixels, uint8_t *out_rgb8);
int rt_write_ppm(const char *path, const float *rgb, uint32_t width, uint32_t height);

/* sizes of the ABI structs as compiled (bindings check their mirrors against these):
 * [rt_scene, rt_camera, rt_params, rt_stats, rt_settings, rtr_hittable, rtr_material, rtr_texture] */
int rt_abi_struct_sizes(uint32_t *out, int n);
/* Build stamp of this library (see rt_hip_build_hash in rt_render.h) */
const char *rt_host_build_hash(void);
const char *rt_host_build_files(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HOST_H */
