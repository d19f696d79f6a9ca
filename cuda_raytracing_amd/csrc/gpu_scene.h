// gpu_scene.h — the compiled scene the render kernel reads (host <-> device shared layout).
//
// The reference walks 120-byte tagged-union records and byte-addressed textures in global memory
// (raytracing.cu:1079-1251, 299-302).  scene_compile.cpp rewrites them once per scene into fixed
// 80-byte nodes (record indices preserved, WorldRefs resolved), deduplicated material / texture
// tables and a Perlin pool.  Every float is copied bit-for-bit; derived values (1/r, r*r, resolved
// refs) are computed with the same single IEEE op the reference performs per visit, so the kernel's
// results are unchanged.  Small scenes are staged into LDS whole (one contiguous word image).
#pragma once
#include <cstdint>
#include <vector>

namespace rt {

// node kinds == reference VisObject values (raytracing.cu:144-153)
enum : uint32_t {
  K_SPHERE = 0, K_BVH = 1, K_TRIANGLE = 2, K_QUAD = 3, K_TRANSLATE = 4, K_YROTATE = 5, K_GROUP = 6
};

constexpr int kNodeWords = 20;   // 80 bytes
// word layout per kind (w0 = kind, w1 = aux):
//   BVH      : w1 = left_href | right_href << 16, w2..w7 = x0 x1 y0 y1 z0 z1
//   SPHERE   : w1 = material, w2..4 centre, w5..7 motion, w8 radius, w9 radius*radius, w10 1/radius
//   TRI/QUAD : w1 = material, w2..4 normal, w5 d, w6..8 q, w9..11 u, w12..14 v, w15..17 w
//   TRANSLATE: w1 = child, w2..4 offset
//   YROTATE  : w1 = child, w2 sin, w3 cos
//   GROUP    : w1 = first child, w2 = count
enum : int {
  W_KIND = 0, W_AUX = 1,
  W_BOX = 2,
  W_CENTER = 2, W_MOTION = 5, W_RADIUS = 8, W_RADIUS2 = 9, W_INV_RADIUS = 10,
  W_NORMAL = 2, W_D = 5, W_Q = 6, W_U = 9, W_V = 12, W_W = 15,
  W_OFFSET = 2, W_SIN = 2, W_COS = 3, W_COUNT = 2,
};

// materials (raytracing.cu:78-99): 8 words
constexpr int kMatWords = 8;
enum : int { M_KIND = 0, M_TEX = 1, M_ALBEDO = 2, M_FUZZ = 5, M_IOR = 6 };

// textures (raytracing.cu:38-54): 8 words
constexpr int kTexWords = 8;
enum : uint32_t { T_SOLID = 0, T_CHECKER = 1, T_IMAGE = 2, T_NOISE = 3 };
enum : int {
  T_KIND = 0,
  T_RGB = 1,                                         // solid: w1..3
  T_EVEN = 1, T_ODD = 2, T_INV_SCALE = 3,            // checker
  T_PERLIN = 1, T_NOISE_SCALE = 3,                   // noise: perlin table index, scale
  T_WIDTH = 1, T_HEIGHT = 2, T_PIXELS = 3, T_HAS_PIXELS = 4,   // image: pixel word offset into pool
};

// Perlin table: 256 gradients as float4 (xyz, pad) + 256 perm_x bytes (perm_y/z are never read,
// perlin_noise.cpp:37-39)
constexpr int kPerlinWords = 256 * 4 + 64;

struct SceneImage {
  // one contiguous word image: [nodes | mats | texs | perlin | image pixels]
  std::vector<uint32_t> words;
  uint32_t node_count = 0, mat_count = 0, tex_count = 0, perlin_count = 0;
  uint32_t off_mats = 0, off_texs = 0, off_perlin = 0, off_pixels = 0;   // word offsets
  uint32_t root = 0;            // root record index (already resolved through the ref list)
  uint32_t stack_need = 0;      // exact worst-case hit-stack depth
  bool needs_uv = false;        // some image texture has pixels => sphere u,v must be computed
  bool has_noise = false;
};

// Returns RT_OK or RT_ERR_SCENE / RT_ERR_STACK.
struct rt_scene_view;
int compile_scene(const void *scene /* const rt_scene* */, SceneImage *out);

}  // namespace rt
