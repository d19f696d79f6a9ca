// gpu_scene.h — the compiled scene the render kernels read (host side).
//
// The reference walks 120-byte tagged-union records and byte-addressed textures in global memory
// (raytracing.cu:1079-1251, 299-302).  scene_compile.cpp rewrites them once per scene into fixed
// 80-byte nodes (record indices preserved, WorldRefs resolved), deduplicated material / texture
// tables and a Perlin pool (word layout: device/rt_layout.h).  Every float is copied bit-for-bit;
// derived values (1/r, r*r, resolved refs) are computed with the same single IEEE op the reference
// performs per visit, so the kernels' results are unchanged.  Small scenes are staged into LDS whole.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "device/rt_layout.h"

namespace rt {

struct SceneImage {
  // one contiguous word image: [nodes | mats | texs | constant colour records | perlin | image pixels]
  std::vector<uint32_t> words;
  uint32_t node_count = 0, mat_count = 0, tex_count = 0, perlin_count = 0;
  uint32_t rec_consts = 0;      // colour-record index of the first constant (= mat_count + tex_count)
  uint32_t off_mats = 0, off_texs = 0, off_perlin = 0, off_pixels = 0;   // word offsets
  uint32_t root = 0;            // root record index (already resolved through the ref list)
  uint32_t stack_need = 0;      // exact worst-case hit-stack depth
  bool needs_uv = false;        // some image texture has pixels => sphere u,v must be computed
  bool has_noise = false;
};

// SAH BVH over the spheres of an all-sphere world (sphere_accel.cpp; word layout: device/rt_layout.h)
struct SphereAccel {
  std::vector<uint32_t> node_words, prim_words;
  uint32_t root = 0, depth = 0, spheres = 0;
  // the same tree 4 wide (accel::collapse_wide, rt_layout.h kAccel4*): root = node 0; wide_stack bounds the
  // ordered walk's stack (up to 3 pushes per level)
  std::vector<uint32_t> wide_words;
  std::vector<uint32_t> wide_q_words;   // the same nodes quantised (accel::quantize_wide; empty: not quantisable)
  uint32_t wide_depth = 0, wide_stack = 0;
};
// false (with a reason) when the world is not an all-sphere BVH/group tree with >= min_spheres spheres
bool build_sphere_accel(const SceneImage &img, uint32_t min_spheres, SphereAccel *out, std::string *why);

// Verified traversal of mixed worlds (mixed_accel.cpp): SAH trees of the macro roots' transform-free
// primitives.  build_mixed_accel also writes W_MACRO / W_XFBOX into `img`'s node words.
struct MixedAccel {
  std::vector<uint32_t> node_words, prim_words;
  uint32_t macros = 0, dynamic = 0, prims = 0, depth = 0, packed = 0;   // packed: sphere chains (kChainPacked)
};
// false (with a reason) when no node qualifies (e.g. a world of transforms only)
bool build_mixed_accel(SceneImage *img, MixedAccel *out, std::string *why);

// Returns RT_OK or RT_ERR_SCENE / RT_ERR_UNSUPPORTED.
int compile_scene(const void *scene /* const rt_scene* */, SceneImage *out);

// Scene-specialised traversal: HIP source of `struct StaticTrace` (the scene's DFS expanded into
// straight-line code with node data as immediates).  Returns false when the expansion would exceed
// max_visits node visits (large scenes keep the generic kernels).  fold: emit the exactly-folded
// primitive tests (scene_codegen.cpp header); *folded reports whether folding was applied.
bool generate_static_trace(const SceneImage &img, uint32_t max_visits, bool fold, std::string *src, uint32_t *visits,
                           bool *folded);

}  // namespace rt
