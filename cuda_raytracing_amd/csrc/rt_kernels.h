// rt_kernels.h — launch interface between the C-ABI (rt_capi.cpp) and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rt {

constexpr int kBlock = 256;        // 4 waves of 64
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int kChunk = 64;         // pixels handed to a wave per work-queue grab
constexpr uint32_t kLdsSceneMaxWords = 12 * 1024;   // stage scenes up to 48 KiB in LDS

struct RenderArgs {
  const uint32_t *scene;      // SceneImage::words in HBM
  uint32_t scene_words;
  uint32_t off_mats, off_texs, off_perlin, off_pixels, pixel_words;
  uint32_t root, stack_cap, stack_lds_word;   // stack region starts at this LDS word
  uint32_t needs_uv;
  // camera (rt_camera)
  float p00[3], du[3], dv[3], center[3], dfu[3], dfv[3], defocus_angle;
  int32_t width, row_offset, row_stride;
  int32_t spp, max_bounces;
  float bg[3];
  float sample_scale;
  uint32_t n_pixels;          // row_count * width (local pixels of this shard)
  const uint32_t *rng;        // [6][n_pixels] seeded XORWOW states {d, x0..x4}
  float *out;                 // [n_pixels][3]
  float *rc;                  // attenuation stack: [max_bounces][3][threads]
  uint32_t threads;           // grid size in threads (rc stride)
  uint32_t *work;             // chunk counter (zeroed per launch)
  unsigned long long *counters;   // RT_CNT__COUNT (RT_FLAG_COUNT only)
};

struct SeedArgs {
  const uint32_t *jump;       // xorwow_jump_tables() on device
  uint32_t base[6];           // rocRAND constant seeding of `seed`
  int32_t width, row_offset, row_stride;
  uint32_t n_pixels;
  uint32_t per_thread;
  uint32_t *rng;              // [6][n_pixels]
};

hipError_t launch_seed(const SeedArgs &a, hipStream_t s);
// lds: stage the scene in LDS; count: collect counters
hipError_t launch_render(const RenderArgs &a, bool lds, bool count, uint32_t blocks, size_t lds_bytes,
                         hipStream_t s);
// resident 256-thread blocks per CU for the chosen variant (occupancy query)
int render_blocks_per_cu(bool lds, bool count, size_t lds_bytes);

}  // namespace rt
