// rt_kernels.h — launch interface between the C-ABI (rt_capi.cpp) and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "device/rt_layout.h"
#include "device/prim_lists.h"

namespace rt {

constexpr uint32_t kLdsSceneMaxWords = 12 * 1024;   // stage scenes up to 48 KiB in LDS
constexpr uint32_t kPacketMaxNodes = 512;           // packet DFS only for scenes up to this size

hipError_t launch_seed(const SeedArgs &a, hipStream_t s);
// pixels_to_ppm byte conversion of n floats (3 per pixel) on the device
hipError_t launch_tonemap(const float *rgb, uint64_t n, uint8_t *out, hipStream_t s);
// tile-major render output (kVarTiledOut: tile t at 192 t floats) -> row-major floats [rows][width][3] and, if out8,
// the PPM bytes of the same floats
hipError_t launch_untile(const float *tiled, float *out, uint8_t *out8, uint32_t rows, uint32_t width, uint32_t tiles_x,
                         uint32_t ts, hipStream_t s);
// longest-first order of n tiles from probe costs (single block)
// tiles_x != 0: grouped into 8 XCD classes (128-pixel column groups of 8x8 tiles), longest-first within each;
// order[n .. n + 8] = the classes' first positions and n (order must hold n + 9 words)
hipError_t launch_order(const uint32_t *cost, uint32_t n, uint32_t *order, uint32_t tiles_x, hipStream_t s);
hipError_t launch_render(const RenderArgs &a, int variant, uint32_t blocks, size_t lds_bytes, hipStream_t s);
// primary-ray candidate lists of the verified sphere walk, one per 8x8 tile of the shard (device/prim_lists.h)
// (entries of `words` = kPrimEntryWords words: SAH prim index and axial bound, rt_layout.h kPrimEntry*)
hipError_t launch_prim_lists(const PrimListGeom &g, const uint32_t *nodes, uint32_t root, const uint32_t *prims,
                             uint32_t n_tiles, uint32_t cap, uint32_t words, uint32_t *lists, uint32_t *counts,
                             hipStream_t s);
// multi-device frames: frame row k <- row k / n of shard k % n in src ([n][max_rows][row_bytes])
hipError_t launch_unpermute(const void *src, void *dst, uint32_t rows, uint32_t n, uint32_t max_rows,
                            uint32_t row_bytes, hipStream_t s);
// resident 256-thread blocks per CU for the chosen variant (occupancy query)
int render_blocks_per_cu(int variant, size_t lds_bytes);
// VGPRs and scratch bytes per lane of the offline render kernel of `variant` (false: unknown variant)
bool render_kernel_attrs(int variant, int *vgprs, int *scratch);

}  // namespace rt
