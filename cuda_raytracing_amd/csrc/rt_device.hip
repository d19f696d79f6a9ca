// rt_device.hip — offline-compiled MI355X (gfx950) kernels: generic render variants + RNG seeding.
//
// The render body lives in device/rt_body.h (shared with the scene-specialised kernels that rt_jit.cpp
// compiles at run time).  Here it is instantiated with the two scene-independent traversal policies:
//   LaneTrace   per-lane DFS over a lane-interleaved LDS stack (any scene size)
//   PacketTrace one DFS per wave with per-entry lane masks (scalar node loads, uniform branches)
// and the variant bits of rt_layout.h (LDS staging, counters, noise textures, image u,v).
#include <hip/hip_runtime.h>

#include "device/rt_body.h"
#include "rt_kernels.h"
#include "xorwow_jump.h"

namespace rt {

template <int F>
__global__ __launch_bounds__(kBlock) void render_kernel(RenderArgs A) {
  if constexpr ((F & kVarPacket) != 0) render_body<F, PacketTrace>(A);
  else render_body<F, LaneTrace>(A);
}

namespace {

// ---------------------------------------------------------------------------------------------
// RNG seeding (init_gpu_data's curand_init, :1591-1606): state(i) = J^i * s0, i = global pixel
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void jump_apply(const uint32_t *__restrict__ M, uint32_t &x0, uint32_t &x1, uint32_t &x2,
                                           uint32_t &x3, uint32_t &x4) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
  const uint32_t xs[5] = {x0, x1, x2, x3, x4};
#pragma unroll
  for (int w = 0; w < 5; ++w) {
    const uint32_t xw = xs[w];
#pragma unroll 8
    for (int b = 0; b < 32; ++b) {
      const uint32_t *row = M + (w * 32 + b) * 5;
      const uint32_t msk = 0u - ((xw >> b) & 1u);
      r0 ^= msk & row[0]; r1 ^= msk & row[1]; r2 ^= msk & row[2]; r3 ^= msk & row[3]; r4 ^= msk & row[4];
    }
  }
  x0 = r0; x1 = r1; x2 = r2; x3 = r3; x4 = r4;
}

// P_0 x by its nibble table in LDS (xorwow_jump.h): 40 lookups of 5 words, XOR-summed — the same
// GF(2) product as jump_apply(P_0) in ~1/7 of its operations
__device__ __forceinline__ void jump_next(const uint4 *__restrict__ lo, const uint32_t *__restrict__ hi, uint32_t &x0,
                                          uint32_t &x1, uint32_t &x2, uint32_t &x3, uint32_t &x4) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
  const uint32_t xs[5] = {x0, x1, x2, x3, x4};
#pragma unroll
  for (int w = 0; w < 5; ++w)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint32_t e = (w * 8 + q) * 16 + ((xs[w] >> (4 * q)) & 15u);
      const uint4 a = lo[e];
      r0 ^= a.x; r1 ^= a.y; r2 ^= a.z; r3 ^= a.w; r4 ^= hi[e];
    }
  x0 = r0; x1 = r1; x2 = r2; x3 = r3; x4 = r4;
}

// Thread t seeds a run of kSeedRun = 16 consecutive pixels of one row (one jump, then P_0 steps): the
// row segments of two horizontally adjacent 8x8 tiles.  Threads are ordered (8-row band, run, row in
// band), so the 8 rows of a run are consecutive lanes.  The 16 states stay in registers until the run is
// done; then each lane stores its two 32-B tile-row segments per state word as 16-B vector stores, and
// the 8 lanes of a run together write each tile's 256 contiguous bytes (two whole 128-B lines) in one
// store instruction.  (Storing each state as it was produced wrote one 4-B piece into 16 different
// lines per instruction: 3.3x the states' bytes reached HBM, profiles/r02_v8_traffic.)  Columns past the
// frame edge inside the last tile are written too (never read).
__global__ __launch_bounds__(kBlock) void seed_kernel(SeedArgs A) {
  __shared__ uint4 s_lo[kJumpNibbles * 16];
  __shared__ uint32_t s_hi[kJumpNibbles * 16];
  {
    const uint4 *glo = reinterpret_cast<const uint4 *>(A.jump + kJumpNibbleOffset);
    const uint32_t *ghi = A.jump + kJumpNibbleOffset + kJumpNibbles * 16 * 4;
    for (uint32_t i = threadIdx.x; i < kJumpNibbles * 16; i += kBlock) { s_lo[i] = glo[i]; s_hi[i] = ghi[i]; }
    __syncthreads();
  }
  static_assert(kSeedRun == 16, "a run is two tile rows");
  const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t W = static_cast<uint32_t>(A.width);
  const uint32_t runs = (W + kSeedRun - 1) / kSeedRun;
  const uint32_t band = t / (8u * runs), q = t - band * 8u * runs;
  const uint32_t lr = band * 8u + (q & 7u), j0 = (q >> 3) * kSeedRun;
  if (lr >= A.rows) return;
  uint32_t x0 = A.base[1], x1 = A.base[2], x2 = A.base[3], x3 = A.base[4], x4 = A.base[5];
  {
    const uint64_t g = static_cast<uint64_t>(A.row_offset + static_cast<int64_t>(lr) * A.row_stride) * W + j0;
    if (g & 1u) jump_next(s_lo, s_hi, x0, x1, x2, x3, x4);
    for (int k = 1; k < kJumpPowers; ++k)
      if ((g >> k) & 1u) jump_apply(A.jump + k * kJumpMatrixWords, x0, x1, x2, x3, x4);
  }
  const uint32_t n = A.n_ids;
  const uint32_t id0 = (lr >> 3) * A.tiles_x * 64u + (j0 >> 3) * 64u + (lr & 7u) * 8u;   // tile A, this row
  const bool second = (j0 >> 3) + 1u < A.tiles_x;                                          // tile B exists
  const uint4 d = make_uint4(A.base[0], A.base[0], A.base[0], A.base[0]);
  for (int h = 0; h < 2; ++h) {   // tile A's row segment, then tile B's
    if (h == 1 && !second) break;
    uint32_t st[5][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (h + j > 0) jump_next(s_lo, s_hi, x0, x1, x2, x3, x4);     // P_0: next global pixel in the row
      st[0][j] = x0; st[1][j] = x1; st[2][j] = x2; st[3][j] = x3; st[4][j] = x4;
    }
    const uint32_t id = id0 + h * 64u;
    *reinterpret_cast<uint4 *>(A.rng + id) = d;
    *reinterpret_cast<uint4 *>(A.rng + id + 4) = d;
#pragma unroll
    for (int w = 0; w < 5; ++w) {
      uint4 *o = reinterpret_cast<uint4 *>(A.rng + static_cast<size_t>(w + 1) * n + id);
      o[0] = make_uint4(st[w][0], st[w][1], st[w][2], st[w][3]);
      o[1] = make_uint4(st[w][4], st[w][5], st[w][6], st[w][7]);
    }
  }
}

// Longest-first tile order from the probe costs: bucket by cost (linear buckets of the max, descending), counting
// sort in LDS.  One block; ~32k tiles at 1080p.  Order inside a bucket is arbitrary — the schedule never changes what
// a lane computes.  XCD classes (tiles_x != 0): the tiles are first grouped by class — 8x8 tile (tx, ty) -> class
// ((tx >> 4) + (ty >> 2)) & 7, i.e. 128-pixel column groups shifted every 32 rows, so every 128-B line of the float
// frame and of the PPM bytes belongs to tiles of one class — then longest-first within the class (128 buckets each);
// order[n + q] = the first position of class q, order[n + 8] = n (the render kernel's per-XCD queues).
constexpr int kOrderThreads = 1024, kOrderBuckets = 1024, kOrderClasses = 8;
__global__ __launch_bounds__(kOrderThreads) void order_kernel(const uint32_t *cost, uint32_t n, uint32_t *order,
                                                              uint32_t tiles_x) {
  __shared__ uint32_t hist[kOrderBuckets];
  __shared__ uint32_t wmax[kOrderThreads / 64];
  __shared__ uint32_t wsum[kOrderThreads / 64];
  const uint32_t t = threadIdx.x;
  uint32_t m = 0;
  for (uint32_t i = t; i < n; i += kOrderThreads) m = max(m, cost[i]);
  for (int off = 32; off > 0; off >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(m, off)));
  if ((t & 63u) == 0) wmax[t >> 6] = m;
  for (uint32_t b = t; b < kOrderBuckets; b += kOrderThreads) hist[b] = 0;
  __syncthreads();
  uint32_t mx = 1;
  for (int w = 0; w < kOrderThreads / 64; ++w) mx = max(mx, wmax[w]);
  const uint32_t per = tiles_x ? kOrderBuckets / kOrderClasses : kOrderBuckets;   // cost buckets per class
  auto key = [&](uint32_t i) {
    const uint32_t b = static_cast<uint32_t>((static_cast<uint64_t>(cost[i]) * (per - 1)) / mx);
    uint32_t k = per - 1 - b;
    if (tiles_x) {
      const uint32_t ty = i / tiles_x, tx = i - ty * tiles_x;
      k += (((tx >> 4) + (ty >> 2)) & (kOrderClasses - 1)) * per;
    }
    return k;
  };
  for (uint32_t i = t; i < n; i += kOrderThreads) atomicAdd(&hist[key(i)], 1u);
  __syncthreads();
  // exclusive scan of the 1024 bucket counts (one per thread: wave prefix, then the 16 wave totals)
  const uint32_t v = hist[t];
  uint32_t incl = v;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = static_cast<uint32_t>(__shfl_up(static_cast<int>(incl), off));
    if ((t & 63u) >= static_cast<uint32_t>(off)) incl += u;
  }
  if ((t & 63u) == 63u) wsum[t >> 6] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < (t >> 6); ++w) before += wsum[w];
  __syncthreads();
  hist[t] = before + incl - v;
  __syncthreads();
  if (tiles_x && t <= kOrderClasses) order[n + t] = t < kOrderClasses ? hist[t * per] : n;
  __syncthreads();
  for (uint32_t i = t; i < n; i += kOrderThreads) order[atomicAdd(&hist[key(i)], 1u)] = i;
}

// linear -> 8-bit sRGB-ish bytes of pixels_to_ppm (raytracing.cu:1391-1395,1419-1431): sqrt gamma
// (0 for non-positive), clamp to [0, 0.999], (u8)(256 * x).  Each thread converts 4 consecutive
// floats (16-B load, 4-B store); HBM-bound (12 B in, 3 B out per pixel).
__global__ __launch_bounds__(256) void tonemap_kernel(const float *__restrict__ rgb, uint64_t n,
                                                      uint8_t *__restrict__ out) {
  const uint64_t i = (static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  auto byte = [](float c) -> uint32_t {
    const float g = c > 0 ? sqrtf(c) : 0.0f;
    const float k = (g < 0.0f) ? 0.0f : ((g > 0.999f) ? 0.999f : g);
    return static_cast<uint32_t>(256 * k) & 0xffu;
  };
  if (i + 4 <= n && (reinterpret_cast<uintptr_t>(rgb + i) & 15) == 0 && (reinterpret_cast<uintptr_t>(out + i) & 3) == 0) {
    const float4 v = *reinterpret_cast<const float4 *>(rgb + i);
    *reinterpret_cast<uint32_t *>(out + i) = byte(v.x) | (byte(v.y) << 8) | (byte(v.z) << 16) | (byte(v.w) << 24);
  } else {
    for (uint64_t k = i; k < n && k < i + 4; ++k) out[k] = static_cast<uint8_t>(byte(rgb[k]));
  }
}

// Tile-major render output (kVarTiledOut) -> the row-major float frame and, fused, the PPM bytes of the same floats.
// One block per band of one tile row x kUntileCols columns: its reads are whole tiles (one XCD's L2 fetches each tile
// line once) and its writes whole 128-B lines of the float rows (kUntileCols x 12 B) and of the byte rows (x 3 B).
constexpr uint32_t kUntileCols = 128;
__global__ __launch_bounds__(256) void untile_kernel(const float *__restrict__ tiled, float *__restrict__ out,
                                                     uint8_t *__restrict__ out8, uint32_t rows, uint32_t width,
                                                     uint32_t tiles_x, uint32_t ts) {
  const uint32_t tsh = 6u - ts, th = 1u << tsh, x0 = blockIdx.x * kUntileCols, y0 = blockIdx.y * th;
  for (uint32_t idx = threadIdx.x; idx < th * kUntileCols * 3u; idx += 256u) {
    const uint32_t r = idx / (kUntileCols * 3u), f = idx - r * (kUntileCols * 3u);
    const uint32_t j = f / 3u, c = f - 3u * j, x = x0 + j, y = y0 + r;
    if (x >= width || y >= rows) continue;
    const uint32_t tile = blockIdx.y * tiles_x + (x >> ts);
    const uint32_t k = (r << ts) | (x & ((1u << ts) - 1u));
    const float v = tiled[static_cast<size_t>(tile) * 192u + 3u * k + c];
    const size_t e = (static_cast<size_t>(y) * width + x) * 3u + c;
    out[e] = v;
    if (out8) {
      const float g = v > 0 ? sqrtf(v) : 0.0f;
      const float q = (g < 0.0f) ? 0.0f : ((g > 0.999f) ? 0.999f : g);
      out8[e] = static_cast<uint8_t>(static_cast<uint32_t>(256 * q) & 0xffu);
    }
  }
}

// Multi-device frames (rt_multi.cpp): the root's gathered buffer holds n shards of max_rows rows each (shard g =
// rows g, g + n, ... of the frame, RCCL gather order); frame row k is shard k % n, row k / n.  One block row per
// frame row; 4-byte words when rows are word-sized, bytes otherwise.
__global__ __launch_bounds__(256) void unpermute_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                        uint32_t rows, uint32_t n, uint32_t max_rows, uint32_t row_bytes) {
  for (uint32_t k = blockIdx.y; k < rows; k += gridDim.y) {
    const uint8_t *s = src + (static_cast<size_t>(k % n) * max_rows + k / n) * row_bytes;
    uint8_t *d = dst + static_cast<size_t>(k) * row_bytes;
    if ((row_bytes & 3u) == 0) {
      const uint32_t *s4 = reinterpret_cast<const uint32_t *>(s);
      uint32_t *d4 = reinterpret_cast<uint32_t *>(d);
      for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < row_bytes / 4; i += gridDim.x * 256) d4[i] = s4[i];
    } else {
      for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < row_bytes; i += gridDim.x * 256) d[i] = s[i];
    }
  }
}

// Primary-ray candidate lists of the verified sphere walk (device/prim_lists.h): one wave per 8x8 tile walks the SAH
// tree breadth-first (a level's surviving nodes in LDS, one per lane), collects the spheres that meet the tile's ray
// cone in LDS and writes them sorted (each entry's rank = the entries before it): the depth of the tree in
// dependent node loads per tile, not a serial walk of every node the cone meets.
constexpr uint32_t kPrimFrontier = 512;   // nodes of one BFS level per tile (more: no list, the rays walk)
constexpr uint32_t kPrimMaxCap = 256;     // list capacity the kernel's LDS holds
__global__ __launch_bounds__(64) void prim_list_kernel(PrimListGeom g, const uint32_t *nodes, uint32_t root,
                                                       const uint32_t *prims, uint32_t n_tiles, uint32_t cap,
                                                       uint32_t words, uint32_t *lists, uint32_t *counts) {
  __shared__ uint32_t front[2][kPrimFrontier];
  __shared__ uint2 cand[kPrimMaxCap];
  __shared__ uint32_t n_next, n_cand, bad;
  const uint32_t tile = blockIdx.x, lane = threadIdx.x;
  if (tile >= n_tiles) return;
  PrimCone k;
  if (!prim_cone(g, tile, &k)) {
    if (lane == 0) counts[tile] = kPrimListNone;
    return;
  }
  if (lane == 0) { front[0][0] = root; n_cand = 0; bad = 0; }
  uint32_t n_cur = 1, cur = 0;
  __syncthreads();
  while (n_cur > 0) {
    if (lane == 0) n_next = 0;
    __syncthreads();
    for (uint32_t i = lane; i < n_cur; i += 64) {
      const uint32_t *nd = nodes + static_cast<size_t>(front[cur][i]) * kAccelNodeWords;
      for (int ch = 0; ch < 2; ++ch) {
        if (!prim_cone_child(k, g, nd, ch)) continue;
        const uint32_t ref = nd[12 + ch];
        if (!(ref & kAccelLeaf)) {
          const uint32_t at = atomicAdd(&n_next, 1u);
          if (at < kPrimFrontier) front[cur ^ 1][at] = ref;
          else bad = 1;
          continue;
        }
        const uint32_t first = ref & 0xffffffu, cnt = ((ref >> 24) & 0x7fu) + 1u;
        for (uint32_t j = 0; j < cnt; ++j) {
          uint32_t key;
          if (!prim_cone_sphere(k, g, prims, first + j, &key)) continue;
          const uint32_t at = atomicAdd(&n_cand, 1u);
          if (at < cap) cand[at] = make_uint2(first + j, key);
          else bad = 1;
        }
      }
    }
    __syncthreads();
    n_cur = n_next < kPrimFrontier ? n_next : kPrimFrontier;
    cur ^= 1;
    if (bad) break;
  }
  __syncthreads();
  if (bad) {
    if (lane == 0) counts[tile] = kPrimListNone;
    return;
  }
  const uint32_t n = n_cand;
  uint32_t *out = lists + static_cast<size_t>(tile) * cap * words;
  for (uint32_t i = lane; i < n; i += 64) {
    const uint2 e = cand[i];
    uint32_t rank = 0;
    for (uint32_t j = 0; j < n; ++j) rank += prim_before(cand[j], e) ? 1u : 0u;
    // the entry: the sphere's SAH prim index and its axial bound (rt_layout.h kPrimEntry*)
    uint32_t *o = out + static_cast<size_t>(rank) * words;
    o[kPrimEntryIdx] = e.x;
    o[kPrimEntryBound] = e.y;
  }
  if (lane == 0) counts[tile] = n;
}

}  // namespace

hipError_t launch_prim_lists(const PrimListGeom &g, const uint32_t *nodes, uint32_t root, const uint32_t *prims,
                             uint32_t n_tiles, uint32_t cap, uint32_t words, uint32_t *lists, uint32_t *counts,
                             hipStream_t s) {
  if (n_tiles == 0) return hipSuccess;
  if (cap == 0 || cap > kPrimMaxCap || words != static_cast<uint32_t>(kPrimEntryWords)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(prim_list_kernel, dim3(n_tiles), dim3(64), 0, s, g, nodes, root, prims, n_tiles, cap, words, lists,
                     counts);
  return hipGetLastError();
}

hipError_t launch_unpermute(const void *src, void *dst, uint32_t rows, uint32_t n, uint32_t max_rows,
                            uint32_t row_bytes, hipStream_t s) {
  if (rows == 0 || row_bytes == 0) return hipSuccess;
  if (n == 0 || static_cast<uint64_t>(n) * max_rows < rows) return hipErrorInvalidValue;
  const uint32_t per = (row_bytes & 3u) == 0 ? row_bytes / 4 : row_bytes;
  const uint32_t bx = (per + 255) / 256 < 16 ? (per + 255) / 256 : 16;
  hipLaunchKernelGGL(unpermute_kernel, dim3(bx, rows < 65535u ? rows : 65535u), dim3(256), 0, s,
                     static_cast<const uint8_t *>(src), static_cast<uint8_t *>(dst), rows, n, max_rows, row_bytes);
  return hipGetLastError();
}

hipError_t launch_untile(const float *tiled, float *out, uint8_t *out8, uint32_t rows, uint32_t width, uint32_t tiles_x,
                         uint32_t ts, hipStream_t s) {
  if (rows == 0 || width == 0 || ts > 6u) return rows == 0 || width == 0 ? hipSuccess : hipErrorInvalidValue;
  const uint32_t th = 1u << (6u - ts);
  hipLaunchKernelGGL(untile_kernel, dim3((width + kUntileCols - 1) / kUntileCols, (rows + th - 1) / th), dim3(256), 0, s,
                     tiled, out, out8, rows, width, tiles_x, ts);
  return hipGetLastError();
}

hipError_t launch_tonemap(const float *rgb, uint64_t n, uint8_t *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 1023) / 1024;
  hipLaunchKernelGGL(tonemap_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, rgb, n, out);
  return hipGetLastError();
}

hipError_t launch_order(const uint32_t *cost, uint32_t n, uint32_t *order, uint32_t tiles_x, hipStream_t s) {
  hipLaunchKernelGGL(order_kernel, dim3(1), dim3(kOrderThreads), 0, s, cost, n, order, tiles_x);
  return hipGetLastError();
}

hipError_t launch_seed(const SeedArgs &a, hipStream_t s) {
  const uint64_t runs = (static_cast<uint64_t>(a.width) + kSeedRun - 1) / kSeedRun;
  const uint64_t threads = (static_cast<uint64_t>(a.rows) + 7) / 8 * 8 * runs;
  const uint32_t blocks = static_cast<uint32_t>((threads + kBlock - 1) / kBlock);
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(seed_kernel, dim3(blocks), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <int... Fs>
struct KernelTable {
  static constexpr int n = sizeof...(Fs);
  const void *ptr[n] = {reinterpret_cast<const void *>(&render_kernel<Fs>)...};
};
static const KernelTable<0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
                         16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31> kKernels;

hipError_t launch_render(const RenderArgs &a, int variant, uint32_t blocks, size_t lds_bytes, hipStream_t s) {
  if (variant < 0 || variant >= kKernels.n) return hipErrorInvalidValue;
  void *args[] = {const_cast<RenderArgs *>(&a)};
  return hipLaunchKernel(kKernels.ptr[variant], dim3(blocks), dim3(kBlock), args, lds_bytes, s);
}

int render_blocks_per_cu(int variant, size_t lds_bytes) {
  int n = 0;
  if (variant < 0 || variant >= kKernels.n ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kKernels.ptr[variant], kBlock, lds_bytes) != hipSuccess || n <= 0)
    n = 1;
  hipFuncAttributes fa;
  if (variant >= 0 && variant < kKernels.n && hipFuncGetAttributes(&fa, kKernels.ptr[variant]) == hipSuccess)
    n = min(n, resident_blocks_by_vgprs(fa.numRegs));
  return n < 1 ? 1 : n;
}

// registers and scratch of an offline render kernel (rt_stats.kernel; spill counts are not in the attributes)
bool render_kernel_attrs(int variant, int *vgprs, int *scratch) {
  hipFuncAttributes fa;
  if (variant < 0 || variant >= kKernels.n || hipFuncGetAttributes(&fa, kKernels.ptr[variant]) != hipSuccess) return false;
  *vgprs = fa.numRegs;
  *scratch = static_cast<int>(fa.localSizeBytes);
  return true;
}

}  // namespace rt
