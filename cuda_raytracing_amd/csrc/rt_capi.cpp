// rt_capi.cpp — the C-ABI of include/rt_render.h over the HIP kernels.
//
// rt_render() is the drop-in for render()'s device half (raytracing.cu:1694-1771): compile + upload
// the scene, seed per-pixel RNG (init_gpu_data, :1591-1606), run the render kernel (cuda_calc,
// :1543-1589) and copy the framebuffer back.  rt_context_* keeps the scene resident in HBM for
// repeated frames and multi-GPU shards.  Every failure is a status code; nothing exits.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <vector>

#include "gpu_scene.h"
#include "rt_jit.h"
#include "rt_kernels.h"
#include "rt_render.h"
#include "xorwow_jump.h"

namespace {

using rt::SceneImage;

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  void release() { if (p) (void)hipFree(p); p = nullptr; bytes = 0; }
};

// Pinned host staging for the per-geometry seeding tables, uploaded with hipMemcpyAsync on the frame's stream (the
// copy is ordered after the previous frame's render on that stream, which may still read the old table); `done`
// marks the copy's completion so the staging bytes are not rewritten while a copy from them is pending
struct PinBuf {
  void *p = nullptr;
  size_t bytes = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
  hipError_t stage(const void *src, size_t n) {
    if (pending) {
      if (hipEventSynchronize(done) != hipSuccess) return hipErrorUnknown;
      pending = false;
    }
    if (n > bytes) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      bytes = 0;
      const hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
      if (e != hipSuccess) return e;
      bytes = n;
    }
    if (!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) return hipErrorUnknown;
    std::memcpy(p, src, n);
    return hipSuccess;
  }
  void release() {
    if (pending && done) (void)hipEventSynchronize(done);
    if (p) (void)hipHostFree(p);
    if (done) (void)hipEventDestroy(done);
    p = nullptr; bytes = 0; done = nullptr; pending = false;
  }
};

struct DeviceGuard {   // restore the caller's current device
  int prev = -1;
  explicit DeviceGuard(int dev) { if (hipGetDevice(&prev) != hipSuccess) prev = -1; (void)hipSetDevice(dev); }
  ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

int params_check(const rt_params *p) {
  if (!p) return RT_ERR_INVALID_ARG;
  if (p->width <= 0 || p->height <= 0 || p->samples_per_pixel <= 0) return RT_ERR_INVALID_ARG;
  if (p->row_stride <= 0 || p->row_count < 0 || p->row_offset < 0) return RT_ERR_INVALID_ARG;
  if (p->row_count > 0 &&
      static_cast<int64_t>(p->row_offset) + static_cast<int64_t>(p->row_count - 1) * p->row_stride >= p->height)
    return RT_ERR_INVALID_ARG;
  if (static_cast<uint64_t>(p->row_count) * static_cast<uint64_t>(p->width) > 0x7fffffffull) return RT_ERR_INVALID_ARG;
  if (static_cast<uint64_t>(p->height) * static_cast<uint64_t>(p->width) >= (1ull << 40)) return RT_ERR_INVALID_ARG;
  // the render kernel holds a lane's pixel as local row << 16 | column
  if (p->width > 65535 || p->row_count > 65535) return RT_ERR_UNSUPPORTED;
  return RT_OK;
}

}  // namespace

static_assert(rt::MAT_LAMBERTIAN == RTR_MAT_LAMBERTIAN && rt::MAT_METAL == RTR_MAT_METAL &&
              rt::MAT_DIELECTRIC == RTR_MAT_DIELECTRIC && rt::MAT_DIFFUSE_LIGHT == RTR_MAT_DIFFUSE_LIGHT, "mat kinds");
static_assert(rt::CNT_BOUNCES == RT_CNT_BOUNCES && rt::CNT_SHADES == RT_CNT_SHADES && rt::CNT_PERLIN == RT_CNT_PERLIN &&
              rt::CNT_SAMPLES == RT_CNT_SAMPLES && rt::CNT_MAX_STACK == RT_CNT_MAX_STACK &&
              rt::CNT_OVERFLOW == RT_CNT_STACK_OVERFLOW && rt::CNT_SLOTS == RT_CNT__COUNT, "counter slots");
static_assert(rt::K_SPHERE == RTR_OBJ_SPHERE && rt::K_BVH == RTR_OBJ_BVH && rt::K_GROUP == RTR_OBJ_GROUP, "kinds");

static_assert(rt::kRngColLo == static_cast<uint32_t>(rt::kColLo) && rt::kRngColLoBits == static_cast<uint32_t>(rt::kColLoBits),
              "two-level column tables: device and host split");
static_assert(rt::kRngNibTableWords == static_cast<uint32_t>(rt::kJumpNibbleWords), "nibble table size");

constexpr int kLptMinSpp = 16;
constexpr uint32_t kAccelMinSpheres = 64;   // smaller all-sphere worlds: the scene-specialised walk
constexpr uint32_t kPrimMinSpheres = 2048;  // primary-ray candidate lists by default from this many spheres
constexpr float kFoldRayBound = 1.0e6f;
constexpr size_t kLdsPerCu = 160 * 1024;       // gfx950
constexpr size_t kLdsReserve = 1024;           // per resident block, see the colour-stack sizing
constexpr size_t kRngSlotBytes = static_cast<size_t>(rt::kWavesPerBlock) * rt::kRngSlotWords * 4;   // per block, LDS
constexpr size_t kStageBlockBytes = static_cast<size_t>(rt::kWavesPerBlock) * rt::kStageSlotWords * 4;   // per slot, block
constexpr size_t kStageWaveExtraBytes = static_cast<size_t>(rt::kWavesPerBlock) * 2 * 4;   // each wave's flag + pad words
constexpr size_t kRcLdsOnlyBlocks = 6;      // LDS-only colour stacks (kVarRcLds) must fit this many blocks per CU
constexpr uint32_t kDefaultTileShift = 3;    // 8x8 tiles
constexpr uint32_t kDefaultStageSlots = 0;   // pixels stored when they end
constexpr int kDefaultRcPool = 8;            // deep-level pool chunks per wave of deep kernels with HBM levels (RT_RC_POOL)
constexpr int kPrioTiles = 256;                 // costliest tiles at raised issue priority (RT_PRIO_TILES)
constexpr int kSparseLanes = 2;                 // noise scenes: busy lanes per wave holding the costliest pixels
constexpr int kSparseTiles = 16;                // ... over this many costliest tiles (RT_PRIO_LANES / _TILES)
constexpr int kMixLanes = 32;                   // mixed hot waves (verified mixed walk): costly pixels per wave
constexpr uint32_t kRcLdsMaxLevels = 256;  // colour-stack levels kept in LDS at most (max_bounces is a u8)
constexpr uint32_t kSpanWord = 48;          // work words 48..51: the render kernel's span (RenderArgs::span)

// LDS bytes of one colour-stack level for a 256-thread block: 32-bit codes, 16-bit in narrow kernels, 8-bit in
// byte kernels (code_bytes 4 / 2 / 1)
constexpr size_t rc_level_bytes(uint32_t code_bytes) { return static_cast<size_t>(rt::kWavesPerBlock) * 64 * code_bytes; }

// Upper bound on |component| of every ray origin/direction this render can trace (folded traversal
// precondition, scene_codegen.cpp).  Primary rays: camera centre + lens offset, directions to the
// viewport.  Secondary rays start on a primitive, inside the root BVH box, and leave in a direction
// of length <= 2 + fuzz (Lambertian n + unit, metal unit + fuzz*unit, dielectric reflect/refract of
// unit vectors).  Returns +inf when no bound is available (root is not a BVH node).
// Every attenuation a material can return is finite: solid texture colours, metal albedos and image
// texels are finite (Perlin noise and dielectrics are finite by construction).  Enables the black-path
// unwind skip (RenderArgs::black_skip).
bool attenuations_finite(const rt::SceneImage &img) {
  auto fin = [&](uint32_t word) {
    float x;
    std::memcpy(&x, &img.words[word], 4);
    return std::isfinite(x);
  };
  for (uint32_t m = 0; m < img.mat_count; ++m) {
    const uint32_t b = img.off_mats + m * rt::kMatWords;
    if (img.words[b + rt::M_KIND] == rt::MAT_METAL)
      for (int k = 0; k < 3; ++k) if (!fin(b + rt::M_ALBEDO + k)) return false;
  }
  for (uint32_t t = 0; t < img.tex_count; ++t) {
    const uint32_t b = img.off_texs + t * rt::kTexWords;
    if (img.words[b + rt::T_KIND] == rt::T_SOLID)
      for (int k = 0; k < 3; ++k) if (!fin(b + rt::T_RGB + k)) return false;
  }
  for (size_t w = img.off_pixels; w < img.words.size(); ++w) if (!fin(static_cast<uint32_t>(w))) return false;
  return true;
}

float ray_bound(const rt::SceneImage &img, const rt_camera *cam, const rt_params *p) {
  auto ab = [](float x) { return std::fabs(x); };
  const rtr_vec3 *c0 = &cam->center, *fu = &cam->defocus_u, *fv = &cam->defocus_v;
  const float ox = ab(c0->x) + ab(fu->x) + ab(fv->x), oy = ab(c0->y) + ab(fu->y) + ab(fv->y),
              oz = ab(c0->z) + ab(fu->z) + ab(fv->z);
  const float W = static_cast<float>(p->width), H = static_cast<float>(p->height);
  const float dx = ab(cam->pixel00.x) + (W + 1) * ab(cam->delta_u.x) + (H + 1) * ab(cam->delta_v.x) + ox;
  const float dy = ab(cam->pixel00.y) + (W + 1) * ab(cam->delta_u.y) + (H + 1) * ab(cam->delta_v.y) + oy;
  const float dz = ab(cam->pixel00.z) + (W + 1) * ab(cam->delta_u.z) + (H + 1) * ab(cam->delta_v.z) + oz;
  float b = std::max({ox, oy, oz, dx, dy, dz});
  const uint32_t *root = &img.words[static_cast<size_t>(img.root) * rt::kNodeWords];
  if (root[rt::W_KIND] != rt::K_BVH) return INFINITY;
  for (int k = 0; k < 6; ++k) {
    float v;
    std::memcpy(&v, &root[rt::W_BOX + k], 4);
    b = std::max(b, 2.0f * ab(v) + 1.0f);
  }
  float fuzz = 0.0f;
  for (uint32_t m = 0; m < img.mat_count; ++m) {
    const uint32_t *mw = &img.words[img.off_mats + static_cast<size_t>(m) * rt::kMatWords];
    if (mw[rt::M_KIND] == rt::MAT_METAL) {
      float f;
      std::memcpy(&f, &mw[rt::M_FUZZ], 4);
      fuzz = std::max(fuzz, ab(f));
    }
  }
  b = std::max(b, 3.0f + fuzz);
  return std::isfinite(b) ? b : INFINITY;
}   // the probe costs 8 paths per 64-pixel tile: <1% of the frame from here

// Frame-write settings of new contexts (and of rt_kernel_source): tile width RT_TILE_W (8, 16, 32, 64) and output
// staging slots per wave RT_STAGE_SLOTS (0..kStageSlotsMax)
uint32_t tile_shift_setting() {
  uint32_t ts = kDefaultTileShift;
  if (const char *e = std::getenv("RT_TILE_W")) {
    const int v = std::atoi(e);
    ts = v == 8 ? 3u : v == 16 ? 4u : v == 32 ? 5u : v == 64 ? 6u : ts;
  }
  return ts;
}
// (RT_STAGE_SLOTS=-1, A/B only: the staging code compiled in, no slots at launch)
int stage_slots_setting() {
  int n = static_cast<int>(kDefaultStageSlots);
  if (const char *e = std::getenv("RT_STAGE_SLOTS")) n = std::max(-1, std::min(static_cast<int>(rt::kStageSlotsMax), std::atoi(e)));
  return n;
}
// Deep-level pool chunks per wave (RT_RC_POOL, 0..kRcPoolChunksMax; RenderArgs::rc_pool_*).  Default: deep kernels
// (max_bounces > kDeepBounces) whose colour stack does not fit LDS; set explicitly: every kernel with HBM levels
int rc_pool_setting(bool *set = nullptr) {
  int n = kDefaultRcPool;
  if (set) *set = false;
  if (const char *e = std::getenv("RT_RC_POOL")) {
    n = std::max(0, std::min(static_cast<int>(rt::kRcPoolChunksMax), std::atoi(e)));
    if (set) *set = true;
  }
  return n;
}

// rt_kernel_info of a run-time kernel from its code object's figures (rt_jit.cpp KernelMeta)
void fill_kernel_info(const rt::KernelMeta &m, const std::string &compiler, rt_kernel_info *k) {
  k->vgprs = m.vgprs;
  k->agprs = m.agprs;
  k->sgprs = m.sgprs;
  k->scratch_bytes = m.scratch;
  k->vgpr_spills = m.vgpr_spills;
  k->sgpr_spills = m.sgpr_spills;
  k->run_time = 1;
  std::snprintf(k->compiler, sizeof k->compiler, "%s", compiler.c_str());
  std::snprintf(k->loader, sizeof k->loader, "%s", rt::jit_compiler_where().c_str());
}

struct rt_context {
  int device = 0;
  int cu_count = 0;
  double wall_khz = 100000.0;   // s_memrealtime ticks per ms (hipDeviceAttributeWallClockRate, kHz)
  SceneImage img;
  // verified sphere traversal (RT_TRAV_ACCEL): SAH tree words appended to the device scene image
  rt::SphereAccel accel;
  bool accel_ok = false;
  uint32_t accel_nodes = 0, accel_prims = 0;   // word offsets in the device image
  uint32_t accel_wide = 0;                      // ... of the 4-wide nodes (0: none)
  bool accel_w4 = false;                        // RT_ACCEL_WIDTH=4: the verified walk uses the 4-wide tree
  bool accel_q = false;                         // ... quantised (RT_ACCEL_QUANT, accel::quantize_wide)
  // top SAH nodes staged in LDS (RT_ACCEL_LDS_NODES): 64 (6 levels, 4 KiB per block) measured best on
  // the 10k scene, 1-3 % over none and over 128 / 256 (profiles/r03_ab_accel_lds_bfs_early*.jsonl)
  uint32_t accel_lds_nodes = 64;
  bool accel_lds_set = false;   // RT_ACCEL_LDS_NODES given (nodes of the tree in use)
  // primary-ray candidate lists of the verified sphere walk (device/prim_lists.h; RT_ACCEL_PRIM=0: off)
  // -1 auto: worlds of at least kPrimMinSpheres spheres (measured: 10k scene -2 % frame time, the 488-sphere scene 2
  // +4 %); 0 off, 1 on (RT_ACCEL_PRIM)
  int prim_mode = -1;
  uint32_t prim_cap = 128;      // entries per tile (RT_PRIM_CAP); a fuller tile's rays walk the tree
  double accel_half_motion = 0;   // max |motion| / 2 over the SAH tree's spheres
  // verified mixed-world traversal (RT_TRAV_MIXED): macro roots marked in the image, SAH words appended
  rt::MixedAccel mixed;
  bool mixed_ok = false;
  uint32_t mix_nodes = 0, mix_prims = 0;
  bool mix_no_proof = false;   // RT_MIX_PROVE=0 (test aid): every macro walk falls back
  int static_ok = -1;          // the scene expands within jit_budget (straight-line, stackless traversal); -1 unknown
  DevBuf scene, jump, rng_rows, rng_cols, rc, work, counters, wave_trace, tile_cost, tile_order, prim_lists, prim_counts;
  DevBuf tiled;                    // tile-major render output (RT_TILED_OUT)
  // seeding tables of the last geometry, kept on the device: the phase bases (xorwow_phase_bases; key = seed, W,
  // rows of the shard) and the column tables (xorwow_column_tables; key = W)
  uint64_t rows_key[5] = {~0ull, 0, 0, 0, 0};
  int cols_width = -1;
  PinBuf rows_stage, cols_stage;   // their pinned staging (stream-ordered uploads)
  bool ev_recorded = false;        // ev[2] has been recorded (a frame was enqueued before)
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};   // seed | schedule (probe + order) | render
  bool lds = false;
  bool counted = false;
  int variant = 0;
  // traversal policy: -1 auto, RT_TRAV_LANE, RT_TRAV_PACKET, RT_TRAV_STATIC (env RT_TRAVERSAL for A/B runs)
  int traversal = -1;
  int used_traversal = RT_TRAV_LANE;
  uint32_t jit_budget = 256;    // max node visits of a scene-specialised traversal (env RT_JIT_BUDGET)
  uint32_t jit_visits = 0;
  std::string jit_why;
  // diagnostics / A-B knobs (env, read at creation): RT_WAVE_TRACE=<file>, RT_TILE_ORDER, RT_BLOCKS_PER_CU
  std::string wave_trace_path;
  size_t wave_trace_words = 0;
  int sched = 0;   // RT_SCHED: 0 auto (longest-first when spp >= kLptMinSpp), 1 row-major, 2 reversed, 3 longest-first
  int blocks_per_cu = 0;
  uint32_t rc_lds_levels = rt::kRcLdsLevels;   // RT_RC_LDS_LEVELS (minimum; more when LDS is free)
  bool rc_lds_auto = true;                      // RT_RC_LDS_LEVELS given: exactly that many
  bool black_skip = false;                      // attenuations_finite(img) (RT_BLACK_SKIP=0 disables)
  uint32_t max_tries = 0;                       // RT_MAX_TRIES: rejection tries per round (0 = unlimited)
  int prio_tiles = -1;                          // RT_PRIO_TILES: costliest tiles run at raised priority (-1 auto)
  int prio_chunk = -1;                          // RT_PRIO_CHUNK: those tiles handed out in pieces of this many pixels
  int tail_prio = -1;                           // RT_TAIL_PRIO: tail issue priority by remaining samples (-1: auto)
  int prio_lanes = 0;                           // RT_PRIO_LANES: waves holding them keep at most this many lanes busy
  int prio_mix = -1;                            // RT_PRIO_MIX=1/0: ... and fill their other lanes with ordinary
                                                // tiles (-1: the default, on for the verified mixed walk)
                                                // (0: the default, kSparseLanes on noise scenes; 64: off)
                                                // (-1 auto: 1 with cooperative noise, else whole tiles)
  uint32_t coop_noise = 32;                     // RT_COOP_NOISE: cooperative noise octaves when <= this many lanes
                                                // of a wave need one (0 = never, max 32)
  uint32_t defer_lanes = 4;                     // RT_DEFER_LANES: end a round's rejection at <= this many lanes
  uint32_t defer_trace = 16, trace_min_iters = 16;  // RT_DEFER_TRACE, RT_TRACE_MIN (paused per-lane walks)
  bool lane_jit = true;                         // RT_JIT_LANE=0: offline all-kinds lane kernel
  bool shade_spec = true;                       // RT_JIT_SHADE=0: run-time kernels keep every material
  uint32_t probe_per_tile = 0;   // RT_PROBE (1..256); 0 = clamp(spp / 4, 8, 64) paths per 64-pixel tile
  bool used_lpt = false;
  bool fold_enabled = true;
  uint32_t fold_violations = 0;      // RT_JIT_FOLD=0 disables exact constant folding (A/B)
  bool used_fold = false;
  // the last render, for the unfolded re-render after a fold-bound violation (rt_context_timing)
  rt_camera last_cam{};
  rt_params last_params{};
  float *last_out = nullptr;
  uint8_t *last_out8 = nullptr;
  void *last_stream = nullptr;
  bool rendered = false;
  uint64_t samples = 0;
  size_t lds_bytes = 0;
  size_t rc_audit_bytes = 0;      // RT_FLAG_RC_AUDIT: bytes of the HBM colour-stack buffer filled before the render
  uint32_t rc_audit_code = 4;     // ... holding codes of this many bytes
  bool rc_no_byte = false;        // RT_RC_BYTE=0: 16-bit codes where 8-bit ones would do (A/B)
  bool rc_lds_only_off = false;   // set while a render is redone without kVarRcLds (its layout did not fit)
  // frame writes (RenderArgs::tile_shift / stage_*): tile width 1 << tile_shift (RT_TILE_W) and the staging slots per
  // wave (RT_STAGE_SLOTS, 0 = every pixel stored when it ends); the slots only take LDS the resident blocks leave
  uint32_t tile_shift = 3;         // (tile_shift_setting)
  int stage_slots = 0;             // (stage_slots_setting; -1: compiled in, none at launch)
  uint32_t used_stage_slots = 0;   // the last render's
  int tiled_out = -1;              // 1: the render writes the frame tile-major, untile_kernel the rows + bytes; 0: row-major
                                   // stores; -1 (default): tile-major (RT_TILED_OUT)
  bool used_tiled = false;         // the last render's
  int tail_chunk = 0;              // RT_TAIL_CHUNK: the tail of the order in pieces of this many pixels (0: whole tiles)
  double tail_gen = 1.0;           // RT_TAIL_GEN: ... over this many times the grid's lanes of ids
  uint32_t used_tail_ids = 0;      // the last render's
  int rc_pool = 0;                 // deep-level pool chunks per wave (rc_pool_setting)
  bool rc_pool_set = false;        // ... given explicitly: also for shallow kernels
  uint32_t used_pool_chunks = 0;   // the last render's
  // per-XCD tile queues (RenderArgs::cls_off; RT_XCD_CLASSES=1/0)
  bool xcd_classes = false;
  bool used_classes = false;
  uint32_t used_rc_levels = 0;    // colour-stack levels the last render kept in LDS
  int jit_source = RT_JIT_NONE;   // last render: where its run-time kernels came from
  double jit_ms = 0.0;            // ... and the host time spent obtaining them
  rt_kernel_info used_kernel{};   // the last render's render kernel (registers, scratch, spills, compiler)
};

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

#ifndef RT_SOURCE_HASH
#define RT_SOURCE_HASH "unstamped"
#define RT_SOURCE_FILES ""
#endif
// the sources this library was built from and the hash of their bytes (Makefile `stamp`; cuda_raytracing_amd/_abi.py
// refuses a library whose hash does not match the tree's files)
const char *rt_hip_build_hash(void) { return RT_SOURCE_HASH; }
const char *rt_hip_build_files(void) { return RT_SOURCE_FILES; }

int rt_accel_build(const rt_scene *scene, uint32_t *words, uint64_t cap, uint32_t info[4]) {
  if (!scene || !info) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  int st = rt::compile_scene(scene, &img);
  if (st != RT_OK) return st;
  rt::SphereAccel a;
  std::string why;
  if (!rt::build_sphere_accel(img, kAccelMinSpheres, &a, &why)) return RT_ERR_UNSUPPORTED;
  info[0] = a.root;
  info[1] = a.depth;
  info[2] = a.spheres;
  info[3] = static_cast<uint32_t>(a.node_words.size());
  const uint64_t n = a.node_words.size() + a.prim_words.size();
  if (words) {
    if (cap < n) return RT_ERR_INVALID_ARG;
    std::memcpy(words, a.node_words.data(), a.node_words.size() * 4);
    std::memcpy(words + a.node_words.size(), a.prim_words.data(), a.prim_words.size() * 4);
  }
  return RT_OK;
}

int rt_accel_build_wide(const rt_scene *scene, uint32_t *words, uint64_t cap, uint32_t info[4]) {
  if (!scene || !info) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  int st = rt::compile_scene(scene, &img);
  if (st != RT_OK) return st;
  rt::SphereAccel a;
  std::string why;
  if (!rt::build_sphere_accel(img, kAccelMinSpheres, &a, &why) || a.wide_words.empty()) return RT_ERR_UNSUPPORTED;
  info[0] = static_cast<uint32_t>(a.wide_words.size() / rt::kAccel4NodeWords);
  info[1] = a.wide_depth;
  info[2] = a.wide_stack;
  info[3] = static_cast<uint32_t>(a.wide_words.size());
  if (words) {
    if (cap < a.wide_words.size()) return RT_ERR_INVALID_ARG;
    std::memcpy(words, a.wide_words.data(), a.wide_words.size() * 4);
  }
  return RT_OK;
}

// max over the SAH prims of |motion| / 2 (rounded up a little)
static double half_motion_of(const std::vector<uint32_t> &prims) {
  double m = 0.0;
  for (size_t k = 0; k + rt::kAccelPrimWords <= prims.size(); k += rt::kAccelPrimWords) {
    float v[3];
    std::memcpy(v, &prims[k + rt::AP_MOTION], sizeof v);
    m = std::max(m, std::sqrt(static_cast<double>(v[0]) * v[0] + static_cast<double>(v[1]) * v[1] + static_cast<double>(v[2]) * v[2]));
  }
  return 0.5 * m * (1.0 + 1.0e-9);
}

static rt::PrimListGeom make_prim_geom(const rt_camera *cam, const rt_params *p, uint32_t tiles_x, uint32_t tile_shift,
                                       double half_motion, float *rho_f);

int rt_accel_build_quant(const rt_scene *scene, uint32_t *words, uint64_t cap, uint32_t info[4]) {
  if (!scene || !info) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  int st = rt::compile_scene(scene, &img);
  if (st != RT_OK) return st;
  rt::SphereAccel a;
  std::string why;
  if (!rt::build_sphere_accel(img, kAccelMinSpheres, &a, &why) || a.wide_q_words.empty()) return RT_ERR_UNSUPPORTED;
  info[0] = static_cast<uint32_t>(a.wide_q_words.size() / rt::kAccel4QNodeWords);
  info[1] = a.wide_depth;
  info[2] = a.wide_stack;
  info[3] = static_cast<uint32_t>(a.wide_q_words.size());
  if (words) {
    if (cap < a.wide_q_words.size()) return RT_ERR_INVALID_ARG;
    std::memcpy(words, a.wide_q_words.data(), a.wide_q_words.size() * 4);
  }
  return RT_OK;
}

int rt_prim_lists(const rt_scene *scene, const rt_camera *cam, const rt_params *p, uint32_t cap, uint32_t *counts,
                  uint32_t *lists, float *rho) {
  if (!scene || !cam || !p || !counts || cap == 0 || p->width <= 0 || p->row_count <= 0 || p->row_stride <= 0)
    return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  int st = rt::compile_scene(scene, &img);
  if (st != RT_OK) return st;
  rt::SphereAccel a;
  std::string why;
  if (!rt::build_sphere_accel(img, kAccelMinSpheres, &a, &why)) return RT_ERR_UNSUPPORTED;
  const double motion = half_motion_of(a.prim_words);
  const uint32_t tiles_x = (static_cast<uint32_t>(p->width) + 7) / 8;
  const uint32_t n_tiles = tiles_x * ((static_cast<uint32_t>(p->row_count) + 7) / 8);
  float rf = 0.0f;
  const rt::PrimListGeom g = make_prim_geom(cam, p, tiles_x, 3u, motion, &rf);   // 8x8 tiles (this host API's contract)
  if (rho) *rho = rf;
  std::vector<uint2> buf(cap);
  for (uint32_t t = 0; t < n_tiles; ++t) {
    counts[t] = rt::prim_list_build_host(g, a.node_words.data(), a.root, a.prim_words.data(), t, cap, buf.data());
    if (lists && counts[t] != rt::kPrimListNone)
      for (uint32_t k = 0; k < counts[t]; ++k) { lists[(static_cast<size_t>(t) * cap + k) * 2] = buf[k].x; lists[(static_cast<size_t>(t) * cap + k) * 2 + 1] = buf[k].y; }
  }
  return RT_OK;
}

int rt_mixed_build(const rt_scene *scene, uint32_t info[4]) {
  if (!scene || !info) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  int st = rt::compile_scene(scene, &img);
  if (st != RT_OK) return st;
  rt::MixedAccel m;
  std::string why;
  if (!rt::build_mixed_accel(&img, &m, &why)) return RT_ERR_UNSUPPORTED;
  info[0] = m.macros;
  info[1] = m.dynamic;
  info[2] = m.prims;
  info[3] = m.depth;
  return RT_OK;
}

const char *rt_status_string(int s) {
  switch (s) {
    case RT_OK: return "ok";
    case RT_ERR_INVALID_ARG: return "invalid argument";
    case RT_ERR_SCENE: return "malformed scene";
    case RT_ERR_HIP: return "HIP runtime error";
    case RT_ERR_NO_DEVICE: return "no HIP device";
    case RT_ERR_STACK: return "traversal stack too deep";
    case RT_ERR_UNSUPPORTED: return "unsupported";
    case RT_ERR_DEVICE_CHECK: return "device check failed";
  }
  return "unknown status";
}

int rt_device_count(int *count) {
  if (!count) return RT_ERR_INVALID_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return RT_OK;
}

void rt_context_destroy(rt_context *c) {
  if (!c) return;
  {
    DeviceGuard g(c->device);
    for (hipEvent_t &e : c->ev) if (e) (void)hipEventDestroy(e);
    c->scene.release(); c->jump.release(); c->rng_rows.release(); c->rng_cols.release(); c->prim_lists.release(); c->prim_counts.release(); c->rc.release();
    c->work.release(); c->counters.release();
    c->wave_trace.release(); c->tile_cost.release(); c->tile_order.release(); c->tiled.release();
    c->rows_stage.release(); c->cols_stage.release();
  }
  delete c;
}

int rt_context_create(const rt_scene *scene, int device, rt_context **out) {
  if (!scene || !out) return RT_ERR_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return RT_ERR_INVALID_ARG;
  rt_context *c = new (std::nothrow) rt_context();
  if (!c) return RT_ERR_INVALID_ARG;
  c->device = device;
  if (const char *e = std::getenv("RT_TRAVERSAL")) c->traversal = std::atoi(e);
  if (const char *e = std::getenv("RT_JIT_BUDGET")) c->jit_budget = static_cast<uint32_t>(std::atoi(e));
  if (const char *e = std::getenv("RT_WAVE_TRACE")) c->wave_trace_path = e;
  if (const char *e = std::getenv("RT_SCHED")) c->sched = std::atoi(e);
  if (const char *e = std::getenv("RT_JIT_FOLD")) c->fold_enabled = e[0] != '0';
  if (const char *e = std::getenv("RT_PROBE"))
    c->probe_per_tile = static_cast<uint32_t>(std::min(256, std::max(1, std::atoi(e))));
  if (const char *e = std::getenv("RT_RC_LDS_LEVELS")) {
    c->rc_lds_levels = static_cast<uint32_t>(std::atoi(e));
    c->rc_lds_auto = false;
  }
  if (const char *e = std::getenv("RT_BLOCKS_PER_CU")) c->blocks_per_cu = std::atoi(e);
  if (const char *e = std::getenv("RT_ACCEL_PRIM")) c->prim_mode = e[0] != '0' ? 1 : 0;
  if (const char *e = std::getenv("RT_PRIM_CAP")) c->prim_cap = static_cast<uint32_t>(std::max(1, std::min(256, std::atoi(e))));
  if (const char *e = std::getenv("RT_JIT_LANE")) c->lane_jit = e[0] != '0';
  if (const char *e = std::getenv("RT_JIT_SHADE")) c->shade_spec = e[0] != '0';
  if (const char *e = std::getenv("RT_MAX_TRIES")) c->max_tries = static_cast<uint32_t>(std::max(0, std::atoi(e)));
  if (const char *e = std::getenv("RT_PRIO_TILES")) c->prio_tiles = std::atoi(e);
  if (const char *e = std::getenv("RT_PRIO_LANES")) c->prio_lanes = std::atoi(e);
  if (const char *e = std::getenv("RT_TAIL_PRIO")) c->tail_prio = e[0] == '1' ? 1 : 0;
  if (const char *e = std::getenv("RT_PRIO_MIX")) c->prio_mix = e[0] == '1' ? 1 : 0;
  if (const char *e = std::getenv("RT_COOP_NOISE")) c->coop_noise = static_cast<uint32_t>(std::min(32, std::max(0, std::atoi(e))));
  if (const char *e = std::getenv("RT_PRIO_CHUNK")) {
    const int v = std::atoi(e);
    c->prio_chunk = (v == 1 || v == 2 || v == 4 || v == 8 || v == 16 || v == 32) ? v : 64;
  }
  if (const char *e = std::getenv("RT_DEFER_TRACE")) c->defer_trace = static_cast<uint32_t>(std::max(0, std::atoi(e)));
  if (const char *e = std::getenv("RT_TRACE_MIN")) c->trace_min_iters = static_cast<uint32_t>(std::max(1, std::atoi(e)));
  if (const char *e = std::getenv("RT_DEFER_LANES")) c->defer_lanes = static_cast<uint32_t>(std::max(0, std::atoi(e)));
  if (const char *e = std::getenv("RT_MIX_PROVE")) c->mix_no_proof = e[0] == '0';
  if (const char *e = std::getenv("RT_RC_BYTE")) c->rc_no_byte = e[0] == '0';
  c->tile_shift = tile_shift_setting();
  if (const char *e = std::getenv("RT_XCD_CLASSES")) c->xcd_classes = e[0] == '1';
  c->stage_slots = stage_slots_setting();
  c->rc_pool = rc_pool_setting(&c->rc_pool_set);
  if (const char *e = std::getenv("RT_TAIL_CHUNK")) {
    const int v = std::atoi(e);
    c->tail_chunk = (v == 1 || v == 2 || v == 4 || v == 8 || v == 16 || v == 32) ? v : 0;
  }
  if (const char *e = std::getenv("RT_TAIL_GEN")) c->tail_gen = std::max(0.0, std::atof(e));
  if (const char *e = std::getenv("RT_TILED_OUT")) c->tiled_out = e[0] == '1' ? 1 : (e[0] == '0' ? 0 : -1);
  if (const char *e = std::getenv("RT_ACCEL_LDS_NODES")) {
    c->accel_lds_nodes = static_cast<uint32_t>(std::max(0, std::atoi(e)));
    c->accel_lds_set = true;
  }
  int st = rt::compile_scene(scene, &c->img);
  if (st != RT_OK) { delete c; return st; }
  while (c->img.words.size() % 4) c->img.words.push_back(0);
  {
    const char *e = std::getenv("RT_ACCEL");
    std::string why;
    if (!(e && e[0] == '0') && rt::build_sphere_accel(c->img, kAccelMinSpheres, &c->accel, &why)) c->accel_ok = true;
    // worlds the sphere walk cannot take: macro roots for the mixed walk (marks W_MACRO / W_XFBOX in the
    // node words, which every other traversal ignores)
    const char *m = std::getenv("RT_MIXED");
    if (!c->accel_ok && !(m && m[0] == '0') && rt::build_mixed_accel(&c->img, &c->mixed, &why)) c->mixed_ok = true;
    if (c->mixed_ok && std::getenv("RT_DEBUG"))
      std::fprintf(stderr, "[rt] mixed accel: %u macros (%u dynamic), %u packed sphere chains\n", c->mixed.macros,
                   c->mixed.dynamic, c->mixed.packed);
  }
  std::vector<uint32_t> dev_words = c->img.words;
  if (c->accel_ok) {
    c->accel_nodes = static_cast<uint32_t>(dev_words.size());
    dev_words.insert(dev_words.end(), c->accel.node_words.begin(), c->accel.node_words.end());
    c->accel_prims = static_cast<uint32_t>(dev_words.size());
    dev_words.insert(dev_words.end(), c->accel.prim_words.begin(), c->accel.prim_words.end());
    c->accel_half_motion = half_motion_of(c->accel.prim_words);
    c->accel_w4 = rt::accel_width() == 4 && !c->accel.wide_words.empty();
    c->accel_q = c->accel_w4 && rt::accel_quant() && !c->accel.wide_q_words.empty();
    if (c->accel_w4) {
      const std::vector<uint32_t> &ww = c->accel_q ? c->accel.wide_q_words : c->accel.wide_words;
      while (dev_words.size() % 16) dev_words.push_back(0);   // 64-B node lines
      c->accel_wide = static_cast<uint32_t>(dev_words.size());
      dev_words.insert(dev_words.end(), ww.begin(), ww.end());
    }
  }
  if (c->mixed_ok) {
    c->mix_nodes = static_cast<uint32_t>(dev_words.size());
    dev_words.insert(dev_words.end(), c->mixed.node_words.begin(), c->mixed.node_words.end());
    c->mix_prims = static_cast<uint32_t>(dev_words.size());
    dev_words.insert(dev_words.end(), c->mixed.prim_words.begin(), c->mixed.prim_words.end());
  }
  // colour-stack codes carry a record index in 23 bits, a texel word offset in 31 (rt_layout.h)
  if (c->img.rec_consts + rt::kRcConsts > rt::kRcPayload ||
      (c->img.needs_uv && c->img.words.size() - c->img.off_pixels > rt::kRcTexelPayload)) {
    delete c;
    return RT_ERR_UNSUPPORTED;
  }
  c->black_skip = attenuations_finite(c->img);
  if (const char *e = std::getenv("RT_BLACK_SKIP")) c->black_skip = c->black_skip && e[0] != '0';
  DeviceGuard g(device);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { rt_context_destroy(c); return RT_ERR_HIP; }
  c->cu_count = prop.multiProcessorCount;
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0) c->wall_khz = khz;
  }
  const std::vector<uint32_t> &J = rt::xorwow_jump_tables();
  bool ok = c->scene.ensure(dev_words.size() * 4) == hipSuccess &&
            hipMemcpy(c->scene.p, dev_words.data(), dev_words.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
            c->jump.ensure(J.size() * 4) == hipSuccess &&
            hipMemcpy(c->jump.p, J.data(), J.size() * 4, hipMemcpyHostToDevice) == hipSuccess &&
            c->work.ensure(256) == hipSuccess &&   // 16 words + the mixed-walk diagnostic (RT_MIX_DIAG)
           
            c->counters.ensure(RT_CNT__COUNT * sizeof(unsigned long long)) == hipSuccess;
  for (hipEvent_t &e : c->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
  if (!ok) { rt_context_destroy(c); return RT_ERR_HIP; }
  *out = c;
  return RT_OK;
}

int rt_context_render(rt_context *c, const rt_camera *cam, const rt_params *p, float *out_dev, void *stream) {
  return rt_context_render_ppm(c, cam, p, out_dev, nullptr, stream);
}

// The ray cone geometry of a frame's camera for the primary-ray candidate lists (device/prim_lists.h): the defocus
// disc's radius bound and the footprint widening cover the float arithmetic of the kernel's camera ray (a few
// roundings of these magnitudes, far inside 2^-18 of them); *rho_f = the radius bound as a float, rounded up.
static rt::PrimListGeom make_prim_geom(const rt_camera *cam, const rt_params *p, uint32_t tiles_x, uint32_t tile_shift,
                                       double half_motion, float *rho_f) {
  rt::PrimListGeom g{};
  const rtr_vec3 *cv[4] = {&cam->pixel00, &cam->delta_u, &cam->delta_v, &cam->center};
  double *gd[4] = {g.p00, g.du, g.dv, g.c};
  for (int k = 0; k < 4; ++k) { gd[k][0] = cv[k]->x; gd[k][1] = cv[k]->y; gd[k][2] = cv[k]->z; }
  auto n1 = [](const rtr_vec3 &v) { return std::fabs(static_cast<double>(v.x)) + std::fabs(static_cast<double>(v.y)) + std::fabs(static_cast<double>(v.z)); };
  auto sq = [](const rtr_vec3 &v) { return static_cast<double>(v.x) * v.x + static_cast<double>(v.y) * v.y + static_cast<double>(v.z) * v.z; };
  const double l1 = n1(cam->center);
  // origin = centre + x u + y v with x^2 + y^2 < 1 (:1459-1476): |origin - centre| <= sqrt(|u|^2 + |v|^2)
  const double rho = cam->defocus_angle > 0 ? std::sqrt(sq(cam->defocus_u) + sq(cam->defocus_v)) : 0.0;
  g.rho = rho * (1.0 + 0x1p-18) + 0x1p-18 * l1;
  const double rows_span = static_cast<double>(p->row_offset) + static_cast<double>(p->row_count) * p->row_stride + 1.0;
  g.eps = 0x1p-18 * (n1(cam->pixel00) + rows_span * n1(cam->delta_v) + (p->width + 1.0) * n1(cam->delta_u) + l1 + g.rho);
  g.width = p->width; g.rows = p->row_count; g.row_offset = p->row_offset; g.row_stride = p->row_stride;
  g.tiles_x = tiles_x;
  g.tile_shift = tile_shift;
  g.half_motion = half_motion;
  float fr = static_cast<float>(g.rho);
  if (static_cast<double>(fr) < g.rho) fr = std::nextafter(fr, std::numeric_limits<float>::infinity());
  *rho_f = fr;
  return g;
}

int rt_context_render_ppm(rt_context *c, const rt_camera *cam, const rt_params *p, float *out_dev, uint8_t *out8_dev,
                          void *stream) {
  if (!c) return RT_ERR_INVALID_ARG;
  c->rendered = false;   // set again once this frame's whole sequence is enqueued
  if (!cam) return RT_ERR_INVALID_ARG;
  int st = params_check(p);
  if (st != RT_OK) return st;
  if (!out_dev && p->row_count > 0) return RT_ERR_INVALID_ARG;
  DeviceGuard g(c->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  // Every frame reuses the context's buffers (work counters, tile order, colour stack, candidate lists, tile-major frame,
  // RNG tables): a frame enqueued on another stream than the previous frame first waits for that frame's end, so
  // alternating streams on one context is safe; frames on one stream are ordered by the stream itself
  if (c->ev_recorded && stream != c->last_stream && hipStreamWaitEvent(s, c->ev[2], 0) != hipSuccess) return RT_ERR_HIP;
  c->last_stream = stream;
  const uint32_t n = static_cast<uint32_t>(p->row_count) * static_cast<uint32_t>(p->width);
  const uint32_t mb = static_cast<uint8_t>(p->max_bounces);   // rc_stack.max_count is u8 (:220,1596)
  // a frame counts as rendered only once its whole sequence is enqueued: any failure below leaves
  // rendered == false, so rt_context_timing never reports an earlier frame's events as this one's
  c->rendered = false;
  c->jit_why.clear();
  c->counted = (p->flags & RT_FLAG_COUNT) != 0;
  c->samples = static_cast<uint64_t>(n) * static_cast<uint64_t>(p->samples_per_pixel);
  c->used_fold = false;
  if ((n == 0 || mb == 0) && hipMemsetAsync(c->work.p, 0, 256, s) != hipSuccess) return RT_ERR_HIP;   // no span
  if (n == 0) {   // same event order as a render: seed | schedule | render, ev[2] (render end) last
    for (int k : {0, 1, 3, 2})
      if (hipEventRecord(c->ev[k], s) != hipSuccess) return RT_ERR_HIP;
    c->ev_recorded = true;
    c->rendered = true;
    return RT_OK;
  }
  if (mb == 0) {   // ray_color returns {0} without tracing (:1339): every pixel is exactly 0
    if (hipEventRecord(c->ev[0], s) != hipSuccess || hipEventRecord(c->ev[1], s) != hipSuccess ||
        hipEventRecord(c->ev[3], s) != hipSuccess)
      return RT_ERR_HIP;
    if (hipMemsetAsync(out_dev, 0, static_cast<size_t>(n) * 12, s) != hipSuccess) return RT_ERR_HIP;
    if (out8_dev && hipMemsetAsync(out8_dev, 0, static_cast<size_t>(n) * 3, s) != hipSuccess) return RT_ERR_HIP;
    if (hipEventRecord(c->ev[2], s) != hipSuccess) return RT_ERR_HIP;
    c->ev_recorded = true;
    c->rendered = true;
    return RT_OK;
  }

  // Traversal policy (flags; the choice between policies follows below).  Auto: the scene-specialised
  // straight-line traversal when the scene expands to at most jit_budget node visits (every catalog scene
  // but the large ones), else the verified SAH walks, else the per-lane DFS.  The wave-packet DFS is kept
  // as an explicit option (fastest on tiny all-sphere scenes).
  int trav = c->traversal;
  if (p->flags & RT_FLAG_FORCE_LANE) trav = RT_TRAV_LANE;
  else if (p->flags & RT_FLAG_FORCE_PACKET) trav = RT_TRAV_PACKET;
  else if (p->flags & RT_FLAG_FORCE_STATIC) trav = RT_TRAV_STATIC;
  else if (p->flags & RT_FLAG_FORCE_ACCEL) trav = RT_TRAV_ACCEL;
  else if (p->flags & RT_FLAG_FORCE_MIXED) trav = RT_TRAV_MIXED;
  if (p->flags & RT_FLAG_NO_JIT && (trav < 0 || trav == RT_TRAV_STATIC || trav == RT_TRAV_ACCEL || trav == RT_TRAV_MIXED))
    trav = RT_TRAV_LANE;
  // the straight-line traversal needs no per-lane stack: known before the LDS budget is split
  if ((trav < 0 || trav == RT_TRAV_STATIC) && c->static_ok < 0) {
    std::string src;
    uint32_t v = 0;
    bool folded = false;
    c->static_ok = rt::jit_source(c->img, 0, c->jit_budget, false, &src, &v, &folded) ? 1 : 0;
  }
  bool stackless = (trav < 0 || trav == RT_TRAV_STATIC) && c->static_ok == 1;

  // launch geometry: persistent grid = resident blocks per CU x CUs
  c->lds = c->img.words.size() <= rt::kLdsSceneMaxWords && !(p->flags & RT_FLAG_GLOBAL_SCENE);
  uint32_t scene_lds_words = c->lds ? static_cast<uint32_t>(c->img.words.size()) : 0;
  // colour stack: 16-bit codes in run-time compiled kernels of scenes without noise and texels (and with
  // < 65536 colour records), 32-bit otherwise; the LDS-scene decision is made with the wide size
  const bool narrow_ok = !c->img.has_noise && !c->img.needs_uv && c->img.rec_consts + rt::kRcConsts < 65536u;   // code 0xffff stays unused (RC_AUDIT sentinel)
  const bool byte_ok = narrow_ok && c->img.rec_consts + rt::kRcConsts < 255u && !c->rc_no_byte;            // 0xff unused likewise
  uint32_t rc_levels = std::min<uint32_t>(mb, c->rc_lds_levels);
  size_t rc_bytes = rc_levels * rc_level_bytes(4);
  // per-lane u16 stack: the reference walk's exact need, or the SAH walk's depth if deeper
  // (the mixed walk keeps a macro's SAH stack above the reference walk's entries)
  // (+ kSumEntries on all-sphere worlds: the verified walk parks each lane's pixel sum in its stack's top entries)
  const uint32_t stack_cap = std::max({c->img.stack_need, c->accel_ok ? c->accel.depth + 1 : 0u,
                                       c->accel_w4 ? c->accel.wide_stack : 0u,
                                       c->mixed_ok ? c->img.stack_need + c->mixed.depth + 1 : 0u}) +
                             (c->accel_ok ? rt::kSumEntries : 0u);
  // the verified walk's parked random_test (entries 0 and 1) and pixel sum (the top kSumEntries) must not overlap
  if (c->accel_ok && stack_cap < rt::kSumEntries + 2u) return RT_ERR_STACK;
  // test aid of the device checks (RT_CHECKS=1 only): a per-lane stack RT_CHECK_STACK_CAP entries deep, too shallow on
  // purpose, so the checks' naming of an overflow can be tested (tests/test_gpu_kernels.py)
  uint32_t stack_cap_launch = stack_cap;
  if (const char *ce = std::getenv("RT_CHECKS"); ce && ce[0] == '1')
    if (const char *e = std::getenv("RT_CHECK_STACK_CAP"); e && std::atoi(e) > 0)
      stack_cap_launch = std::min<uint32_t>(stack_cap, static_cast<uint32_t>(std::atoi(e)));
  // (+ the block's RNG slots, kRngSlotBytes: the "stack" region's fixed tail)
  const size_t full_stack_bytes = static_cast<size_t>(rt::kWavesPerBlock) * stack_cap * 64 * 2 + kRngSlotBytes;
  size_t stack_bytes = stackless ? kRngSlotBytes : full_stack_bytes;
  // one block may declare at most the CU's 160 KiB: a deep per-lane stack first evicts the LDS copy of
  // the scene (read from HBM instead); if the stack and the minimum colour-stack levels alone do not
  // fit, the scene is too deep for this kernel (a status, not a failed launch)
  if (rc_bytes + stack_bytes > kLdsPerCu - kLdsReserve) return RT_ERR_STACK;
  if (c->lds && static_cast<size_t>(scene_lds_words) * 4 + rc_bytes + stack_bytes > kLdsPerCu - kLdsReserve) {
    c->lds = false;
    scene_lds_words = 0;
  }
  c->lds_bytes = static_cast<size_t>(scene_lds_words) * 4 + rc_bytes + stack_bytes;
  c->variant = (c->lds ? rt::kVarLds : 0) | (c->counted ? rt::kVarCount : 0) |
               (c->img.has_noise ? rt::kVarNoise : 0) | (c->img.needs_uv ? rt::kVarUv : 0);
  // every colour-stack level of a run-time kernel in LDS at 6 blocks/CU (the residency of every run-time render kernel
  // measured: 77-169 VGPRs; one that would reach 7-8 loses that step to LDS, never correctness), scene staging, per-lane
  // stacks and RNG slots included: such kernels carry no HBM level code (kVarRcLds).  Set below only when the levels
  // are kept.
  const uint32_t cb_jit = byte_ok ? 1u : (narrow_ok ? 2u : 4u);
  const size_t lds_only_need = static_cast<size_t>((mb + 3) & ~3u) * rc_level_bytes(cb_jit) +
                               (c->lds ? static_cast<size_t>(scene_lds_words) * 4 : 4096u /* staged SAH top nodes */) +
                               (stackless ? kRngSlotBytes : full_stack_bytes) + kLdsReserve;
  const bool rc_lds_only = c->rc_lds_auto && !c->rc_lds_only_off && lds_only_need <= kLdsPerCu / kRcLdsOnlyBlocks;
  // tile-major output (run-time kernels; not with output staging, which stores whole tiles row-major itself), in every
  // kernel since round 6: the Perlin d50 kernel's 15-21 % slowdown with it (round 5) was the LLVM 20 build's;
  // built by LLVM 22 it runs level (profiles/r06_ab_perlin_tiled.jsonl: 98.8 / 98.7 / 97.7 vs 99.3 / 98.9 / 99.3 ms)
  const bool tiled_kernel = c->tiled_out != 0 && c->stage_slots == 0 && out_dev != nullptr;
  // the deep-level pool's code in run-time kernels with HBM levels (sized below, once the residency is known)
  // (by default deep kernels with automatic levels; pinned levels, RT_RC_LDS_LEVELS, get one only with RT_RC_POOL)
  const bool pool_kernel = c->rc_pool > 0 && !rc_lds_only &&
                           (c->rc_pool_set || (c->rc_lds_auto && mb > static_cast<uint32_t>(rt::kDeepBounces)));
  // run-time compiled kernels only: diagnostics timeline + the scene's material/texture kinds
  const int trace_bit = (c->wave_trace_path.empty() ? 0 : rt::kVarTrace) | (c->shade_spec ? rt::scene_shading_bits(c->img) : 0) |
                        (mb > static_cast<uint32_t>(rt::kDeepBounces) ? rt::kVarDeep : 0) |
                        (narrow_ok ? rt::kVarNarrow : 0) | (byte_ok ? rt::kVarByte : 0) | (rc_lds_only ? rt::kVarRcLds : 0) |
                        static_cast<int>(c->tile_shift << rt::kVarTileShift) | (c->stage_slots ? rt::kVarStage : 0) |
                        (pool_kernel ? rt::kVarRcPool : 0) | (c->tail_chunk > 0 ? rt::kVarTail : 0) |
                        (tiled_kernel ? rt::kVarTiledOut : 0);
  const bool accel_allowed = c->accel_ok && !(p->flags & RT_FLAG_NO_ACCEL) && !(p->flags & RT_FLAG_NO_JIT);
  const bool mixed_allowed = c->mixed_ok && !(p->flags & RT_FLAG_NO_MIXED) && !(p->flags & RT_FLAG_NO_JIT);
  if (trav == RT_TRAV_ACCEL && !accel_allowed) trav = mixed_allowed && (p->flags & RT_FLAG_FORCE_ACCEL) ? RT_TRAV_MIXED : RT_TRAV_LANE;
  if (trav == RT_TRAV_MIXED && !mixed_allowed) trav = RT_TRAV_LANE;
  if (trav == RT_TRAV_PACKET && c->img.stack_need > 64) trav = RT_TRAV_LANE;
  hipFunction_t jit_fn = nullptr, jit_probe = nullptr;
  bool jit_lane = false;
  c->jit_source = RT_JIT_NONE;
  c->jit_ms = 0.0;
  auto note_jit = [c](const rt::JitKernels &jk) {
    c->jit_source = std::max(c->jit_source, jk.source);
    c->jit_ms += jk.ms;
    fill_kernel_info(c->counted ? jk.meta_count : jk.meta_render, jk.compiler, &c->used_kernel);
  };
  c->used_kernel = rt_kernel_info{};
  c->used_fold = false;
  if (trav < 0 || trav == RT_TRAV_STATIC) {
    rt::JitKernels jk;
    std::string why;
    const bool want_fold = c->fold_enabled && !(p->flags & RT_FLAG_NO_FOLD) &&
                           ray_bound(c->img, cam, p) <= kFoldRayBound;
    if (rt::jit_kernels(c->img, c->variant | trace_bit | (c->img.has_noise ? rt::kVarCoop : 0), c->jit_budget, want_fold,
                        &jk, &why)) {
      note_jit(jk);
      c->used_fold = jk.folded;
      jit_fn = c->counted ? jk.render_count : jk.render;
      jit_probe = jk.probe;
      c->jit_visits = jk.visits;
      trav = RT_TRAV_STATIC;
    } else {
      c->jit_why = why;
      trav = accel_allowed ? RT_TRAV_ACCEL : (mixed_allowed ? RT_TRAV_MIXED : RT_TRAV_LANE);
    }
  }
  if (!jit_fn && stackless) {   // the straight-line kernel was expected but not obtained: stacks after all
    stackless = false;
    stack_bytes = full_stack_bytes;
    if (rc_bytes + stack_bytes > kLdsPerCu - kLdsReserve) return RT_ERR_STACK;
    if (c->lds && static_cast<size_t>(scene_lds_words) * 4 + rc_bytes + stack_bytes > kLdsPerCu - kLdsReserve) {
      c->lds = false;
      scene_lds_words = 0;
      c->variant &= ~rt::kVarLds;
    }
  }
  if (trav == RT_TRAV_MIXED) {
    rt::JitKernels jk;
    std::string why;
    if (rt::jit_mixed_kernels(c->img, c->variant | trace_bit, &jk, &why)) {
      note_jit(jk);
      jit_fn = c->counted ? jk.render_count : jk.render;
      jit_probe = jk.probe;
      jit_lane = true;   // per-lane stacks
    } else {
      c->jit_why = why;
      trav = RT_TRAV_LANE;
    }
  }
  if (trav == RT_TRAV_ACCEL) {
    rt::JitKernels jk;
    std::string why;
    if (rt::jit_accel_kernels(c->img, c->variant | trace_bit, c->accel_q ? 2 : (c->accel_w4 ? 1 : 0), &jk, &why)) {
      note_jit(jk);
      jit_fn = c->counted ? jk.render_count : jk.render;
      jit_probe = jk.probe;
      jit_lane = true;   // per-lane stacks
    } else {
      c->jit_why = why;
      trav = RT_TRAV_LANE;
    }
  }
  if (trav == RT_TRAV_LANE && c->lane_jit && !(p->flags & RT_FLAG_NO_JIT)) {
    // per-lane DFS compiled for the node kinds this scene has (fewer branches and registers than
    // the offline all-kinds kernel); the offline kernel stays the fallback
    rt::JitKernels jk;
    std::string why;
    if (rt::jit_lane_kernels(c->img, c->variant | trace_bit, &jk, &why)) {
      note_jit(jk);
      jit_fn = c->counted ? jk.render_count : jk.render;
      jit_probe = jk.probe;
      jit_lane = true;
    } else if (c->jit_why.empty()) {
      c->jit_why = why;
    }
  }
  if (trav == RT_TRAV_PACKET) c->variant |= rt::kVarPacket;
  if (jit_fn && !jit_lane) stack_bytes = kRngSlotBytes;   // straight-line traversal: no stacks (the RNG slots stay)
  // the verified walk's top nodes staged in LDS (breadth-first prefix of the SAH tree) where the scene
  // itself is not: they take the scene's place at the start of the block's LDS
  uint32_t accel_lds_nodes = 0;
  if (trav == RT_TRAV_ACCEL && !c->lds && c->accel_lds_nodes > 0) {
    const uint32_t node_words = c->accel_q ? rt::kAccel4QNodeWords : (c->accel_w4 ? rt::kAccel4NodeWords : rt::kAccelNodeWords);
    // the same LDS bytes either way by default (64 2-wide nodes = 32 4-wide ones); RT_ACCEL_LDS_NODES counts nodes
    const uint32_t want = c->accel_lds_set ? c->accel_lds_nodes : c->accel_lds_nodes * rt::kAccelNodeWords / node_words;
    accel_lds_nodes = std::min<uint32_t>(want, static_cast<uint32_t>((c->accel_q ? c->accel.wide_q_words.size() : c->accel_w4 ? c->accel.wide_words.size()
                                                                                  : c->accel.node_words.size()) / node_words));
    // only what the block's LDS budget leaves after the colour-stack levels and the stacks (an explicit
    // RT_RC_LDS_LEVELS may already take most of it): the staging shrinks, the launch never exceeds 160 KiB
    const uint32_t cb = jit_fn == nullptr ? 4u : (byte_ok ? 1u : (narrow_ok ? 2u : 4u));
    const uint32_t per_word = 4u / cb;
    const size_t used = ((rc_levels + per_word - 1) / per_word * per_word) * rc_level_bytes(cb) + stack_bytes + kLdsReserve;
    const size_t node_bytes = static_cast<size_t>(node_words) * 4;
    size_t room = used < kLdsPerCu ? (kLdsPerCu - used) / node_bytes : 0;
    // By default the colour stack comes first: staged nodes only take what a block at kRcLdsOnlyBlocks per CU leaves
    // once every level fits beside the stacks (round 5: the 10k walk's parked pixel sum made the stacks 3 KB larger,
    // and 64 staged nodes then left 8 of its 16 levels, whose HBM twins cost 1.6 GB per frame at the same speed:
    // profiles/r05_ab_s37_10k.jsonl).  An explicit RT_ACCEL_LDS_NODES keeps the round-4 rule above.
    if (!c->accel_lds_set && c->rc_lds_auto) {
      const size_t all = static_cast<size_t>((mb + per_word - 1) / per_word * per_word) * rc_level_bytes(cb) + stack_bytes + kLdsReserve;
      const size_t budget = kLdsPerCu / kRcLdsOnlyBlocks;
      room = std::min(room, all < budget ? (budget - all) / node_bytes : 0);
    }
    accel_lds_nodes = static_cast<uint32_t>(std::min<size_t>(accel_lds_nodes, room));
    scene_lds_words = accel_lds_nodes * node_words;
  }
  // the offline kernels use 32-bit codes; run-time ones 16-bit (narrow) or 8-bit (byte) where the scene allows
  const uint32_t code_bytes = jit_fn == nullptr ? 4u : (byte_ok ? 1u : (narrow_ok ? 2u : 4u));
  const bool lds_only_kernel = jit_fn != nullptr && rc_lds_only;   // its variant carries kVarRcLds (trace_bit)
  const uint32_t codes_per_word = 4u / code_bytes;
  const size_t level_bytes = rc_level_bytes(code_bytes);
  rc_levels = (rc_levels + codes_per_word - 1) / codes_per_word * codes_per_word;   // whole LDS words per lane
  c->lds_bytes = static_cast<size_t>(scene_lds_words) * 4 + rc_levels * level_bytes + stack_bytes;
  c->used_traversal = trav;
  if (!jit_fn) {   // an offline kernel of this library: its attributes (the allocator's spill counts are not among them)
    int vg = -1, sc = -1;
    rt::render_kernel_attrs(c->variant, &vg, &sc);
    rt::KernelMeta m;
    m.vgprs = vg;
    m.scratch = sc;
    fill_kernel_info(m, "", &c->used_kernel);
    c->used_kernel.run_time = 0;
    c->used_kernel.loader[0] = '\0';
  }
  int per_cu = jit_fn ? rt::jit_blocks_per_cu(jit_fn, c->lds_bytes) : rt::render_blocks_per_cu(c->variant, c->lds_bytes);
  if (c->blocks_per_cu > 0) per_cu = std::min(c->blocks_per_cu, per_cu);   // fewer blocks: more LDS levels each
  if (c->rc_lds_auto) {
    // give the colour stack every LDS byte the resident blocks leave unused (deeper paths then never
    // touch HBM), without lowering residency
    const size_t per_block = kLdsPerCu / static_cast<size_t>(std::max(per_cu, 1));
    const size_t fixed = static_cast<size_t>(scene_lds_words) * 4 + stack_bytes;
    if (per_block > fixed) {
      // keep 1 KiB per block in reserve: resident blocks whose LDS sums to within ~1% of 160 KiB were
      // measured NOT to be co-resident on gfx950 (3 x 53808 B: a third of the blocks started late)
      uint32_t fit = per_block > fixed + kLdsReserve ? static_cast<uint32_t>((per_block - fixed - kLdsReserve) / level_bytes) : 0u;
      uint32_t lv = std::min<uint32_t>(mb, std::min<uint32_t>(kRcLdsMaxLevels, std::max(fit, rc_levels)));
      lv = std::max<uint32_t>(lv / codes_per_word * codes_per_word, rc_levels);   // whole words (rc_levels already is)
      // a kernel without HBM levels (kVarRcLds) holds every level: mb rounded up to whole words (the host check
      // above predicts they fit at kRcLdsOnlyBlocks = 6 blocks/CU; verified below once the layout is final)
      if (lds_only_kernel) lv = (mb + codes_per_word - 1) / codes_per_word * codes_per_word;
      if (lv > rc_levels || lds_only_kernel) {
        const size_t lds2 = fixed + lv * level_bytes;
        int per_cu2 = jit_fn ? rt::jit_blocks_per_cu(jit_fn, lds2) : rt::render_blocks_per_cu(c->variant, lds2);
        if (c->blocks_per_cu > 0) per_cu2 = std::min(c->blocks_per_cu, per_cu2);
        if (per_cu2 >= per_cu || lds_only_kernel) {
          rc_levels = lv;
          c->lds_bytes = lds2;
        }
      }
    }
  }
  if (lds_only_kernel) {
    // The kVarRcLds decision was made on a predicted layout (before the kernels were built: straight-line stackless
    // traversal, 4 KiB of staged SAH nodes).  The kernel stores every level in LDS, so the final layout must hold all
    // mb levels within one block's LDS, or the render is made again without that variant (nothing is enqueued yet);
    // residency is then whatever that layout allows (the grid never exceeds the resident blocks).
    const uint32_t need_levels = (mb + codes_per_word - 1) / codes_per_word * codes_per_word;
    if (rc_levels < need_levels || c->lds_bytes + kLdsReserve > kLdsPerCu) {
      if (std::getenv("RT_DEBUG"))
        std::fprintf(stderr, "[rt] LDS-only colour stack does not fit (%u of %u levels, %zu B): rebuilding with HBM levels\n",
                     rc_levels, need_levels, c->lds_bytes);
      c->rc_lds_only_off = true;
      const int r = rt_context_render_ppm(c, cam, p, out_dev, out8_dev, stream);
      c->rc_lds_only_off = false;
      return r;
    }
    int per_cu_lds = rt::jit_blocks_per_cu(jit_fn, c->lds_bytes);
    if (c->blocks_per_cu > 0) per_cu_lds = std::min(c->blocks_per_cu, per_cu_lds);
    per_cu = std::min(per_cu, per_cu_lds);
  }
  // Deep-level pool (kVarRcPool kernels): rc_pool chunks per wave of the levels past the LDS ones.  With automatic
  // levels the pool takes its bytes from the per-lane levels (the most levels that fit beside it at this residency);
  // with pinned levels (RT_RC_LDS_LEVELS) it is added if the residency keeps it.  Fewer chunks if neither fits.
  uint32_t pool_chunks = 0;
  size_t pool_base = c->lds_bytes, pool_bytes = 0;
  if (jit_fn && pool_kernel) {
    const size_t fixed = c->lds_bytes - rc_levels * level_bytes;   // scene (or SAH top nodes), stacks, RNG slots
    const size_t cap = kLdsPerCu / static_cast<size_t>(std::max(per_cu, 1)) - kLdsReserve;
    auto bytes_of = [&](uint32_t P, uint32_t L) {
      return static_cast<size_t>(rt::kWavesPerBlock) * (rt::kRcPoolHead + P * (mb > L ? mb - L : 0u)) * 4u;
    };
    const uint32_t min_levels = std::max<uint32_t>(c->rc_lds_levels, codes_per_word);
    uint32_t L = rc_levels;
    for (uint32_t P = static_cast<uint32_t>(c->rc_pool); P > 0 && rc_levels < mb; --P) {
      uint32_t l = rc_levels;
      if (c->rc_lds_auto)
        while (l > min_levels && fixed + l * level_bytes + bytes_of(P, l) > cap) l -= codes_per_word;
      if (fixed + l * level_bytes + bytes_of(P, l) <= cap) {
        pool_chunks = P;
        L = l;
        break;
      }
    }
    rc_levels = L;
    pool_base = fixed + rc_levels * level_bytes;
    pool_bytes = bytes_of(pool_chunks, rc_levels);   // the headers even without chunks (the kernel sets them)
    c->lds_bytes = pool_base + pool_bytes;
  }
  c->used_pool_chunks = pool_chunks;
  // output staging slots (coalesced tile writes): as many as the requested number that keep this residency, from the
  // LDS the blocks leave unused (kLdsReserve per block kept, as above)
  uint32_t stage_slots = 0;
  for (uint32_t r = jit_fn ? static_cast<uint32_t>(std::max(c->stage_slots, 0)) : 0u; r > 0 && p->row_count > 0; --r) {
    const size_t l = c->lds_bytes + r * kStageBlockBytes + kStageWaveExtraBytes;
    if (static_cast<size_t>(std::max(per_cu, 1)) * (l + kLdsReserve) <= kLdsPerCu) {
      stage_slots = r;
      break;
    }
  }
  const size_t stage_base = c->lds_bytes;
  c->lds_bytes += stage_slots ? stage_slots * kStageBlockBytes + kStageWaveExtraBytes : 0u;
  c->used_stage_slots = stage_slots;
  const uint32_t rc_lds_words = static_cast<uint32_t>(rc_levels * level_bytes / 4);
  c->used_kernel.blocks_per_cu = c->blocks_per_cu > 0 ? std::min(c->blocks_per_cu, per_cu) : per_cu;
  uint64_t blocks = static_cast<uint64_t>(c->blocks_per_cu > 0 ? std::min(c->blocks_per_cu, per_cu) : per_cu) *
                    static_cast<uint64_t>(c->cu_count);
  const uint64_t needed = (static_cast<uint64_t>(n) + rt::kBlock - 1) / rt::kBlock;
  blocks = std::max<uint64_t>(1, std::min(blocks, needed));
  const uint32_t threads = static_cast<uint32_t>(blocks * rt::kBlock);
  if (std::getenv("RT_DEBUG"))
    std::fprintf(stderr, "[rt] launch: traversal %d, %d blocks/CU, %llu blocks, lds %zu B (scene %u words, colour-stack levels %u, "
                 "stack cap %u, tiles %ux%u, staging slots %u, pool chunks %u)\n",
                 trav, per_cu, static_cast<unsigned long long>(blocks), c->lds_bytes, scene_lds_words, rc_levels, stack_cap,
                 1u << c->tile_shift, 64u >> c->tile_shift, stage_slots, pool_chunks);

  // tiles of 64 pixels (RenderArgs::tile_shift): 8x8 by default (kDefaultTileShift); RT_TILE_W = 16 / 32 / 64 gives wider
  // tiles (32x2: every 128-B line of a 32-aligned float frame row belongs to one tile)
  const uint32_t tile_shift = c->tile_shift;
  const uint32_t tw = 1u << tile_shift, th = 64u >> tile_shift;
  const uint32_t tiles_x = (static_cast<uint32_t>(p->width) + tw - 1) / tw;
  const uint32_t n_ids = 64u * ((static_cast<uint32_t>(p->row_count) + th - 1) / th) * tiles_x;
  // RNG: the phase bases of this shard's rows and the column tables (host, once per geometry: a few ms; the
  // per-pixel jumps — one nibble-table product each — run in the render kernel at tile pickup) and the per-wave
  // slots
  // The tables are rewritten in place when the geometry changes, so the upload is stream-ordered: an async copy on
  // the frame's stream from pinned staging, after the previous frame's render (stream order; a frame on another stream
  // waited for the previous frame's end at entry), so a frame still in flight keeps reading the table it was launched
  // with (a blocking null-stream copy did not wait for non-blocking streams).
  {
    // (phase width = the tile width: every lane of a tile applies the same column table)
    const uint64_t key[5] = {p->seed, static_cast<uint64_t>(p->width) | (static_cast<uint64_t>(tile_shift) << 32),
                             static_cast<uint64_t>(p->row_offset), static_cast<uint64_t>(p->row_stride),
                             static_cast<uint64_t>(p->row_count)};
    const int cols_key = p->width | static_cast<int>(tile_shift << 24);
    const bool rows_new = std::memcmp(key, c->rows_key, sizeof key) != 0, cols_new = c->cols_width != cols_key;
    auto upload = [s](DevBuf &dst, PinBuf &stage, const std::vector<uint32_t> &v) {
      const size_t n = v.size() * 4;
      if (dst.ensure(n) != hipSuccess || stage.stage(v.data(), n) != hipSuccess ||
          hipMemcpyAsync(dst.p, stage.p, n, hipMemcpyHostToDevice, s) != hipSuccess ||
          hipEventRecord(stage.done, s) != hipSuccess)
        return false;
      stage.pending = true;
      return true;
    };
    if (rows_new) {
      std::vector<uint32_t> rb;
      rt::xorwow_phase_bases(p->seed, p->width, p->row_offset, p->row_stride, p->row_count, &rb, static_cast<int>(tile_shift));
      if (!upload(c->rng_rows, c->rows_stage, rb)) return RT_ERR_HIP;
      std::memcpy(c->rows_key, key, sizeof key);
    }
    if (cols_new) {
      std::vector<uint32_t> ct;
      rt::xorwow_column_tables(p->width, &ct, static_cast<int>(tile_shift));
      if (!upload(c->rng_cols, c->cols_stage, ct)) return RT_ERR_HIP;
      c->cols_width = cols_key;
    }
  }
  if (c->rc.ensure(static_cast<size_t>(mb) * threads * 4) != hipSuccess) return RT_ERR_HIP;   // (wide codes' size)
  c->used_rc_levels = rc_levels;
  c->rc_audit_bytes = 0;
  // every slot 0xff..: a written code never is — narrow codes are record indices < 65535 (narrow_ok), wide
  // record codes have the sign bit clear, greys are finite with the sign clear, and a texel code's offset is at
  // most pixel_words - 3 < 0x7fffffff (rt_layout.h kRc*)
  if (p->flags & RT_FLAG_RC_AUDIT) {
    c->rc_audit_bytes = static_cast<size_t>(mb) * threads * code_bytes;
    c->rc_audit_code = code_bytes;
    if (hipMemsetAsync(c->rc.p, 0xff, c->rc_audit_bytes, s) != hipSuccess) return RT_ERR_HIP;
  }

  uint32_t seed_base[6];
  rt::xorwow_seed_base(p->seed, seed_base);

  rt::RenderArgs a{};
  a.scene = static_cast<const uint32_t *>(c->scene.p);
  a.scene_words = static_cast<uint32_t>(c->img.words.size());
  a.off_mats = c->img.off_mats; a.off_texs = c->img.off_texs; a.off_perlin = c->img.off_perlin;
  a.off_pixels = c->img.off_pixels;
  a.pixel_words = static_cast<uint32_t>(c->img.words.size()) - c->img.off_pixels;
  a.root = c->img.root;
  a.stack_cap = stack_cap_launch;
  a.accel_nodes = c->accel_nodes;
  a.accel_prims = c->accel_prims;
  a.accel_root = c->accel.root;
  a.accel_lds_nodes = accel_lds_nodes;
  a.accel_wide = (trav == RT_TRAV_ACCEL && c->accel_w4) ? c->accel_wide : 0u;
  a.accel_node_u4 = (trav == RT_TRAV_ACCEL && c->accel_w4 && !c->accel_q) ? 8u : 4u;
  a.accel_fallbacks = static_cast<uint32_t *>(c->work.p) + 12;   // zeroed with the work counters
  a.mix_nodes = c->mix_nodes;
  a.mix_prims = c->mix_prims;
  a.mix_fallbacks = static_cast<uint32_t *>(c->work.p) + 11;   // reasons at work[2], work[3]
  a.mix_no_proof = c->mix_no_proof ? 1u : 0u;
  a.rc_lds_word = scene_lds_words;
  a.rc_lds_levels = rc_levels;
  a.rc_pool_word = static_cast<uint32_t>(pool_base / 4);
  a.rc_pool_chunks = pool_chunks;
  a.rc_tex0 = c->img.mat_count;
  a.rc_consts = c->img.rec_consts;
  a.stack_lds_word = scene_lds_words + rc_lds_words;
  const rtr_vec3 *v3s[6] = {&cam->pixel00, &cam->delta_u, &cam->delta_v, &cam->center, &cam->defocus_u, &cam->defocus_v};
  float *dst[6] = {a.p00, a.du, a.dv, a.center, a.dfu, a.dfv};
  for (int k = 0; k < 6; ++k) { dst[k][0] = v3s[k]->x; dst[k][1] = v3s[k]->y; dst[k][2] = v3s[k]->z; }
  a.defocus_angle = cam->defocus_angle;
  a.width = p->width; a.row_offset = p->row_offset; a.row_stride = p->row_stride;
  a.spp = p->samples_per_pixel;
  a.max_bounces = static_cast<int32_t>(mb);
  a.bg[0] = p->background.x; a.bg[1] = p->background.y; a.bg[2] = p->background.z;
  a.sample_scale = 1.0f / static_cast<float>(p->samples_per_pixel);   // :1657
  a.n_pixels = n;
  a.rows = static_cast<uint32_t>(p->row_count);
  a.tiles_x = tiles_x;
  a.tile_shift = tile_shift;
  a.stage_slots = stage_slots;
  a.stage_word = static_cast<uint32_t>(stage_base / 4);   // after the stacks and RNG slots (an even word: 8-B masks)
  a.n_ids = n_ids;
  a.rng_rows = static_cast<const uint32_t *>(c->rng_rows.p);
  a.rng_nib = static_cast<const uint32_t *>(c->rng_cols.p);
  a.rng_d = seed_base[0];
  a.rng_slot_word = scene_lds_words + rc_lds_words + static_cast<uint32_t>((stack_bytes - kRngSlotBytes) / 4);
  // tile-major output: the render kernel (a run-time kernel built with kVarTiledOut) writes the float frame tile by tile
  // into c->tiled; untile_kernel then writes the caller's row-major floats and the PPM bytes (after the render, below)
  const bool tiled = tiled_kernel && jit_fn != nullptr;
  c->used_tiled = tiled;
  if (tiled && c->tiled.ensure(static_cast<size_t>(n_ids) * 3u * 4u) != hipSuccess) return RT_ERR_HIP;
  a.out = tiled ? static_cast<float *>(c->tiled.p) : out_dev;
  a.out8 = tiled ? nullptr : out8_dev;
  a.rc = c->rc.p;
  a.threads = threads;
  a.work = static_cast<uint32_t *>(c->work.p);
  a.counters = static_cast<unsigned long long *>(c->counters.p);
  a.tile_order = nullptr;
  a.probe_cost = nullptr;
  a.reverse_tiles = c->sched == 2 ? 1u : 0u;
  a.fold_violation = static_cast<uint32_t *>(c->work.p) + 15;   // zeroed with the work counters
  a.black_skip = c->black_skip ? 1u : 0u;
  a.coop_noise = c->coop_noise;
  a.max_tries = c->max_tries;
  a.defer_lanes = c->defer_lanes;
  a.defer_trace = c->defer_trace;
  a.trace_min_iters = c->trace_min_iters;
  a.prio_chunk = 64u;   // whole tiles unless the longest-first schedule splits its costliest ones
  a.prio_lanes = 64u;   // no sparse waves (the probe launch keeps these defaults)
  a.prio_mix = 0u;
  a.tail_prio = 0u;   // the probe launch keeps it off
  a.span = nullptr;   // set for the render launch below (the probe launch keeps no span)
  const uint32_t n_tiles = a.n_ids / 64u;
  c->used_lpt = c->sched == 3 || (c->sched == 0 && p->samples_per_pixel >= kLptMinSpp);
  a.wave_trace = nullptr;
  c->wave_trace_words = 0;
  if (!c->wave_trace_path.empty()) {
    c->wave_trace_words = static_cast<size_t>(blocks) * rt::kWavesPerBlock * rt::kWaveTraceWords;
    if (c->wave_trace.ensure(c->wave_trace_words * 8) != hipSuccess) return RT_ERR_HIP;
    if (hipMemsetAsync(c->wave_trace.p, 0, c->wave_trace_words * 8, s) != hipSuccess) return RT_ERR_HIP;
    a.wave_trace = static_cast<unsigned long long *>(c->wave_trace.p);
  }

  if (hipMemsetAsync(c->work.p, 0, 256, s) != hipSuccess) return RT_ERR_HIP;
  if (c->counted && hipMemsetAsync(c->counters.p, 0, RT_CNT__COUNT * 8, s) != hipSuccess) return RT_ERR_HIP;
  a.prim_lists = nullptr;
  a.prim_counts = nullptr;
  const bool prim_on = c->prim_mode == 1 || (c->prim_mode < 0 && c->accel_ok && c->accel.spheres >= kPrimMinSpheres);
  if (trav == RT_TRAV_ACCEL && prim_on && c->accel_ok) {
    // primary-ray candidate lists of this frame's camera (device/prim_lists.h), before the probe and the render
    float prim_rho = 0.0f;
    const rt::PrimListGeom g = make_prim_geom(cam, p, tiles_x, tile_shift, c->accel_half_motion, &prim_rho);
    const uint32_t words = rt::kPrimEntryWords;
    if (c->prim_lists.ensure(static_cast<size_t>(n_tiles) * c->prim_cap * words * 4) != hipSuccess ||
        c->prim_counts.ensure(static_cast<size_t>(n_tiles) * 4) != hipSuccess)
      return RT_ERR_HIP;
    const uint32_t *sw = static_cast<const uint32_t *>(c->scene.p);
    if (rt::launch_prim_lists(g, sw + c->accel_nodes, c->accel.root, sw + c->accel_prims, n_tiles, c->prim_cap, words,
                              static_cast<uint32_t *>(c->prim_lists.p), static_cast<uint32_t *>(c->prim_counts.p), s) != hipSuccess)
      return RT_ERR_HIP;
    a.prim_words = words;
    a.prim_lists = static_cast<const uint32_t *>(c->prim_lists.p);
    a.prim_counts = static_cast<const uint32_t *>(c->prim_counts.p);
    a.prim_cap = c->prim_cap;
    a.prim_rho = prim_rho;
    if (std::getenv("RT_DEBUG")) {   // diagnostics only: a synchronous copy of the counts
      std::vector<uint32_t> cnt(n_tiles);
      if (hipStreamSynchronize(s) == hipSuccess &&
          hipMemcpy(cnt.data(), c->prim_counts.p, cnt.size() * 4, hipMemcpyDeviceToHost) == hipSuccess) {
        uint64_t with = 0, sum = 0, mx = 0;
        for (uint32_t v : cnt)
          if (v != rt::kPrimListNone) { ++with; sum += v; mx = std::max<uint64_t>(mx, v); }
        std::fprintf(stderr, "[rt] primary lists: %llu of %u tiles, mean %.1f, max %llu spheres\n",
                     static_cast<unsigned long long>(with), n_tiles, with ? static_cast<double>(sum) / with : 0.0,
                     static_cast<unsigned long long>(mx));
      }
    }
  }
  // no seeding launch: the render kernel seeds each pixel's state at tile pickup (init_ms is the empty interval)
  if (hipEventRecord(c->ev[0], s) != hipSuccess) return RT_ERR_HIP;
  if (hipEventRecord(c->ev[1], s) != hipSuccess) return RT_ERR_HIP;
  if (c->used_lpt) {
    // longest-first schedule: probe probe_per_tile throwaway 1-spp paths per tile (their own RNG,
    // no output), then counting-sort tiles by probe cost; counted in render_ms
    if (c->tile_cost.ensure(static_cast<size_t>(n_tiles) * 4) != hipSuccess ||
        c->tile_order.ensure((static_cast<size_t>(n_tiles) + 16) * 4) != hipSuccess)   // + the class offsets
      return RT_ERR_HIP;
    if (hipMemsetAsync(c->tile_cost.p, 0, static_cast<size_t>(n_tiles) * 4, s) != hipSuccess) return RT_ERR_HIP;
    rt::RenderArgs pa = a;
    pa.probe_cost = static_cast<uint32_t *>(c->tile_cost.p);
    pa.probe_per_tile = c->probe_per_tile ? c->probe_per_tile
                                          : static_cast<uint32_t>(std::min(64, std::max(8, p->samples_per_pixel / 4)));
    pa.n_ids = n_tiles * pa.probe_per_tile;
    pa.spp = 1;
    pa.out = nullptr;
    pa.out8 = nullptr;
    pa.rng_rows = nullptr;
    pa.work = static_cast<uint32_t *>(c->work.p) + 8;
    pa.wave_trace = nullptr;
    pa.fold_violation = static_cast<uint32_t *>(c->work.p) + 14;   // probe rays: flag ignored
    pa.accel_fallbacks = static_cast<uint32_t *>(c->work.p) + 13;  // probe rays: not reported
    pa.mix_fallbacks = nullptr;   // probe rays: not reported
    const hipError_t pe = jit_probe ? rt::jit_launch(jit_probe, pa, static_cast<uint32_t>(blocks), c->lds_bytes, s)
                                    : rt::launch_render(pa, c->variant & ~rt::kVarCount, static_cast<uint32_t>(blocks),
                                                        c->lds_bytes, s);
    if (pe != hipSuccess) return RT_ERR_HIP;
    // XCD classes (RT_XCD_CLASSES): 8x8 tiles handed out whole, no sparse / mixed hot waves — per-XCD queues, so that
    // each 128-B line of the frame is written through one XCD's L2
    const bool mix_sched0 = c->prio_mix == 1 || (c->prio_mix < 0 && c->used_traversal == RT_TRAV_MIXED);
    const bool classes = c->xcd_classes && tile_shift == 3u && !mix_sched0 && !(c->img.has_noise && c->coop_noise) &&
                         (c->prio_chunk < 0 || c->prio_chunk >= 64) && (c->prio_lanes == 0 || c->prio_lanes >= 64);
    if (rt::launch_order(pa.probe_cost, n_tiles, static_cast<uint32_t *>(c->tile_order.p), classes ? tiles_x : 0u, s) !=
        hipSuccess)
      return RT_ERR_HIP;
    a.tile_order = static_cast<const uint32_t *>(c->tile_order.p);
    a.cls_off = classes ? static_cast<const uint32_t *>(c->tile_order.p) + n_tiles : nullptr;
    c->used_classes = classes;
    // noise scenes: sparse hot waves (below) by default, over the 16 costliest tiles; the verified mixed
    // walk: mixed hot waves over the costliest quarter of the tiles (below)
    const bool mix_sched = c->prio_mix == 1 || (c->prio_mix < 0 && c->used_traversal == RT_TRAV_MIXED);
    const bool noise_sched = c->img.has_noise && c->coop_noise && !mix_sched;
    const int lanes_hot = c->prio_lanes != 0 ? c->prio_lanes : (mix_sched ? kMixLanes : noise_sched ? kSparseLanes : 0);
    const int pt = c->prio_tiles >= 0 ? c->prio_tiles
                                      : mix_sched ? static_cast<int>(std::max<uint32_t>(n_tiles / 4u, kSparseTiles))
                                      : ((lanes_hot > 0 && lanes_hot < 64) ? kSparseTiles : kPrioTiles);
    a.prio_ids = static_cast<uint32_t>(std::min<uint64_t>(static_cast<uint64_t>(pt) * 64u, a.n_ids));
    // The costliest tiles of a noise scene hold pixels whose paths are trapped between noise surfaces
    // (the Perlin scene's contact point: ~35k serial rounds per pixel); handed out one pixel at a time
    // they spread over many waves, each with few noise lanes, whose octaves the idle lanes then share
    // (measured on scene 17, d50, spp 1024: 204 ms whole tiles without cooperation, 168 with, 135 with
    // single pixels; scene 0 and Cornell lose 4-10 % with split tiles, so they keep whole tiles)
    const int pcn = c->prio_chunk >= 0 ? c->prio_chunk : ((noise_sched || mix_sched) ? 1 : 64);
    a.prio_chunk = a.prio_ids ? static_cast<uint32_t>(pcn) : 64u;
    // Sparse hot waves: a wave holding pixels of those tiles keeps at most lanes_hot of them busy and takes
    // no other pixel meanwhile, so the trapped chains run in waves with few divergent lanes (and issue
    // priority) for the whole frame, not only once the rest is done (single-pixel hand-out).  Scene 17:
    // 135-139 -> 99-101 ms per frame, scene 19: 205 -> 165; scene 0 +12 %, Cornell +5 %, 10k +-3 %, so
    // noise scenes only (profiles/r03_ab_sparse_hot_waves_*.jsonl).  RT_PRIO_LANES=64 turns it off.
    // Mixed hot waves: the same cap, but the wave's other lanes take ordinary tiles meanwhile, so the
    // costliest pixels start at once, spread over every wave, and their walks share trips with cheap
    // pixels (the paused walk lets those finish their samples meanwhile).  final_scene: see DESIGN §2.
    if (a.prio_ids && lanes_hot > 0 && lanes_hot < 64) {
      a.prio_lanes = static_cast<uint32_t>(lanes_hot);
      a.prio_mix = mix_sched ? 1u : 0u;
      a.prio_chunk = 1u;
    }
  }
  // Tail issue priority: on for the verified mixed walk (final_scene 800x800 spp 64: 638-649 -> 598-611 ms
  // per frame), within noise elsewhere (scene 0 -1 %, 10k +1 %; profiles/r03_ab_tail_prio.jsonl)
  a.tail_prio = (c->tail_prio == 1 || (c->tail_prio < 0 && c->used_traversal == RT_TRAV_MIXED)) ? 1u : 0u;
  // Tail pieces (RT_TAIL_CHUNK, RT_TAIL_GEN): the last tail_gen x (grid lanes) ids of the longest-first order go out in
  // tail_chunk-pixel pieces, so that a wave holds few pixels it has not started when the queue drains (whole tiles: up
  // to 63), and the waves' last pixels start closer together.  Longest-first order only, whole-tile queues.
  a.tail_ids = 0u;
  a.tail_chunk = 0u;
  if (c->used_lpt && !a.cls_off && c->tail_chunk > 0) {
    const uint32_t prio_lo = a.prio_chunk < 64u ? a.prio_ids : 0u;   // split costliest ids come first, never in the tail
    const double want = c->tail_gen * static_cast<double>(threads);
    const uint32_t room = (a.n_ids - std::min(a.n_ids, (prio_lo + 63u) / 64u * 64u)) / 64u * 64u;
    a.tail_ids = std::min<uint32_t>(room, static_cast<uint32_t>(std::max(0.0, want) / 64.0) * 64u);
    a.tail_chunk = a.tail_ids ? static_cast<uint32_t>(c->tail_chunk) : 0u;
  }
  c->used_tail_ids = a.tail_ids;
  if (std::getenv("RT_DEBUG") && c->used_lpt)
    std::fprintf(stderr, "[rt] tile queues: %s, tail pieces: %u ids in %u-pixel pieces\n", a.cls_off ? "8 XCD classes" : "one",
                 a.tail_ids, a.tail_chunk);
  a.span = reinterpret_cast<unsigned long long *>(static_cast<uint32_t *>(c->work.p) + kSpanWord);   // zeroed above
  if (hipEventRecord(c->ev[3], s) != hipSuccess) return RT_ERR_HIP;
  const hipError_t le = jit_fn ? rt::jit_launch(jit_fn, a, static_cast<uint32_t>(blocks), c->lds_bytes, s)
                               : rt::launch_render(a, c->variant, static_cast<uint32_t>(blocks), c->lds_bytes, s);
  if (le != hipSuccess) return RT_ERR_HIP;
  if (tiled && rt::launch_untile(static_cast<const float *>(c->tiled.p), out_dev, out8_dev, static_cast<uint32_t>(p->row_count),
                                 static_cast<uint32_t>(p->width), tiles_x, tile_shift, s) != hipSuccess)
    return RT_ERR_HIP;
  if (hipEventRecord(c->ev[2], s) != hipSuccess) return RT_ERR_HIP;
  c->ev_recorded = true;
  c->last_cam = *cam;
  c->last_params = *p;
  c->last_out = out_dev;
  c->last_out8 = out8_dev;
  c->rendered = true;
  return RT_OK;
}

int rt_context_timing(rt_context *c, rt_stats *st) {
  if (!c || !st) return RT_ERR_INVALID_ARG;
  std::memset(st, 0, sizeof *st);
  st->stack_needed = static_cast<int32_t>(c->img.stack_need);
  st->scene_in_lds = c->lds ? 1 : 0;
  st->traversal = c->used_traversal;
  st->jit_visits = static_cast<int32_t>(c->jit_visits);
  st->folded = c->used_fold ? 1 : 0;
  st->fold_rerenders = static_cast<int32_t>(c->fold_violations);
  st->accel_spheres = c->accel_ok ? static_cast<int32_t>(c->accel.spheres) : 0;
  st->accel_depth = c->accel_ok ? static_cast<int32_t>(c->accel.depth) : 0;
  st->mix_macros = c->mixed_ok ? static_cast<int32_t>(c->mixed.macros) : 0;
  if (!c->rendered) return RT_OK;
  st->rc_lds_levels = static_cast<int32_t>(c->used_rc_levels);
  st->rc_pool_chunks = static_cast<int32_t>(c->used_pool_chunks);
  st->tiled_out = c->used_tiled ? 1 : 0;
  st->jit_source = c->jit_source;
  st->jit_ms = c->jit_ms;
  st->kernel = c->used_kernel;
  DeviceGuard g(c->device);
  if (hipEventSynchronize(c->ev[2]) != hipSuccess) return RT_ERR_HIP;
  if (c->used_fold) {
    // a ray outside the host's bound voids the folding precondition: render the frame again unfolded
    uint32_t v = 0;
    if (hipMemcpy(&v, static_cast<uint32_t *>(c->work.p) + 15, 4, hipMemcpyDeviceToHost) != hipSuccess)
      return RT_ERR_HIP;
    if (v) {
      c->fold_violations++;
      rt_params q = c->last_params;
      q.flags |= RT_FLAG_NO_FOLD;
      const int rc = rt_context_render_ppm(c, &c->last_cam, &q, c->last_out, c->last_out8, c->last_stream);
      if (rc != RT_OK) return rc;
      return rt_context_timing(c, st);
    }
  }
  float a = 0, b = 0, d = 0;
  if (hipEventElapsedTime(&a, c->ev[0], c->ev[1]) != hipSuccess) return RT_ERR_HIP;
  if (hipEventElapsedTime(&b, c->ev[1], c->ev[3]) != hipSuccess) return RT_ERR_HIP;
  if (hipEventElapsedTime(&d, c->ev[3], c->ev[2]) != hipSuccess) return RT_ERR_HIP;
  if (c->used_traversal == RT_TRAV_ACCEL &&
      hipMemcpy(&st->accel_fallbacks, static_cast<uint32_t *>(c->work.p) + 12, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return RT_ERR_HIP;
  if (c->used_traversal == RT_TRAV_MIXED) {
    uint32_t w[16];
    if (hipMemcpy(w, c->work.p, sizeof w, hipMemcpyDeviceToHost) != hipSuccess) return RT_ERR_HIP;
    st->mix_fallbacks = w[11];
    if (std::getenv("RT_DEBUG"))
      std::fprintf(stderr, "[rt] mixed walk fallbacks: %u (tie %u, reach %u; probe %u)\n", w[11], w[2], w[3], w[10]);
    unsigned long long dg[10];
    if (hipMemcpy(dg, static_cast<uint32_t *>(c->work.p) + 16, sizeof dg, hipMemcpyDeviceToHost) != hipSuccess)
      return RT_ERR_HIP;
    if (dg[0] && std::getenv("RT_DEBUG"))   // RT_JIT_OPTS=-DRT_MIX_DIAG builds only
      std::fprintf(stderr, "[rt] mixed diag: trips %llu ref_lanes %llu macro_lanes %llu both %llu ref_trips %llu "
                   "bvh %llu planar %llu chain %llu kind_groups %llu walk_lanes %llu\n", dg[0], dg[1], dg[2], dg[3],
                   dg[4], dg[5], dg[6], dg[7], dg[8], dg[9]);
  }
  st->init_ms = a;
  st->sched_ms = b;
  st->render_ms = d;
  st->samples = c->samples;
  st->devices = 1;
  {   // device checks (RT_CHECKS=1 builds): the first index a kernel found out of its capacity fails the frame, named
    uint32_t ck[3] = {0, 0, 0};
    if (hipMemcpy(ck, static_cast<uint32_t *>(c->work.p) + rt::kCheckWord, sizeof ck, hipMemcpyDeviceToHost) != hipSuccess)
      return RT_ERR_HIP;
    if (ck[0] != rt::CHK_NONE) {
      static const char *const names[rt::CHK__COUNT] = {"none", "lane DFS stack", "verified sphere walk stack",
                                                        "verified mixed walk stack", "colour-stack LDS level",
                                                        "colour-stack deep level", "deep-level pool chunk", "output pixel",
                                                        "kernel-argument re-read"};
      char b[200];
      std::snprintf(b, sizeof b, "device check failed: %s index %u >= capacity %u (site %u)",
                    ck[0] < rt::CHK__COUNT ? names[ck[0]] : "unknown", ck[1], ck[2], ck[0]);
      c->jit_why = b;
      if (std::getenv("RT_DEBUG")) std::fprintf(stderr, "[rt] %s\n", b);
      return RT_ERR_DEVICE_CHECK;
    }
  }
  {   // the render kernel's own span (RenderArgs::span): first wave start to last wave end
    unsigned long long sp[2] = {0, 0};
    if (hipMemcpy(sp, static_cast<uint32_t *>(c->work.p) + kSpanWord, sizeof sp, hipMemcpyDeviceToHost) != hipSuccess)
      return RT_ERR_HIP;
    const unsigned long long t0 = ~sp[0], t1 = sp[1];
    st->render_kernel_ms = (sp[0] != 0 && t1 >= t0) ? static_cast<double>(t1 - t0) / c->wall_khz : 0.0;
  }
  if (c->rc_audit_bytes) {   // RT_FLAG_RC_AUDIT: slots the render wrote
    std::vector<uint8_t> rb(c->rc_audit_bytes);
    if (hipMemcpy(rb.data(), c->rc.p, rb.size(), hipMemcpyDeviceToHost) != hipSuccess) return RT_ERR_HIP;
    const size_t w = c->rc_audit_code;
    uint64_t n = 0;
    for (size_t i = 0; i < rb.size(); i += w) {
      bool untouched = true;
      for (size_t k = 0; k < w; ++k) untouched = untouched && rb[i + k] == 0xff;
      n += untouched ? 0 : 1;
    }
    st->rc_hbm_slots = n;
  }
  if (c->counted) {
    unsigned long long h[RT_CNT__COUNT];
    if (hipMemcpy(h, c->counters.p, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return RT_ERR_HIP;
    for (int k = 0; k < RT_CNT__COUNT; ++k) st->counters[k] = h[k];
  }
  if (c->wave_trace_words) {   // diagnostics: raw per-wave records, appended per render
    std::vector<unsigned long long> w(c->wave_trace_words);
    if (hipMemcpy(w.data(), c->wave_trace.p, w.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return RT_ERR_HIP;
    if (FILE *f = std::fopen(c->wave_trace_path.c_str(), "ab")) {
      std::fwrite(w.data(), 8, w.size(), f);
      std::fclose(f);
    }
  }
  return RT_OK;
}

int rt_render(const rt_scene *scene, const rt_camera *cam, const rt_params *p, float *out_rgb, rt_stats *stats) {
  auto t0 = std::chrono::steady_clock::now();
  int st = params_check(p);
  if (st != RT_OK) return st;
  if (!scene || !cam || (!out_rgb && p->row_count > 0)) return RT_ERR_INVALID_ARG;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  rt_context *c = nullptr;
  st = rt_context_create(scene, dev, &c);
  if (st != RT_OK) return st;
  const size_t bytes = static_cast<size_t>(p->row_count) * static_cast<size_t>(p->width) * 12;
  DevBuf out;
  {
    DeviceGuard g(dev);
    if (bytes && out.ensure(bytes) != hipSuccess) { rt_context_destroy(c); return RT_ERR_HIP; }
    st = rt_context_render(c, cam, p, static_cast<float *>(out.p), nullptr);
    // rt_context_timing checks the folded traversal's bound flag and re-renders the frame unfolded
    // when a ray exceeded it: it must run before the copy, stats requested or not
    rt_stats local{};
    if (st == RT_OK) st = rt_context_timing(c, stats ? stats : &local);
    if (st == RT_OK && hipDeviceSynchronize() != hipSuccess) st = RT_ERR_HIP;
    if (st == RT_OK && bytes && hipMemcpy(out_rgb, out.p, bytes, hipMemcpyDeviceToHost) != hipSuccess) st = RT_ERR_HIP;
    out.release();
  }
  rt_context_destroy(c);
  if (st == RT_OK && stats)
    stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return st;
}

}  // extern "C"

namespace {
void copy_out(const std::string &s, char *buf, uint64_t cap) {
  if (!buf || cap == 0) return;
  const size_t n = std::min<size_t>(s.size(), static_cast<size_t>(cap - 1));
  std::memcpy(buf, s.data(), n);
  buf[n] = '\0';
}
}  // namespace

int rt_static_source(const rt_scene *scene, uint32_t max_visits, char *buf, uint64_t cap, uint32_t *visits) {
  if (!scene) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  const int rc = rt::compile_scene(scene, &img);
  if (rc != RT_OK) return rc;
  std::string src;
  uint32_t v = 0;
  const int variant = (img.has_noise ? rt::kVarNoise : 0) | (img.needs_uv ? rt::kVarUv : 0) | rt::scene_shading_bits(img);
  const bool ok = rt::jit_source(img, variant, max_visits, true, &src, &v);
  if (visits) *visits = v;
  if (!ok) return RT_ERR_UNSUPPORTED;
  copy_out(src, buf, cap);
  return RT_OK;
}

int rt_static_compile(const rt_scene *scene, uint32_t max_visits, const char *arch, char *log, uint64_t cap) {
  if (!scene || !arch) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  const int rc = rt::compile_scene(scene, &img);
  if (rc != RT_OK) return rc;
  std::string src, lg;
  uint32_t v = 0;
  const int variant = (img.has_noise ? rt::kVarNoise : 0) | (img.needs_uv ? rt::kVarUv : 0) | rt::scene_shading_bits(img);
  if (!rt::jit_source(img, variant, max_visits, true, &src, &v)) return RT_ERR_UNSUPPORTED;
  std::vector<char> code;
  const bool ok = rt::jit_compile(src, arch, &code, &lg);
  copy_out(lg, log, cap);
  return ok ? RT_OK : RT_ERR_HIP;
}

// the run-time source a render of `scene` would build for `traversal` (rt_kernel_source, rt_kernel_build); *img_out (if
// non-null) receives the compiled scene, *accel_w0 (accel traversal) the source at the allocator's register choice
static int kernel_source_impl(const rt_scene *scene, int traversal, int32_t max_bounces, std::string *out,
                              rt::SceneImage *img_out, std::string *accel_w0) {
  if (!scene) return RT_ERR_INVALID_ARG;
  rt::SceneImage img;
  int rc = rt::compile_scene(scene, &img);
  if (rc != RT_OK) return rc;
  while (img.words.size() % 4) img.words.push_back(0);
  const uint32_t mb = static_cast<uint8_t>(max_bounces);
  int variant = (img.words.size() <= rt::kLdsSceneMaxWords ? rt::kVarLds : 0) | (img.has_noise ? rt::kVarNoise : 0) |
                      (img.needs_uv ? rt::kVarUv : 0) | rt::scene_shading_bits(img) |
                      (mb > static_cast<uint32_t>(rt::kDeepBounces) ? rt::kVarDeep : 0) |
                      (!img.has_noise && !img.needs_uv && img.rec_consts + rt::kRcConsts < 65536u ? rt::kVarNarrow : 0) |
                      (!img.has_noise && !img.needs_uv && img.rec_consts + rt::kRcConsts < 255u ? rt::kVarByte : 0) |
                      static_cast<int>(tile_shift_setting() << rt::kVarTileShift) | (stage_slots_setting() ? rt::kVarStage : 0);
  {   // tile-major output as a render with a device frame decides (RT_TILED_OUT, output staging)
    const char *e = std::getenv("RT_TILED_OUT");
    const int t = e ? (e[0] == '1' ? 1 : (e[0] == '0' ? 0 : -1)) : -1;
    if (t != 0 && !stage_slots_setting()) variant |= rt::kVarTiledOut;
  }
  {   // kVarRcLds as a static-traversal render would set it (scene in LDS, no per-lane stacks), else the pool's code
    const uint32_t cb = (variant & rt::kVarByte) ? 1u : ((variant & rt::kVarNarrow) ? 2u : 4u);
    const size_t need = static_cast<size_t>((mb + 3) & ~3u) * rc_level_bytes(cb) +
                        (img.words.size() <= rt::kLdsSceneMaxWords ? img.words.size() * 4 : 4096u) + kRngSlotBytes + kLdsReserve;
    bool pool_set = false;
    const int pool = rc_pool_setting(&pool_set);
    if (traversal == RT_TRAV_STATIC && need <= kLdsPerCu / kRcLdsOnlyBlocks) variant |= rt::kVarRcLds;
    else if (pool > 0 && (mb > static_cast<uint32_t>(rt::kDeepBounces) || pool_set)) variant |= rt::kVarRcPool;
  }
  std::string src;
  if (traversal == RT_TRAV_STATIC) {
    uint32_t v = 0;
    if (!rt::jit_source(img, variant | (img.has_noise ? rt::kVarCoop : 0), 256, true, &src, &v)) return RT_ERR_UNSUPPORTED;
  } else if (traversal == RT_TRAV_ACCEL) {
    rt::SphereAccel a;
    std::string why;
    if (!rt::build_sphere_accel(img, kAccelMinSpheres, &a, &why)) return RT_ERR_UNSUPPORTED;
    const int wide = rt::accel_width() == 4 ? (rt::accel_quant() ? 2 : 1) : 0;
    src = rt::jit_accel_source(img, variant, rt::accel_waves(wide), wide);
    if (accel_w0) *accel_w0 = rt::jit_accel_source(img, variant, 0, wide);
  } else if (traversal == RT_TRAV_MIXED) {
    rt::MixedAccel m;
    std::string why;
    if (!rt::build_mixed_accel(&img, &m, &why)) return RT_ERR_UNSUPPORTED;
    src = rt::jit_mixed_source(img, variant);
  } else if (traversal == RT_TRAV_LANE) {
    src = rt::jit_lane_source(img, variant);
  } else {
    return RT_ERR_INVALID_ARG;
  }
  *out = src;
  if (img_out) *img_out = std::move(img);
  return RT_OK;
}

int rt_kernel_source(const rt_scene *scene, int traversal, int32_t max_bounces, char *buf, uint64_t cap) {
  if (!scene || !buf || cap == 0) return RT_ERR_INVALID_ARG;
  std::string src;
  const int rc = kernel_source_impl(scene, traversal, max_bounces, &src, nullptr, nullptr);
  if (rc != RT_OK) return rc;
  copy_out(src, buf, cap);
  return RT_OK;
}

int rt_kernel_build(const rt_scene *scene, int traversal, int32_t max_bounces, rt_kernel_info *out) {
  if (!scene || !out) return RT_ERR_INVALID_ARG;
  *out = rt_kernel_info{};
  std::string src, w0;
  rt::SceneImage img;
  const int rc = kernel_source_impl(scene, traversal, max_bounces, &src, &img, &w0);
  if (rc != RT_OK) return rc;
  const char *prefix = traversal == RT_TRAV_STATIC ? "rt_static" : traversal == RT_TRAV_ACCEL ? "rt_accel"
                     : traversal == RT_TRAV_MIXED ? "rt_mixed" : "rt_lane";
  const std::vector<std::string> extra = traversal == RT_TRAV_STATIC ? rt::static_sched(img)
                                       : traversal == RT_TRAV_ACCEL ? rt::accel_sched()
                                       : traversal == RT_TRAV_MIXED ? rt::mixed_sched() : std::vector<std::string>{};
  rt::KernelMeta m;
  std::string compiler, why;
  auto fail = [&why]() {
    if (std::getenv("RT_DEBUG")) std::fprintf(stderr, "[rt] rt_kernel_build: %s\n", why.c_str());
    return RT_ERR_UNSUPPORTED;
  };
  if (!rt::jit_build_meta(src, prefix, extra, "gfx950", &m, &compiler, &why)) return fail();
  // the verified walk's 6-wave request is kept only without scratch (rt_jit.cpp jit_accel_kernels): else the
  // allocator's own build
  if (traversal == RT_TRAV_ACCEL && !std::getenv("RT_ACCEL_WAVES") && rt::accel_waves() > 0 &&
      !rt::accel_waves_build_kept(m.scratch) &&
      !rt::jit_build_meta(w0, prefix, extra, "gfx950", &m, &compiler, &why))
    return fail();
  fill_kernel_info(m, compiler, out);
  return RT_OK;
}

int rt_tonemap_device(const float *rgb, uint64_t pixels, uint8_t *out, void *stream) {
  if ((!rgb || !out) && pixels) return RT_ERR_INVALID_ARG;
  if (rt::launch_tonemap(rgb, pixels * 3, out, static_cast<hipStream_t>(stream)) != hipSuccess) return RT_ERR_HIP;
  return RT_OK;
}

int rt_seed_states(uint64_t seed, int width, int row_offset, int row_stride, int rows, uint32_t *out) {
  if (!out || width <= 0 || rows <= 0 || row_offset < 0 || row_stride <= 0) return RT_ERR_INVALID_ARG;
  const uint64_t n = static_cast<uint64_t>(rows) * static_cast<uint64_t>(width);
  if (n > 0x7fffffffull) return RT_ERR_INVALID_ARG;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RT_ERR_NO_DEVICE;
  const uint32_t tiles_x = (static_cast<uint32_t>(width) + 7) / 8;
  const uint64_t n_ids = 64ull * ((static_cast<uint64_t>(rows) + 7) / 8) * tiles_x;
  if (n_ids > 0xffffffffull) return RT_ERR_INVALID_ARG;
  const std::vector<uint32_t> &J = rt::xorwow_jump_tables();
  DevBuf jump, states;
  std::vector<uint32_t> tiled;
  int rc = RT_OK;
  if (jump.ensure(J.size() * 4) != hipSuccess || states.ensure(n_ids * 6 * 4) != hipSuccess ||
      hipMemcpy(jump.p, J.data(), J.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    rc = RT_ERR_HIP;
  } else {
    rt::SeedArgs sa{};
    sa.jump = static_cast<const uint32_t *>(jump.p);
    rt::xorwow_seed_base(seed, sa.base);
    sa.width = width; sa.row_offset = row_offset; sa.row_stride = row_stride;
    sa.rows = static_cast<uint32_t>(rows);
    sa.tiles_x = tiles_x;
    sa.n_ids = static_cast<uint32_t>(n_ids);
    sa.rng = static_cast<uint32_t *>(states.p);
    tiled.resize(n_ids * 6);
    if (rt::launch_seed(sa, nullptr) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(tiled.data(), states.p, n_ids * 6 * 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = RT_ERR_HIP;
  }
  jump.release();
  states.release();
  if (rc != RT_OK) return rc;
  // tile-major (the kernels' layout) -> [6][rows * width] in pixel order (this function's contract)
  for (uint64_t lr = 0; lr < static_cast<uint64_t>(rows); ++lr)
    for (uint64_t j = 0; j < static_cast<uint64_t>(width); ++j) {
      const uint64_t id = ((lr >> 3) * tiles_x + (j >> 3)) * 64 + (lr & 7) * 8 + (j & 7);
      for (int w = 0; w < 6; ++w) out[w * n + lr * width + j] = tiled[w * n_ids + id];
    }
  return RT_OK;
}

int rt_rng_table_states(uint64_t seed, int width, int row_offset, int row_stride, int rows, uint32_t *out) {
  if (!out || width <= 0 || rows <= 0 || row_offset < 0 || row_stride <= 0) return RT_ERR_INVALID_ARG;
  std::vector<uint32_t> pb, ct;
  const int ph = static_cast<int>(tile_shift_setting());   // the phase width of a new context's renders (the tile width)
  const int pw = 1 << ph;
  rt::xorwow_phase_bases(seed, width, row_offset, row_stride, rows, &pb, ph);
  rt::xorwow_column_tables(width, &ct, ph);
  uint32_t base[6];
  rt::xorwow_seed_base(seed, base);
  for (int lr = 0; lr < rows; ++lr)
    for (int j = 0; j < width; ++j) {   // the render kernel's pickup: phase base (lr, j & (pw-1)), table j >> ph
      uint32_t x[5];
      std::memcpy(x, &pb[(static_cast<size_t>(lr) * pw + (j & (pw - 1))) * 8], sizeof x);
      const int t = j >> ph;
      rt::xorwow_apply_nib(ct.data() + static_cast<size_t>(t & (rt::kColLo - 1)) * rt::kJumpNibbleWords, x);
      rt::xorwow_apply_nib(ct.data() + static_cast<size_t>(rt::kColLo + (t >> rt::kColLoBits)) * rt::kJumpNibbleWords, x);
      uint32_t *o = out + (static_cast<size_t>(lr) * width + j) * 6;
      o[0] = base[0];
      std::memcpy(o + 1, x, sizeof x);
    }
  return RT_OK;
}

const char *rt_context_note(const rt_context *c) { return c ? c->jit_why.c_str() : ""; }
