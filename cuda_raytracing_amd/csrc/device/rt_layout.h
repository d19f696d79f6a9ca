// rt_layout.h — device-visible layout of the compiled scene and the kernel argument blocks.
//
// Shared by the host (scene_compile.cpp, rt_capi.cpp), the offline HIP kernels (rt_device.hip) and the
// scene-specialised kernels compiled at run time with hipRTC (rt_jit.cpp), so it may only include
// <stdint.h> (the one C header hipRTC provides).
#pragma once
#include <stdint.h>

namespace rt {

// node kinds == reference VisObject values (raytracing.cu:144-153)
enum : uint32_t {
  K_SPHERE = 0, K_BVH = 1, K_TRIANGLE = 2, K_QUAD = 3, K_TRANSLATE = 4, K_YROTATE = 5, K_GROUP = 6
};

// Every scene record becomes one 80-byte node (record indices preserved, WorldRefs resolved).
// Word layout per kind (w0 = kind, w1 = aux):
//   BVH      : w1 = left_href | right_href << 16, w2..w7 = x0 x1 y0 y1 z0 z1
//   SPHERE   : w1 = material, w2..4 centre, w5..7 motion, w8 radius, w9 radius*radius, w10 1/radius,
//              w11 = 1 if the material's texture reads u,v (an image texture: the walk computes them)
//   TRI/QUAD : w1 = material, w2..4 normal, w5 d, w6..8 q, w9..11 u, w12..14 v, w15..17 w
//   TRANSLATE: w1 = child, w2..4 offset
//   YROTATE  : w1 = child, w2 sin, w3 cos
//   GROUP    : w1 = first child, w2 = count
constexpr int kNodeWords = 20;
enum : int {
  W_KIND = 0, W_AUX = 1,
  W_BOX = 2,
  W_CENTER = 2, W_MOTION = 5, W_RADIUS = 8, W_RADIUS2 = 9, W_INV_RADIUS = 10, W_SPHERE_UV = 11,
  W_NORMAL = 2, W_D = 5, W_Q = 6, W_U = 9, W_V = 12, W_W = 15,
  W_OFFSET = 2, W_SIN = 2, W_COS = 3, W_COUNT = 2,
};

// Verified sphere traversal (sphere_accel.cpp, AccelTraceK): a binned-SAH BVH2 over the spheres of
// an all-sphere world.  Node = 16 words: child boxes (x0 x1 y0 y1 z0 z1) at 0 and 6, child refs at
// 12/13 (kAccelLeaf | (count-1) << 24 | first prim, or a node index), per child at 14/15 an upper
// bound M of |centre(t)| + radius over its spheres.  Prim = 16 words, in leaf order.
constexpr int kAccelNodeWords = 16, kAccelPrimWords = 16;
// 4-wide form of the same tree (accel::collapse_wide): a node = the 4 subtrees reached by opening the BVH2
// child with the largest box twice; 32 words, structure-of-arrays so one 16-B load brings a plane of all four
// children: x0[4] x1[4] y0[4] y1[4] z0[4] z1[4] at words 0..23 (the BVH2 child boxes, padding included), child
// refs at 24..27 (kAccelLeaf leaf ref as in the BVH2, else a 4-wide node index), words 28..31 unused.  An empty
// slot has the box (+inf, -inf) on every axis (never hit) and ref 0.
constexpr int kAccel4NodeWords = 32, kAccel4Ref = 24;
// Quantised form of the 4-wide tree (accel::quantize_wide; RT_ACCEL_QUANT): 16 words, one 64-B line per node.
// Words 0..2 = the node's origin o_a (float), word 3 = the per-axis scale exponents e_a + 127 in bytes 0..2 and
// the valid-child mask in bits 24..27; words 4..9 = the planes as bytes (byte c = child c): x_lo x_hi y_lo y_hi
// z_lo z_hi, plane = o_a + q * 2^e_a; words 10..13 = the child refs (as kAccel4Ref); words 14..15 unused.  Each
// decoded box contains the float child box, itself widened by 2^-20 of the node's largest magnitude on that axis
// (the rounding of the fma(q, 2^e / d, fma(o, 1/d, -o_ray / d)) evaluation), so the culling stays conservative.
constexpr int kAccel4QNodeWords = 16, kAccel4QRef = 10;
// Primary-ray candidate list entry (prim_list_kernel): the sphere inline, so a camera ray's list loop loads one
// entry per sphere: words 0..3 = centre at time 0 and r^2, 4 = SAH prim index, 5 = axial lower bound (float bits),
// 6..7 = motion x, y, 8 = motion z (entries of 12 words when some sphere moves, else 8 and no motion)
enum : int { kPrimEntryIdx = 0, kPrimEntryBound = 1, kPrimEntryWords = 2 };   // sphere index, axial bound
constexpr uint32_t kAccelLeaf = 0x80000000u;
constexpr float kAccelKappa = 1.953125e-3f;   // 2^-9 >= sqrt(32 * 2^-24): cone padding per unit of |oc|
enum : int { AP_CENTER = 0, AP_MOTION = 3, AP_RADIUS2 = 6, AP_INV_RADIUS = 7, AP_MAT = 8, AP_NODE = 9, AP_VBOX = 10 };

// Verified traversal of mixed worlds (mixed_accel.cpp, MixedTraceK): some reference BVH/group nodes are
// macro roots, whose transform-free primitives (quads, triangles, spheres) also sit in a SAH tree of their
// own (node layout as above).  Node words W_MACRO (the SAH root | kMacro* flags, 0 = plain node) and
// W_XFBOX..+5 (dynamic macros: the union of the boxes of the BVH nodes below with a translate / rotate
// child) are unused by the record kinds (a BVH node ends at word 7, a group at word 2).  Static macro:
// the subtree holds no transform.  Dynamic macro: the ray may take the SAH walk only when the reference's
// own slab test on W_XFBOX fails (then it enters no transform below).
constexpr int W_MACRO = 12, W_XFBOX = 13;
constexpr uint32_t kMacroStatic = 0x80000000u, kMacroDynamic = 0x40000000u, kMacroRootMask = 0x00ffffffu;
// Mixed prims (leaf order): words 0..19 = the primitive's node record (kind, material, geometry), MP_GROUP =
// its deepest reference BVH ancestor below the macro root (~0u: none), MP_GBOX..+5 = that ancestor's box
// Transform chains (translate -> [y-rotate ->] primitive, or y-rotate -> primitive): W_MACRO of the head
// record = kChainFused [| kChainRotate: the translate's child is a y-rotation] | the primitive's record.
// MixedTraceK runs the reference's five stack steps of such a chain (:1176-1237) as one.
// kChainPacked: the chain ends in a sphere whose record words sit in the head's unused words, so the fused
// step needs no further load: sphere words 1..3 (material, centre x, y) at head words 5..7, sphere words
// 4..7 (centre z, motion) at 16..19, sphere words 8..11 (radius, radius^2, 1/radius) at 8..11, the
// y-rotation's sin / cos at 13 / 14.
constexpr uint32_t kChainFused = 0x20000000u, kChainRotate = 0x10000000u, kChainPacked = 0x08000000u,
                   kChainPrimMask = 0x0000ffffu;
enum : int { W_PK_SPHERE0 = 5, W_PK_SPHERE8 = 8, W_PK_SIN = 13, W_PK_COS = 14, W_PK_SPHERE4 = 16 };
constexpr int kMixPrimWords = 32;
enum : int { MP_GROUP = 20, MP_GBOX = 21, MP_RECORD = 27 };
constexpr uint32_t kMixNoGroup = 0xffffffffu;

// materials (raytracing.cu:78-99): 8 words; kinds == RTR_MAT_* (rt_ref_layout.h).  A metal's albedo
// sits at words 1..3 like a solid texture's colour (M_TEX is only used by Lambertian / light kinds), so
// both are "colour records" the compact colour stack can point at (see kRecWords below).
constexpr int kMatWords = 8;
enum : int { M_KIND = 0, M_TEX = 1, M_ALBEDO = 1, M_FUZZ = 5, M_IOR = 6 };
enum : uint32_t { MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_DIFFUSE_LIGHT = 3 };

// textures (raytracing.cu:38-54): 8 words
constexpr int kTexWords = 8;

// Colour records: materials, then textures, then kRcConsts constant records, contiguous from
// off_mats, 8 words each, an attenuation colour (when the record has one) at words 1..3.  Record r
// starts at word off_mats + 8 r.  Constants: the magenta and black of image_texture_get_pixel /
// texture_get_color (raytracing.cu:346-347, 397) and a NaN grey (a noise value that is not finite).
constexpr int kRecWords = 8;
enum : uint32_t { RC_MAGENTA = 0, RC_BLACK = 1, RC_NAN = 2, kRcConsts = 3 };
// Colour-stack codes (ray_color's attenuation stack, :1253-1276).  Every attenuation the reference
// pushes is a record's colour, a texel, or a noise grey (r = g = b, 0.5 (1 + sin) >= +0, never negative);
// a level stores a code for it:
//   wide (32 bit):  grey float bits (finite, sign bit clear) | kRcRecTag + record (23 bits) |
//                   kRcTexelTag + texel word offset (31 bits: the whole 2^31-word pixel pool)
//   narrow (16 bit, scenes without noise and texels and < 65536 records): the record index
constexpr uint32_t kRcRecTag = 0x7F800000u, kRcPayload = 0x007FFFFFu;
constexpr uint32_t kRcTexelTag = 0x80000000u, kRcTexelPayload = 0x7FFFFFFFu;
static_assert(kMatWords == kRecWords && kTexWords == kRecWords, "colour records are 8 words");
enum : uint32_t { T_SOLID = 0, T_CHECKER = 1, T_IMAGE = 2, T_NOISE = 3 };
enum : int {
  T_KIND = 0,
  T_RGB = 1,                                         // solid: w1..3
  T_EVEN = 1, T_ODD = 2, T_INV_SCALE = 3,            // checker
  T_PERLIN = 1, T_NOISE_SCALE = 3,                   // noise: perlin table index, scale
  T_WIDTH = 1, T_HEIGHT = 2, T_PIXELS = 3, T_HAS_PIXELS = 4,   // image: pixel word offset into pool
};

// Perlin table: 256 gradients as float4 (xyz, pad) + 256 perm_x bytes (perm_y/z are never read,
// perlin_noise.cpp:37-39) + 256 u16 pairs perm_x[i] | perm_x[(i + 1) & 255] << 8 (one load per axis)
constexpr int kPerlinWords = 256 * 4 + 64 + 128;
constexpr int kPerlinPermWord = 256 * 4, kPerlinPerm2Word = 256 * 4 + 64;

// counter slots == RT_CNT_* (rt_render.h)
enum : int {
  CNT_VISIT0 = 0, CNT_BOUNCES = 7, CNT_SHADES = 8, CNT_PERLIN = 9, CNT_RNG = 10, CNT_SAMPLES = 11,
  CNT_MAX_STACK = 12, CNT_OVERFLOW = 13, CNT_EXEC_NODE = 14, CNT_EXEC_PRIM = 15, CNT_SLOTS = 16
};

constexpr int kBlock = 256;        // 4 waves of 64
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int kChunk = 64;         // pixel ids handed to a wave per work-queue grab (one 8x8 tile)

// render-kernel variants: scene staged in LDS, counters, Perlin noise textures, sphere u,v (image
// textures with pixels), wave-packet traversal.  Specialising keeps unused texture code out of the
// register allocation (the Perlin + double-sine path alone costs ~40 VGPRs).
enum : int { kVarLds = 1, kVarCount = 2, kVarNoise = 4, kVarUv = 8, kVarPacket = 16,
             kVarTrace = 32 /* wave timeline diagnostics; scene-specialised kernels only */ };
// run-time compiled kernels also carry the material kinds (bits 6..9, bit MAT_*) and texture kinds
// (bits 10..13, bit T_*) present in the scene; 0 in a field means "all" (the offline kernels)
constexpr int kVarMatShift = 6, kVarTexShift = 10;
// run-time compiled kernels for deep paths (max_bounces > kDeepBounces): colour-stack levels in HBM are
// unwound with batched loads (costs registers, so shallow renders keep the plain loop)
constexpr int kVarDeep = 1 << 14;
constexpr int kDeepBounces = 16;
// run-time compiled kernels whose colour-stack codes fit 16 bits (no noise, no texels, < 65536 colour
// records): two levels per LDS word.  The offline kernels always use 32-bit codes.
constexpr int kVarNarrow = 1 << 15;
// run-time compiled scene-specialised kernels of noise scenes: cooperative noise octaves (render_body);
// the large-scene walks leave it out (its registers cost them a wave; noise is not their bottleneck)
constexpr int kVarCoop = 1 << 16;
// run-time compiled kernels: the schedule probe's kernel (kVarProbe) and the render kernels that are never
// launched as the probe (kVarNoProbe) resolve RenderArgs::probe_cost at compile time (offline: at run time)
constexpr int kVarProbe = 1 << 17, kVarNoProbe = 1 << 18;
// run-time compiled narrow kernels whose colour records number < 255: 8-bit codes, four levels per LDS word (a
// d50 Cornell box keeps all 50 levels of every lane in LDS: no colour-stack traffic to HBM)
constexpr int kVarByte = 1 << 19;
// run-time compiled kernels whose colour stack lives in LDS entirely (rc_lds_levels >= max_bounces at any
// residency, rt_capi.cpp): no HBM level code (the deep unwind's batch registers) in the kernel
constexpr int kVarRcLds = 1 << 20;
// run-time compiled kernels with the output staging code (RenderArgs::stage_*; used when the launch gets slots), and
// the tile shape as a constant (bits 22..24 = RenderArgs::tile_shift; 0: read from RenderArgs, the offline kernels)
constexpr int kVarStage = 1 << 21;
constexpr int kVarTileShift = 22;
// run-time compiled kernels with HBM colour-stack levels and the per-wave deep-level pool (RenderArgs::rc_pool_*)
constexpr int kVarRcPool = 1 << 25;
// run-time compiled kernels with the tail-piece hand-out (RenderArgs::tail_*; RT_TAIL_CHUNK)
constexpr int kVarTail = 1 << 26;
// run-time compiled kernels that write the float frame tile-major (RenderArgs::out: tile t's 64 pixels x 3 floats at
// 192 t, pixel k of the tile at 3 k), so that every 128-B line of it is written by one wave through one XCD's L2; the
// row-major frame and the PPM bytes come from untile_kernel after the render (RT_TILED_OUT)
constexpr int kVarTiledOut = 1 << 27;
// variant bits the run-time compiled kernels are specialised on
constexpr int kJitVarMask = kVarLds | kVarNoise | kVarUv | kVarTrace | kVarDeep | kVarNarrow | kVarCoop | kVarByte | kVarRcLds |
                            kVarStage | (7 << kVarTileShift) | kVarRcPool | kVarTail | kVarTiledOut | (15 << kVarMatShift) | (15 << kVarTexShift);

// per wave: start, end (s_memrealtime), tiles, hw ids, rounds, busy lane-rounds, s_memtime cycles in
// refill / traversal / unwind+accumulate+next camera ray / material scatter / rejection sampling
constexpr uint32_t kWaveTraceWords = 23;   // rt_body.h: timeline, phases, tail-round phases, noise share

// Resident 256-thread blocks per CU allowed by the VGPR budget: 512 VGPRs per lane per SIMD, one
// wave of each block per SIMD.  The persistent grid must never exceed residency (a block that starts
// late only lengthens the tail).  Measured on gfx950 with per-wave start stamps (tools/wave_trace.py):
// kernels of 70 and 75 VGPRs ran 6 resident blocks/CU although the occupancy API reported 7, and
// 80-86 VGPRs ran 5: consistent with an allocation granule of 16 for wave64, which is used here.
inline int resident_blocks_by_vgprs(int vgprs, int granule = 16) {
  const int g = granule == 8 ? 8 : 16;
  const int alloc = ((vgprs > 0 ? vgprs : 1) + g - 1) / g * g;
  const int w = 512 / alloc;
  return w < 1 ? 1 : (w > 8 ? 8 : w);
}

struct RenderArgs {
  const uint32_t *scene;      // compiled scene word image in HBM
  uint32_t scene_words;
  uint32_t off_mats, off_texs, off_perlin, off_pixels, pixel_words;
  uint32_t root, stack_cap, stack_lds_word;   // per-lane stack region starts at this LDS word
  uint32_t rc_lds_word, rc_lds_levels;        // colour-stack levels [0, rc_lds_levels) live in LDS
  // Deep-level pool (kVarRcPool kernels): per wave, from LDS word rc_pool_word + wave * (kRcPoolHead + rc_pool_chunks *
  // (max_bounces - rc_lds_levels)), a free-chunk mask word, the lanes' chunk bytes (16 words), then rc_pool_chunks chunks
  // of max_bounces - rc_lds_levels words.  A path's levels past the LDS ones go to a chunk when one is free at its first
  // such push, else to HBM (rc)
  uint32_t rc_pool_word, rc_pool_chunks;
  uint32_t rc_tex0, rc_consts;                // colour records: first texture, first constant
  // camera (rt_camera)
  float p00[3], du[3], dv[3], center[3], dfu[3], dfv[3], defocus_angle;
  int32_t width, row_offset, row_stride;
  int32_t spp, max_bounces;
  float bg[3];
  float sample_scale;
  uint32_t n_pixels;          // row_count * width (local pixels of this shard)
  uint32_t rows;              // row_count
  uint32_t tiles_x;           // ceil(width / tile width)
  uint32_t n_ids;             // 64 * ceil(rows / tile height) * tiles_x: tile-major pixel ids handed to waves
  // Tiles of 64 pixels, tw = 1 << tile_shift wide and 64 / tw tall (3: 8x8, 5: 32x2).  A 32-pixel tile row of the
  // float frame is 384 B = three whole 128-B lines (W % 32 == 0), so every frame line is written by one wave
  uint32_t tile_shift;
  // Output staging (coalesced tile writes): a finished pixel's floats wait in its wave's LDS slot for the tile and the
  // wave stores the whole tile at once (whole lines, the PPM bytes next to them) when its last pixel ends.
  // stage_slots tiles per wave (0: every pixel written when it ends), kStageSlotWords each, then the wave's word of
  // "slot complete" bits and a pad word (per wave stage_slots * kStageSlotWords + 2), from LDS word stage_word
  uint32_t stage_word, stage_slots;
  // XCD classes (non-null: tile_order is grouped by class, cls_off[q] = class q's first position, cls_off[8] = tiles):
  // a wave takes its XCD's class first (work[kClsWord + q]: class q's counter), then steals from the others
  const uint32_t *cls_off;
  // RNG seeding fused into the tile pickup (init_gpu_data's curand_init, raytracing.cu:1591-1606): when a wave
  // takes a chunk of pixel ids, lane l applies the column table of its pixel's tile column (rng_nib) to the phase
  // base of its pixel (rng_rows) and leaves the state in the wave's slot; the lanes that take those pixels read
  // their states from there (xorwow_jump.h xorwow_phase_bases / xorwow_column_tables)
  const uint32_t *rng_rows;   // [rows][tw columns][8] phase bases {x0..x4, pad}: pixel (lr, c), c < tw (the tile width)
  const uint32_t *rng_nib;    // [kRngColLo + ceil(tiles_x / kRngColLo)][kRngNibTableWords]: J^(tw b), J^(16 tw a)
  uint32_t rng_d;             // the Weyl word d (the same for every subsequence)
  uint32_t rng_slot_word;     // LDS word of the block's per-wave slots, [wave][5][64]: the states of the chunk of pixel
                              // ids the wave took last (kRngSlotWords per wave)
  float *out;                 // [n_pixels][3]
  uint8_t *out8;              // optional [n_pixels][3] P6 payload bytes (pixels_to_ppm), null = none
  void *rc;                   // colour-stack levels past the LDS ones: [threads][max_bounces] codes
                              // (u32, or u16 in narrow kernels)
  uint32_t threads;           // grid size in threads (rc stride)
  uint32_t *work;             // chunk counter (zeroed per launch)
  unsigned long long *counters;   // CNT_SLOTS (counting variants only)
  unsigned long long *wave_trace; // diagnostics (null = off): kWaveTraceWords per wave
  // Schedule.  A lane owns a pixel for all its samples (one XORWOW stream per pixel), so the frame
  // ends when the slowest pixels end: tiles are handed out longest-first (LPT) using a cheap probe.
  const uint32_t *tile_order;     // non-null: the t-th tile handed out is tile_order[t]
  uint32_t probe_per_tile;        // probe paths per 8x8 tile (1..64)
  uint32_t *probe_cost;           // non-null: PROBE launch — probe_per_tile 1-spp paths per tile with
                                  // a hashed RNG; adds each path's round count to probe_cost[tile]
  uint32_t reverse_tiles;         // no order array: 1 = hand tiles out bottom row first
  uint32_t *fold_violation;       // folded traversal: set to 1 if a ray exceeded the host's bound
  uint32_t max_tries;             // rejection tries per round before deferring (0 = unlimited)
  uint32_t accel_nodes, accel_prims, accel_root;   // verified sphere traversal (word offsets, root node)
  uint32_t accel_wide;            // word offset of the 4-wide nodes (kAccel4NodeWords each, root = node 0)
  uint32_t accel_node_u4;         // uint4 per node of the walked tree (4: BVH2 or quantised 4-wide, 8: 4-wide)
  uint32_t accel_lds_nodes;       // its first nodes (breadth-first: the top levels) staged at LDS word 0
  uint32_t *accel_fallbacks;      // rays the verified traversal handed to the reference walk (diagnostic)
  // Primary-ray candidate lists (verified sphere walk; prim_list_kernel): per 8x8 tile of the shard, the spheres
  // whose padded ball meets the cone that holds every camera ray of the tile, ascending by a lower bound of
  // their distance along the cone axis; a camera ray tests them in that order instead of walking the tree
  const uint32_t *prim_lists;     // [tiles][prim_cap] entries of prim_words words (kPrimEntry*: SAH prim index and
                                  // axial bound; the sphere's words are read from the tree's prims); null = off
  const uint32_t *prim_counts;    // [tiles] entries; > prim_cap: no list (overflow), the ray walks the tree
  uint32_t prim_cap;
  uint32_t prim_words;            // kPrimEntryWords
  float prim_rho;                 // bound on |ray origin - camera centre| (defocus disc, rounding included)
  uint32_t defer_trace;           // verified traversal: the round's walk stops once at most this many
  uint32_t trace_min_iters;       // lanes (and <= 1/4 of the starters) still walk, after this many steps
  uint32_t prio_ids;              // pixels among the first prio_ids handed out (the costliest tiles of
                                  // the longest-first order) run their wave at raised issue priority
  uint32_t prio_chunk;            // < 64: those ids are handed out in pieces of this many (work[1])
  uint32_t prio_lanes;            // < 64: a wave holds at most this many of them and nothing else meanwhile
  uint32_t prio_mix;              // with prio_lanes < 64: the wave's other lanes take ordinary tiles meanwhile
  uint32_t defer_lanes;           // the round's rejection stops once at most this many lanes of the
                                  // wave still need a try (they resume next round; 0 = never early)
  uint32_t black_skip;            // every attenuation is finite (host-checked): a path ending in
                                  // (0,0,0) unwinds to +0 without reading its colour stack
  uint32_t coop_noise;            // noise kernels: spread perlin_turbulence's octaves over the wave's lanes
                                  // when at most this many (<= 32) lanes need one (0 = never)
  uint32_t mix_nodes, mix_prims;  // verified mixed-world traversal: word offsets of its SAH nodes / prims
  uint32_t *mix_fallbacks;        // macro walks it handed back to the reference walk (diagnostic)
  uint32_t mix_no_proof;          // test aid (RT_MIX_PROVE=0): every macro walk takes the fallback
  uint32_t tail_prio;             // queue drained: a wave's issue priority grows with the samples its least
                                  // advanced pixel has left (the frame ends with its longest chain)
  uint32_t tail_ids, tail_chunk;  // the last tail_ids ids of the order (a multiple of 64; 0 = none) are handed out in
                                  // pieces of tail_chunk (a power of two < 64) from work[kTailWord]
  // kernel-only timing (non-null on the render launch): span[0] = max over waves of ~start, span[1] = max of
  // end, s_memrealtime ticks (the device's wall clock) — the launch's first wave start to its last wave end,
  // like a profiler's kernel duration and unlike stream events, never widened by neighbouring work
  unsigned long long *span;
};

// nibble table of a 160x160 GF(2) jump matrix (xorwow_jump.h): for input nibble c (bits 4c..4c+3 of the state)
// and value v, the XOR of the rows of v's bits: words 0..3 as uint4 [c * 16 + v], then word 4 as u32 [c * 16 + v]
constexpr uint32_t kRngNibTableWords = 40 * 16 * 5;
// column tables in two levels (xorwow_jump.h xorwow_column_tables): J^(tw b) at table b < kRngColLo, J^(kRngColLo tw a)
// at table kRngColLo + a, for tile column t = kRngColLo a + b
constexpr uint32_t kRngColLoBits = 4, kRngColLo = 1u << kRngColLoBits;
constexpr uint32_t kRngSlotWords = 5 * 64;   // per wave
// output staging slot (RenderArgs::stage_*): 64 pixels x 3 floats in tile order (pixel k at 3 k), then a header:
// the finished-pixel mask (u64), the tile (kStageFree: unused slot), the valid-pixel mask (u64) — 8-B aligned
constexpr uint32_t kStageSlotWords = 192 + 6;
enum : uint32_t { kStageDone = 192, kStageTile = 194, kStageValid = 196 };
constexpr uint32_t kStageFree = 0xffffffffu;
constexpr uint32_t kStageSlotsMax = 4;
constexpr uint32_t kXcdClasses = 8, kClsWord = 36;   // (work words 16..35: the mixed walk's RT_MIX_DIAG counters)
constexpr uint32_t kTailWord = 44;                   // work word of the tail pieces' counter
// Device checks (kernels built with RT_DEVICE_CHECKS: RT_CHECKS=1, rt_capi.cpp): the first index found out of its
// capacity leaves {site, index, capacity} in work words kCheckWord..+2 and its access is skipped; the host then fails
// the frame with RT_ERR_DEVICE_CHECK naming the site (rt_context_note).  (work words 48..51: the kernel span)
constexpr uint32_t kCheckWord = 52;
enum CheckSite : uint32_t {
  CHK_NONE = 0,
  CHK_LANE_STACK = 1,      // per-lane DFS stack pointer vs the lane's stack capacity (the walk's share of it)
  CHK_ACCEL_STACK = 2,     // verified sphere walk's stack vs stack_cap - kSumEntries (the parked pixel sum above it)
  CHK_MIXED_STACK = 3,     // verified mixed walk's reference stack + macro SAH stack vs stack_cap
  CHK_RC_LDS = 4,          // colour-stack level stored in LDS vs rc_lds_levels
  CHK_RC_DEEP = 5,         // colour-stack level past the LDS ones vs max_bounces
  CHK_POOL_CHUNK = 6,      // a lane's deep-level pool chunk vs rc_pool_chunks
  CHK_PIXEL = 7,           // output pixel / tile index vs the frame
  CHK_KARGS = 8,           // the kernarg segment's RenderArgs (kargs(), rt_body.h) differs from the kernel's argument
  CHK__COUNT = 9
};

constexpr uint32_t kProbePerTile = 8;   // default probe paths per 8x8 tile
constexpr uint32_t kRcLdsLevels = 4;    // colour-stack levels kept in LDS (deeper ones spill to HBM)
constexpr uint32_t kSumEntries = 6;        // u16 stack entries holding a lane's pixel sum (kParkSum traces)
constexpr uint32_t kRcPoolChunksMax = 32;   // deep-level pool chunks per wave (one mask word)
constexpr uint32_t kRcPoolHead = 17;         // per wave: the free-chunk mask word, then each lane's chunk byte (16 words)

struct SeedArgs {
  const uint32_t *jump;       // xorwow_jump_tables() on device
  uint32_t base[6];           // rocRAND constant seeding of `seed`
  int32_t width, row_offset, row_stride;
  uint32_t rows;              // local rows of the shard
  uint32_t tiles_x;           // ceil(width / 8)
  uint32_t n_ids;             // 64 * ceil(rows / 8) * tiles_x (stride between the six state words)
  uint32_t *rng;              // [6][n_ids], tile-major (RenderArgs::rng)
};
constexpr uint32_t kSeedRun = 16;   // consecutive pixels of a row seeded per thread (one jump, then steps)

}  // namespace rt
