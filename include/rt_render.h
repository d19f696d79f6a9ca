/*
 * rt_render.h — C-ABI of the MI355X per-pixel render path (the drop-in boundary).
 *
 * Replaces, in luk-zm/cuda_raytracing:
 *   - the device half of `void render(World*, RenderSettings*)` (src/raytracing.cu:1694-1771):
 *     buffer allocation + H2D copies (1694-1744), `init_gpu_data` RNG seeding (1591-1606,1746),
 *     the `cuda_calc` launch (1543-1589,1754) and the D2H framebuffer copy (1770-1771);
 *   - the kernel argument list of `cuda_calc` (1543-1547), which becomes rt_camera + rt_params.
 *
 * The host keeps scene building, BVH construction, camera setup and PPM output (rt_host.h) and
 * hands the reference's own scene buffers (layout: rt_ref_layout.h) across this boundary.
 *
 * Conventions (unlike the reference, which prints errors and returns void):
 *   - every entry point returns RT_OK (0) or a negative RT_ERR_* code and never exits;
 *   - all buffers are caller-owned; nothing is retained after return except inside an rt_context;
 *   - thread-compatible: one call per context (or per device for rt_render) at a time.
 * The CPU oracle (oracle/) exports the same signature as `rt_render_cpu` for parity tests.
 */
#ifndef RT_RENDER_H
#define RT_RENDER_H

#include <stdint.h>
#include "rt_ref_layout.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6

/* status codes */
#define RT_OK                 0
#define RT_ERR_INVALID_ARG   -1   /* null pointer, bad size, bad shard geometry */
#define RT_ERR_SCENE         -2   /* malformed scene bytes (bad record kind, ref or texture offset) */
#define RT_ERR_HIP           -3   /* HIP runtime failure (allocation, launch, copy) */
#define RT_ERR_NO_DEVICE     -4   /* no HIP device visible */
#define RT_ERR_STACK         -5   /* scene needs a deeper traversal stack than the kernel supports */
#define RT_ERR_UNSUPPORTED   -6   /* feature outside this build */
#define RT_ERR_DEVICE_CHECK  -7   /* a kernel built with device checks (RT_CHECKS=1) found an index out of its capacity;
                                     rt_context_note names the site, the index and the capacity (rt_context_timing) */

/* Scene bytes exactly as the reference builds them (raytracing.cu:1699-1733). */
typedef struct rt_scene {
  const rtr_hittable *hittables;   /* HittableList.objects[count]          (raytracing.cu:155-160) */
  uint32_t hittable_count;
  const uint16_t *refs;            /* HittableRefList.data: WorldRef -> record index (raytracing.cu:1-7) */
  uint32_t ref_count;
  uint16_t root;                   /* WorldRef of the root BVH node (SceneData.root_bvh_node, :234) */
  uint16_t pad_;
  const uint8_t *textures;         /* TextureList arena bytes [0, texture_bytes) (raytracing.cu:56-59) */
  uint64_t texture_bytes;
} rt_scene;

/* Camera values `render()` computes on the host and passes to cuda_calc (raytracing.cu:1657-1692). */
typedef struct rt_camera {
  rtr_vec3 pixel00;        /* current_pixel_center: centre of pixel (0,0) (:1690-1692) */
  rtr_vec3 delta_u;        /* pixel_delta_u (:1679) */
  rtr_vec3 delta_v;        /* pixel_delta_v (:1678) */
  rtr_vec3 center;         /* camera_pos = lookfrom (:1669) */
  rtr_vec3 defocus_u;      /* defocus_disk_u (:1687) */
  rtr_vec3 defocus_v;      /* defocus_disk_v (:1688) */
  float defocus_angle;     /* settings.defocus_angle: > 0 enables the lens sample (:1571) */
} rt_camera;

/* Render parameters.  Rows rendered: row_offset + k*row_stride for k in [0, row_count).
 * A full frame is {0, 1, height}; GPU g of G renders {g, G, ceil((height-g)/G)} (row-interleaved
 * shards).  The RNG subsequence of pixel (i,j) is always the GLOBAL index i*width+j (:1604), so
 * the image is bit-identical for any shard geometry. */
typedef struct rt_params {
  int32_t width, height;
  int32_t row_offset, row_stride, row_count;
  int32_t samples_per_pixel;       /* settings.samples_per_pixel (:1568) */
  int32_t max_bounces;             /* settings.max_bounces, truncated to u8 like rc_stack.max_count (:220,1596) */
  rtr_vec3 background;             /* settings.background_color (:1584) */
  uint64_t seed;                   /* XORWOW seed; the reference uses 1234 (:1747) */
  uint32_t flags;                  /* RT_FLAG_* */
  uint32_t pad_;
} rt_params;

#define RT_FLAG_COUNT       0x1u   /* collect traversal/shading counters into rt_stats.counters */
#define RT_FLAG_GLOBAL_SCENE 0x2u  /* keep the scene in global memory even when it fits in LDS */
#define RT_FLAG_NO_JIT      0x4u   /* never use the scene-specialised (hipRTC) traversal */
#define RT_FLAG_FORCE_LANE   0x8u  /* force RT_TRAV_LANE   (A/B and parity tests; default: auto) */
#define RT_FLAG_FORCE_PACKET 0x10u /* force RT_TRAV_PACKET (falls back to LANE if the stack is too deep) */
#define RT_FLAG_FORCE_STATIC 0x20u /* force RT_TRAV_STATIC (over the visit budget: ACCEL if eligible, else LANE) */
#define RT_FLAG_NO_FOLD      0x40u /* RT_TRAV_STATIC without exact constant folding of primitive tests */
#define RT_FLAG_FORCE_ACCEL  0x80u /* force RT_TRAV_ACCEL (falls back to LANE when the world is not all spheres) */
#define RT_FLAG_NO_ACCEL     0x100u /* never use RT_TRAV_ACCEL */
#define RT_FLAG_FORCE_MIXED  0x400u /* force RT_TRAV_MIXED (falls back to LANE when no subtree qualifies) */
#define RT_FLAG_NO_MIXED     0x800u /* never use RT_TRAV_MIXED */
#define RT_FLAG_RC_AUDIT     0x200u /* test aid: count the colour-stack levels the render spilled to HBM
                                       (rt_stats.rc_hbm_slots); costs a fill + a read-back of that buffer */

/* traversal policies (rt_stats.traversal) */
#define RT_TRAV_LANE   0   /* per-lane DFS over an LDS stack (any scene) */
#define RT_TRAV_PACKET 1   /* one DFS per wave with per-entry lane masks */
#define RT_TRAV_STATIC 2   /* the scene's DFS expanded to straight-line code, compiled with hipRTC */
#define RT_TRAV_ACCEL  3   /* all-sphere worlds: SAH tree walk, verified against the reference tree per ray
                              (rays it cannot verify take the reference walk; bit-identical records) */
#define RT_TRAV_MIXED  4   /* worlds with transforms: the reference DFS above the transform-free subtrees, a
                              verified SAH walk inside them (same fallback rule; bit-identical records) */

/* rt_stats.counters[] slots (filled only with RT_FLAG_COUNT) */
enum {
  RT_CNT_VISIT_SPHERE = 0, RT_CNT_VISIT_BVH, RT_CNT_VISIT_TRIANGLE, RT_CNT_VISIT_QUAD,
  RT_CNT_VISIT_TRANSLATE, RT_CNT_VISIT_YROTATE, RT_CNT_VISIT_GROUP,
  RT_CNT_BOUNCES,          /* scattering hits (pushes onto the colour stack) */
  RT_CNT_SHADES,           /* closest-hit shading events (any material) */
  RT_CNT_PERLIN,           /* Perlin turbulence evaluations */
  RT_CNT_RNG_DRAWS,        /* uniform draws */
  RT_CNT_SAMPLES,
  RT_CNT_MAX_STACK,        /* deepest hit-stack use seen (max, not sum) */
  RT_CNT_STACK_OVERFLOW,   /* traversals that would have overflowed (must be 0) */
  RT_CNT_EXEC_NODE,        /* verified SAH walk (all-sphere worlds): node visits it executes (2 child boxes each) */
  RT_CNT_EXEC_PRIM,        /* verified SAH walk: leaf spheres it tests */
  RT_CNT__COUNT = 16
};

/* ABI 6: a render kernel as the register allocator built it.  Run-time (hipRTC) kernels: from the code object's
 * metadata note (NT_AMDGPU_METADATA) and its .comment; offline kernels: hipFuncGetAttributes (spill counts -1). */
typedef struct rt_kernel_info {
  int32_t vgprs;           /* VGPRs per lane (the wave's residency follows from it, 512 / granule-rounded count) */
  int32_t agprs;           /* AGPRs per lane (0: the path has no MFMA) */
  int32_t sgprs;           /* SGPRs per wave */
  int32_t scratch_bytes;   /* private segment per lane: > 0 means registers were spilled to memory */
  int32_t vgpr_spills;     /* VGPRs the allocator spilled (-1: unknown) */
  int32_t sgpr_spills;     /* SGPRs the allocator spilled (into VGPR lanes, or scratch) (-1: unknown) */
  int32_t blocks_per_cu;   /* resident blocks per CU the launch used (0 if not launched) */
  int32_t run_time;        /* 1: run-time compiled (hipRTC), 0: an offline kernel of librt_hip.so */
  char compiler[128];      /* the compiler's identification ("AMD clang version ..."), "" if unknown */
  char loader[128];        /* run-time kernels: where they were compiled ("helper:<lib dir>/rt_jitc", the child process
                              linked against /opt/rocm's hipRTC, or "process": this process's hipRTC); offline kernels: "" */
} rt_kernel_info;

typedef struct rt_stats {
  double init_ms;          /* RNG seeding kernel (reference: init_gpu_data, untimed there) */
  double render_ms;        /* render kernel (the reference's "Rendering time" region, :1752-1768) */
  double total_ms;         /* host wall time of the whole call */
  uint64_t samples;        /* pixels * spp rendered by this call */
  uint64_t counters[RT_CNT__COUNT];
  int32_t stack_needed;    /* exact worst-case hit-stack depth of this scene */
  int32_t scene_in_lds;    /* 1 if the compiled scene was staged in LDS */
  int32_t traversal;       /* RT_TRAV_* used by the last render */
  int32_t jit_visits;      /* node visits of the specialised traversal (RT_TRAV_STATIC) */
  double sched_ms;         /* longest-first schedule: probe paths + tile sort, before the render kernel */
  int32_t folded;          /* 1 if the specialised traversal used exactly folded primitive tests */
  int32_t fold_rerenders;  /* frames re-rendered unfolded after a ray left the host's bound (expect 0) */
  int32_t accel_spheres;   /* spheres in the verified traversal's tree (RT_TRAV_ACCEL), else 0 */
  int32_t accel_depth;     /* depth of that tree */
  uint32_t accel_fallbacks; /* rays of the last render the verified traversal re-traced with the reference walk */
  int32_t jit_source;      /* where the last render's run-time kernels came from: RT_JIT_* below */
  double jit_ms;           /* host time the last render spent obtaining them (compile or cache load) */
  uint64_t rc_hbm_slots;   /* RT_FLAG_RC_AUDIT: distinct HBM colour-stack slots (thread, level) written by the
                              render — > 0 proves levels past the LDS ones were pushed and unwound (:1253-1276) */
  int32_t rc_lds_levels;   /* colour-stack levels the last render kept in LDS (deeper ones live in HBM) */
  int32_t mix_macros;      /* RT_TRAV_MIXED: transform-free subtrees with a SAH walk (0 otherwise) */
  uint32_t mix_fallbacks;  /* RT_TRAV_MIXED: macro walks of the last render handed back to the reference walk */
  int32_t tiled_out;       /* 1: the last render wrote the float frame tile-major (coalesced 128-B lines) and a second
                              kernel wrote the caller's row-major floats and bytes; 0: each pixel stored row-major */
  /* ABI 5 */
  double render_kernel_ms; /* the render kernel alone: its first wave's start to its last wave's end on the device's
                              wall clock (s_memrealtime), what a profiler reports as the kernel duration; render_ms
                              is the stream-event window around the launch (>= this) */
  double gather_ms;        /* rt_multi_render / rt_render_devices: RCCL gather of the shards + on-device un-permute */
  int32_t devices;         /* devices that rendered the frame (1 for the single-device entry points) */
  int32_t rc_pool_chunks;  /* deep colour-stack levels: LDS pool chunks per wave of the last render (0: levels past
                              rc_lds_levels in HBM only; RT_RC_POOL) */
  /* ABI 6 */
  rt_kernel_info kernel;   /* the last render's render kernel */
} rt_stats;

/* rt_stats.jit_source */
#define RT_JIT_NONE      0   /* offline kernels only */
#define RT_JIT_MEMORY    1   /* module already loaded in this process */
#define RT_JIT_DISK      2   /* code object read from the on-disk cache (RT_JIT_CACHE_DIR) */
#define RT_JIT_COMPILED  3   /* compiled by hipRTC in this call (then written to the disk cache) */

/* One-shot: compile scene, upload, seed RNG, render, copy back.  out_rgb: host buffer of
 * row_count*width*3 floats (linear RGB, already scaled by 1/spp, row-major over the shard's rows).
 * The drop-in for raytracing.cu:1694-1771. */
int rt_render(const rt_scene *scene, const rt_camera *camera, const rt_params *params,
              float *out_rgb, rt_stats *stats);

/* Device-resident path: the scene stays in HBM across calls (bench / multi-GPU). */
typedef struct rt_context rt_context;
int rt_context_create(const rt_scene *scene, int device, rt_context **out);
/* out_rgb_device: device buffer of row_count*width*3 floats.  stream: hipStream_t (NULL = null
 * stream).  Asynchronous; timings are read with rt_context_timing() after the stream completes. */
int rt_context_render(rt_context *ctx, const rt_camera *camera, const rt_params *params,
                      float *out_rgb_device, void *stream);
/* rt_context_render that also writes the P6 payload (3 bytes per pixel, pixels_to_ppm's conversion,
 * raytracing.cu:1391-1395,1419-1431, bit-identical to rt_tonemap) of every pixel as the render kernel
 * finishes it, into out_ppm_device (row_count*width*3 bytes): no separate tonemap pass. */
int rt_context_render_ppm(rt_context *ctx, const rt_camera *camera, const rt_params *params,
                          float *out_rgb_device, uint8_t *out_ppm_device, void *stream);
/* Blocks on the last render's events; fills init/render ms, samples and (if counted) counters.
 * If the last rt_context_render* call failed (or none was made) the timings, samples and counters are
 * left 0: a failed call never reports an earlier frame's events.  A folded frame whose rays exceeded
 * the host's bound is re-rendered unfolded here (fold_rerenders), into the same float and PPM buffers. */
int rt_context_timing(rt_context *ctx, rt_stats *stats);
void rt_context_destroy(rt_context *ctx);

/* ---- one process, several devices (rows interleaved across the GPUs of a node, one RCCL gather) ----
 * The frame rows of `params` (row_offset + k*row_stride, k < row_count) are dealt round-robin: row k goes to
 * devices[k % n].  Each device renders its shard with its own rt_context on its own stream (no exchange while
 * rendering: pixels are independent and the RNG subsequence is the global pixel index, so the image is the same
 * bits for any n); then ONE grouped ncclGather (RCCL, rccl.h:745) collects every shard's rows — the P6 bytes
 * (3 B/px) and, when out_rgb is requested, the linear floats (12 B/px) — on devices[0], an un-permute kernel
 * restores row order there, and the frame is copied to the host.  RCCL is loaded on first use (dlopen of
 * librccl.so.1, the library torch.distributed's "nccl" backend also binds); without it these return
 * RT_ERR_UNSUPPORTED.  devices: distinct HIP device ordinals (ncclCommInitAll, rccl.h:236).
 * out_rgb (host, row_count*width*3 floats) and out_ppm (host, row_count*width*3 bytes, the P6 payload
 * of pixels_to_ppm): either may be NULL, not both.  stats (optional): timings are the maximum over the
 * devices, samples the total, plus gather_ms and devices.
 * rt_render_devices is the one-shot form (create, render, destroy): the multi-GPU drop-in for the device half
 * of render() (raytracing.cu:1694-1771, called once from main.cu:130). */
typedef struct rt_multi rt_multi;
int rt_multi_create(const rt_scene *scene, const int *devices, int n_devices, rt_multi **out);
int rt_multi_render(rt_multi *m, const rt_camera *camera, const rt_params *params, float *out_rgb, uint8_t *out_ppm,
                    rt_stats *stats);
void rt_multi_destroy(rt_multi *m);
int rt_render_devices(const rt_scene *scene, const rt_camera *camera, const rt_params *params, const int *devices,
                      int n_devices, float *out_rgb, uint8_t *out_ppm, rt_stats *stats);
/* The row deal of rt_multi_render (no device needed; tests): for the k-th row of a row_count-row frame over
 * n_devices devices, *device = k % n_devices and *local = k / n_devices, the row's index in that device's shard;
 * *shard_rows = that device's row count, *max_rows = the longest shard (the gather's per-device stride). */
int rt_multi_row_map(int32_t row_count, int32_t n_devices, int32_t k, int32_t *device, int32_t *local,
                     int32_t *shard_rows, int32_t *max_rows);
/* The root's un-permute step of rt_multi_render on its own (tests; one device is enough): `gathered` holds n_devices
 * shards of max_rows rows of row_bytes bytes (device memory; shard g's local row i at (g * max_rows + i) * row_bytes,
 * rows past a shard's own count are padding and never read), `out` receives row_count rows in frame order (frame row
 * k = shard k % n_devices, local row k / n_devices), asynchronously on `stream` (NULL: the null stream). */
int rt_multi_unpermute(const void *gathered_device, void *out_device, int32_t row_count, int32_t n_devices,
                       int32_t max_rows, uint32_t row_bytes, void *stream);

/* Device tonemap: the byte conversion of pixels_to_ppm (raytracing.cu:1391-1395,
 * 1419-1431) — sqrt gamma, clamp [0, 0.999], (u8)(256 x) — from a device framebuffer of `pixels`
 * RGB float triples to 3*pixels device bytes (P6 payload order), asynchronously on `stream`.
 * Bit-identical to the host conversion (rt_tonemap in rt_host.h). */
int rt_tonemap_device(const float *rgb_device, uint64_t pixels, uint8_t *out_device, void *stream);

/* Diagnostics for the scene-specialised traversal (no device needed).
 * rt_static_source: writes the hipRTC source for `scene` (NUL-terminated, truncated to cap) and the
 *   number of node visits of the expanded DFS; RT_ERR_UNSUPPORTED if it exceeds max_visits.
 * rt_static_compile: compiles that source for `arch` (e.g. "gfx950"); the compiler log goes to log. */
int rt_static_source(const rt_scene *scene, uint32_t max_visits, char *buf, uint64_t cap, uint32_t *visits);
int rt_static_compile(const rt_scene *scene, uint32_t max_visits, const char *arch, char *log, uint64_t cap);
/* The run-time (hipRTC) source of any traversal's kernels for `scene` as a render with max_bounces
 * would build it (traversal = RT_TRAV_STATIC, RT_TRAV_ACCEL, RT_TRAV_MIXED or RT_TRAV_LANE; no device
 * needed): ISA / register / scratch inspection with hipcc (tools/isa_stats.sh). */
int rt_kernel_source(const rt_scene *scene, int traversal, int32_t max_bounces, char *buf, uint64_t cap);
/* The render kernel that source compiles to (no device needed): rt_kernel_source's source built by the same run-time
 * compiler, options and register-budget rules a render applies before its device-dependent residency step (the verified
 * sphere walk's 6-wave request kept only without scratch).  Diagnostics and the CPU test that the default kernels of
 * every BASELINE config build without spills. */
int rt_kernel_build(const rt_scene *scene, int traversal, int32_t max_bounces, rt_kernel_info *out);
/* Diagnostics for the verified mixed-world traversal (no device needed): info = {macro roots, dynamic
 * ones, primitives in their SAH trees, deepest SAH tree}; RT_ERR_UNSUPPORTED when no subtree qualifies.
 * The build reads the RT_MIX_* environment knobs (e.g. RT_MIX_DYN_MIN, the dynamic-macro primitive
 * threshold) exactly as rt_context_create does, so the counts depend on them. */
int rt_mixed_build(const rt_scene *scene, uint32_t info[4]);
/* Diagnostics for the verified sphere traversal (no device needed): builds the SAH tree of an
 * all-sphere world.  info = {root node, depth, spheres, node words}; words (if non-null, cap words)
 * receives the node words then the prim words (layout: device/rt_layout.h kAccel*).
 * RT_ERR_UNSUPPORTED when the world is not eligible. */
int rt_accel_build(const rt_scene *scene, uint32_t *words, uint64_t cap, uint32_t info[4]);
/* The same tree 4 wide (the verified walk's RT_ACCEL_WIDTH=4 form, device/rt_layout.h kAccel4*; no device
 * needed): info = {wide nodes, depth, stack bound of the ordered walk, node words}; words (if non-null, cap
 * words) receives the node words.  RT_ERR_UNSUPPORTED when the world is not eligible. */
int rt_accel_build_wide(const rt_scene *scene, uint32_t *words, uint64_t cap, uint32_t info[4]);
/* The 4-wide tree quantised (the verified walk's RT_ACCEL_QUANT=1 form; device/rt_layout.h kAccel4Q*,
 * one 64-B line per node; no device needed): info and words as rt_accel_build_wide's, same node numbering.
 * RT_ERR_UNSUPPORTED when the world is not eligible or its boxes exceed the quantiser's exponent range. */
int rt_accel_build_quant(const rt_scene *scene, uint32_t *words, uint64_t cap, uint32_t info[4]);
/* The verified sphere walk's primary-ray candidate lists of a frame, built on the host with the code the device
 * runs per frame (device/prim_lists.h; no device needed; tests): for every 8x8 tile of the shard p describes,
 * counts[tile] = entries (0xffffffff: no list, the tile's camera rays walk the tree) and, if lists is non-null,
 * lists[(tile * cap + k) * 2 + {0, 1}] = {sphere index in the SAH prim order, axial lower bound as float bits},
 * ascending; *rho (if non-null) = the origin radius bound the kernel's early exit uses.  RT_ERR_UNSUPPORTED when
 * the world is not eligible for the verified sphere walk. */
int rt_prim_lists(const rt_scene *scene, const rt_camera *cam, const rt_params *p, uint32_t cap, uint32_t *counts,
                  uint32_t *lists, float *rho);
/* The per-pixel XORWOW states rt_render seeds on the device (init_gpu_data's curand_init,
 * raytracing.cu:1591-1606, subsequence = global pixel index), for rows row_offset + k*row_stride,
 * k < rows, of a width-wide frame: out_states (host) receives [6][rows*width] words {d, x0..x4}.
 * Diagnostics/tests: the render path seeds into device memory and never copies the states back. */
int rt_seed_states(uint64_t seed, int width, int row_offset, int row_stride, int rows, uint32_t *out_states);
/* The per-pixel states as the render kernel derives them at tile pickup, computed on the host from the same
 * tables (no device needed; tests): phase base (row, column & 7) — the row's first state jumped over its first
 * columns — times the nibble table of J^(8 * (column >> 3)).  For rows row_offset + k*row_stride, k < rows, of
 * a width-wide frame, out (rows*width*6 words, pixel-major) receives {d, x0..x4}; equal to rt_seed_states's
 * states of the same pixels. */
int rt_rng_table_states(uint64_t seed, int width, int row_offset, int row_stride, int rows, uint32_t *out);
/* Last fallback reason of a context (why RT_TRAV_STATIC was not used); "" if none. */
const char *rt_context_note(const rt_context *ctx);

const char *rt_status_string(int status);
/* Build stamp: the files this library was built from (space separated, repository-relative) and the first 16 hex digits
 * of the sha256 of their bytes in that order; the Python binding refuses a library that does not match its tree. */
const char *rt_hip_build_hash(void);
const char *rt_hip_build_files(void);
int rt_device_count(int *count);
int rt_abi_version(void);

/* CPU oracle (oracle/liboracle_rt.so) — test infrastructure only, same contract as rt_render. */
int rt_render_cpu(const rt_scene *scene, const rt_camera *camera, const rt_params *params,
                  float *out_rgb, rt_stats *stats);

#ifdef __cplusplus
}
#endif
#endif /* RT_RENDER_H */
