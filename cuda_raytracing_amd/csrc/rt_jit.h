// rt_jit.h — scene-specialised render kernels compiled at run time with hipRTC.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "code_object.h"
#include "gpu_scene.h"

namespace rt {

struct JitKernels {
  hipFunction_t render = nullptr;        // StaticTrace, no counters
  hipFunction_t render_count = nullptr;  // StaticTrace, counters
  hipFunction_t probe = nullptr;         // StaticTrace, schedule probe launches (same body, own symbol)
  uint32_t visits = 0;                   // node visits in the expanded traversal
  bool folded = false;                   // primitive tests exactly folded (scene_codegen.cpp)
  int source = 0;                        // RT_JIT_MEMORY / RT_JIT_DISK / RT_JIT_COMPILED (rt_render.h)
  double ms = 0.0;                       // host time spent obtaining the module in this call
  KernelMeta meta_render, meta_count;    // what the register allocator made of render / render_count (code object)
  std::string compiler;                  // the compiler that built the module (its .comment line)
};

// Compile (or fetch from the process-wide cache) the StaticTrace kernels of `img` for `variant`
// (kVarLds | kVarNoise | kVarUv bits) on the current device.  Returns false (and a reason in *why)
// when the scene is too large for the expansion budget or hipRTC is unavailable / fails: callers
// then keep the generic kernels.
bool jit_kernels(const SceneImage &img, int variant, uint32_t max_visits, bool fold, JitKernels *out, std::string *why);

// Full hipRTC source of the StaticTrace kernels for `variant` (no device needed).
bool jit_source(const SceneImage &img, int variant, uint32_t max_visits, bool fold, std::string *src, uint32_t *visits,
                bool *folded = nullptr, int waves = 0);   // waves > 0: amdgpu_waves_per_eu (0: RT_JIT_WAVES or none)
// Compile `src` for `arch` (e.g. "gfx950"); on success the code object is in *code.  No device needed.
// `extra`: options after the common ones (the verified sphere walk's scheduler strategy, accel_sched)
bool jit_compile(const std::string &src, const std::string &arch, std::vector<char> *code, std::string *log,
                 const std::vector<std::string> &extra = {});

// Per-lane DFS kernels specialised on the node kinds present in the scene (large scenes: the
// kind dispatch of trav_step keeps only those branches).  Same contract as jit_kernels.
bool jit_lane_kernels(const SceneImage &img, int variant, JitKernels *out, std::string *why);
std::string jit_lane_source(const SceneImage &img, int variant);
// Verified sphere traversal kernels (AccelTraceK over the scene's node kinds for the fallback walk); wide: the
// 4-wide tree (SphereAccel::wide_words)
bool jit_accel_kernels(const SceneImage &img, int variant, int wide, JitKernels *out, std::string *why);   // wide: 0 BVH2, 1 4-wide, 2 quantised 4-wide
std::string jit_accel_source(const SceneImage &img, int variant, int waves = 0, int wide = 0);   // waves > 0: amdgpu_waves_per_eu
int accel_width();   // 2 or 4 (RT_ACCEL_WIDTH)
bool accel_quant();  // the 4-wide tree quantised (RT_ACCEL_QUANT, default off)
int accel_waves(int wide = 0);   // the verified walk's waves per SIMD request (6, 4-wide 5; RT_ACCEL_WAVES, 0 = allocator's choice)
// verified mixed-world traversal kernels (MixedTraceK over the scene's node kinds)
bool jit_mixed_kernels(const SceneImage &img, int variant, JitKernels *out, std::string *why);
std::string jit_mixed_source(const SceneImage &img, int variant, int waves = 0);
uint32_t scene_kinds(const SceneImage &img);
// material / texture kinds present, as variant bits (kVarMatShift / kVarTexShift)
int scene_shading_bits(const SceneImage &img);

// where the run-time compiler comes from: "dlmopen:<libhiprtc path>" (default: /opt/rocm's, in a link namespace of
// its own) or "process" (RT_JIT_COMPILER=process, or the fallback when that load fails)
std::string jit_compiler_where();

// extra hipRTC options from the RT_JIT_OPTS environment variable (space separated)
std::vector<std::string> jit_extra_options();
// the complete hipRTC option vector for `arch` (numerics flags + RT_JIT_OPTS); hashed into the disk-cache key
std::vector<std::string> jit_options(const std::string &arch, const std::vector<std::string> &extra = {});

// the machine-scheduler options of the scene-specialised kernels and of the verified sphere walk (RT_STATIC_SCHED,
// RT_ACCEL_SCHED)
std::vector<std::string> static_sched(const SceneImage &img);
std::vector<std::string> accel_sched();
std::vector<std::string> mixed_sched();
// the verified walk's default waves request is kept only when its build has no more scratch than this (0)
bool accel_waves_build_kept(int scratch_bytes);
// compile `src` for `arch` with the run-time compiler and options (no device) and read <prefix>_render's figures
bool jit_build_meta(const std::string &src, const std::string &prefix, const std::vector<std::string> &extra,
                    const std::string &arch, KernelMeta *m, std::string *compiler, std::string *why);

hipError_t jit_launch(hipFunction_t fn, const RenderArgs &a, uint32_t blocks, size_t lds_bytes, hipStream_t s);
int jit_blocks_per_cu(hipFunction_t fn, size_t lds_bytes);

}  // namespace rt
