// rt_multi.cpp — one process, several devices: the multi-GPU form of render()'s device half
// (raytracing.cu:1694-1771, called once from main.cu:130), SURVEY §8e.
//
// Pixels are independent and the RNG subsequence is the global pixel index (:1604), so a frame shards by rows
// with no exchange while rendering.  Rows are dealt round-robin (row k of the frame -> device k % n): contiguous
// bands would be unbalanced (a scene's sky rows end at bounce 0).  Each device renders its shard through its own
// rt_context on its own stream; then one grouped RCCL gather (ncclGather, rccl.h:745) brings every shard's rows
// to devices[0] — the P6 bytes (3 B/px) and, when asked for, the linear floats — where an un-permute kernel
// puts them back in frame order before the single copy to the host.  Over xGMI the root receives the n-1 other
// shards on distinct links at once; at 1080p that is 0.78 MB of bytes per device at n = 8.
//
// RCCL is bound at run time (dlopen of librccl.so.1 — the library torch.distributed's "nccl" backend maps too, so
// a process that already loaded it shares that copy): the single-device entry points do not depend on it, and
// without it these entry points return RT_ERR_UNSUPPORTED instead of failing to load.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "rt_kernels.h"
#include "rt_render.h"

namespace {

struct Rccl {
  bool ok = false;
  ncclResult_t (*comm_init_all)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(h, "ncclGather"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.ok = r.comm_init_all && r.comm_destroy && r.gather && r.group_start && r.group_end;
  });
  return r;
}

struct Buf {
  void *p = nullptr;
  size_t bytes = 0;
  bool ensure(size_t n) {
    if (n <= bytes && p) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, n ? n : 1) != hipSuccess) { p = nullptr; return false; }
    bytes = n;
    return true;
  }
  void release() { if (p) (void)hipFree(p); p = nullptr; bytes = 0; }
};

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) { if (hipGetDevice(&prev) != hipSuccess) prev = -1; (void)hipSetDevice(dev); }
  ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// rows of the round-robin deal: device g of n renders frame rows g, g + n, ... (row_count rows in all)
inline int32_t shard_rows(int32_t rows, int32_t n, int32_t g) { return rows > g ? (rows - g + n - 1) / n : 0; }

}  // namespace

struct rt_multi {
  int n = 0;
  std::vector<int> dev;
  std::vector<rt_context *> ctx;
  std::vector<hipStream_t> stream;
  std::vector<ncclComm_t> comm;
  std::vector<Buf> f32, u8;      // per device: its shard, padded to the longest shard
  Buf g_f32, g_u8, o_f32, o_u8;  // devices[0]: gathered shards, frame in row order
  hipEvent_t ev[2] = {nullptr, nullptr};   // devices[0]: gather start, un-permute end
};

extern "C" {

int rt_multi_row_map(int32_t row_count, int32_t n, int32_t k, int32_t *device, int32_t *local, int32_t *rows_of,
                     int32_t *max_rows) {
  if (row_count < 0 || n <= 0 || k < 0 || k >= row_count) return RT_ERR_INVALID_ARG;
  const int32_t g = k % n;
  if (device) *device = g;
  if (local) *local = k / n;
  if (rows_of) *rows_of = shard_rows(row_count, n, g);
  if (max_rows) *max_rows = shard_rows(row_count, n, 0);
  return RT_OK;
}

int rt_multi_unpermute(const void *gathered_device, void *out_device, int32_t row_count, int32_t n_devices,
                       int32_t max_rows, uint32_t row_bytes, void *stream) {
  if (row_count < 0 || n_devices <= 0 || max_rows < 0 || (row_count > 0 && (!gathered_device || !out_device)))
    return RT_ERR_INVALID_ARG;
  if (max_rows < shard_rows(row_count, n_devices, 0)) return RT_ERR_INVALID_ARG;
  return rt::launch_unpermute(gathered_device, out_device, static_cast<uint32_t>(row_count),
                              static_cast<uint32_t>(n_devices), static_cast<uint32_t>(max_rows), row_bytes,
                              static_cast<hipStream_t>(stream)) == hipSuccess ? RT_OK : RT_ERR_HIP;
}

void rt_multi_destroy(rt_multi *m) {
  if (!m) return;
  const Rccl &R = rccl();
  for (size_t g = 0; g < m->dev.size(); ++g) {
    DeviceGuard guard(m->dev[g]);
    if (g < m->comm.size() && m->comm[g] && R.ok) (void)R.comm_destroy(m->comm[g]);
    if (g < m->ctx.size() && m->ctx[g]) rt_context_destroy(m->ctx[g]);
    if (g < m->stream.size() && m->stream[g]) (void)hipStreamDestroy(m->stream[g]);
    if (g < m->f32.size()) m->f32[g].release();
    if (g < m->u8.size()) m->u8[g].release();
    if (g == 0) {
      m->g_f32.release(); m->g_u8.release(); m->o_f32.release(); m->o_u8.release();
      for (hipEvent_t &e : m->ev) if (e) (void)hipEventDestroy(e);
    }
  }
  delete m;
}

int rt_multi_create(const rt_scene *scene, const int *devices, int n, rt_multi **out) {
  if (!scene || !devices || n <= 0 || !out) return RT_ERR_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_ERR_NO_DEVICE;
  for (int g = 0; g < n; ++g) {
    if (devices[g] < 0 || devices[g] >= ndev) return RT_ERR_INVALID_ARG;
    for (int h = 0; h < g; ++h) if (devices[h] == devices[g]) return RT_ERR_INVALID_ARG;   // one rank per GPU
  }
  const Rccl &R = rccl();
  if (!R.ok) return RT_ERR_UNSUPPORTED;
  rt_multi *m = new (std::nothrow) rt_multi();
  if (!m) return RT_ERR_INVALID_ARG;
  m->n = n;
  m->dev.assign(devices, devices + n);
  m->ctx.assign(n, nullptr);
  m->stream.assign(n, nullptr);
  m->f32.resize(n);
  m->u8.resize(n);
  for (int g = 0; g < n; ++g) {
    const int st = rt_context_create(scene, devices[g], &m->ctx[g]);
    if (st != RT_OK) { rt_multi_destroy(m); return st; }
    DeviceGuard guard(devices[g]);
    if (hipStreamCreateWithFlags(&m->stream[g], hipStreamNonBlocking) != hipSuccess) { rt_multi_destroy(m); return RT_ERR_HIP; }
    if (g == 0)
      for (hipEvent_t &e : m->ev)
        if (hipEventCreate(&e) != hipSuccess) { rt_multi_destroy(m); return RT_ERR_HIP; }
  }
  m->comm.assign(n, nullptr);
  if (R.comm_init_all(m->comm.data(), n, devices) != ncclSuccess) {
    m->comm.assign(n, nullptr);
    rt_multi_destroy(m);
    return RT_ERR_HIP;
  }
  *out = m;
  return RT_OK;
}

int rt_multi_render(rt_multi *m, const rt_camera *cam, const rt_params *p, float *out_rgb, uint8_t *out_ppm,
                    rt_stats *stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (!m || !cam || !p || (!out_rgb && !out_ppm)) return RT_ERR_INVALID_ARG;
  if (p->width <= 0 || p->row_count < 0 || p->row_stride <= 0 || p->row_offset < 0) return RT_ERR_INVALID_ARG;
  const int n = m->n;
  const int32_t rows = p->row_count, W = p->width;
  const int32_t max_rows = shard_rows(rows, n, 0);
  const size_t px_max = static_cast<size_t>(max_rows) * static_cast<size_t>(W);
  // the shards (row_offset + g*stride, stride*n, shard_rows) — rt_context_render_ppm checks each against the frame
  if (static_cast<int64_t>(p->row_stride) * n > 0x7fffffffll) return RT_ERR_INVALID_ARG;
  rt_stats acc{};
  acc.devices = n;
  std::vector<rt_params> sp(n, *p);
  for (int g = 0; g < n; ++g) {
    sp[g].row_offset = p->row_offset + (rows > g ? g * p->row_stride : 0);
    sp[g].row_stride = p->row_stride * n;
    sp[g].row_count = shard_rows(rows, n, g);
    DeviceGuard guard(m->dev[g]);
    if (!m->f32[g].ensure(px_max * 12) || !m->u8[g].ensure(px_max * 3)) return RT_ERR_HIP;
    const int st = rt_context_render_ppm(m->ctx[g], cam, &sp[g], static_cast<float *>(m->f32[g].p),
                                         out_ppm ? static_cast<uint8_t *>(m->u8[g].p) : nullptr, m->stream[g]);
    if (st != RT_OK) return st;
  }
  // every shard done (rt_context_timing also re-renders a folded frame whose rays left the host's bound, before
  // its rows are gathered); timings are the slowest device's, samples and counters the sums
  for (int g = 0; g < n; ++g) {
    rt_stats s{};
    const int st = rt_context_timing(m->ctx[g], &s);
    if (st != RT_OK) return st;
    if (g == 0) acc = s;
    else {
      acc.init_ms = std::max(acc.init_ms, s.init_ms);
      acc.render_ms = std::max(acc.render_ms, s.render_ms);
      acc.sched_ms = std::max(acc.sched_ms, s.sched_ms);
      acc.render_kernel_ms = std::max(acc.render_kernel_ms, s.render_kernel_ms);
      acc.samples += s.samples;
      for (int k = 0; k < RT_CNT__COUNT; ++k)
        acc.counters[k] = k == RT_CNT_MAX_STACK ? std::max(acc.counters[k], s.counters[k]) : acc.counters[k] + s.counters[k];
      acc.fold_rerenders += s.fold_rerenders;
      acc.accel_fallbacks += s.accel_fallbacks;
      acc.mix_fallbacks += s.mix_fallbacks;
      acc.rc_hbm_slots += s.rc_hbm_slots;
    }
  }
  acc.devices = n;
  if (rows > 0) {
    const Rccl &R = rccl();
    const size_t u8_count = px_max * 3, f32_count = px_max * 3;
    {
      DeviceGuard guard(m->dev[0]);
      if ((out_ppm && (!m->g_u8.ensure(u8_count * n) || !m->o_u8.ensure(static_cast<size_t>(rows) * W * 3))) ||
          (out_rgb && (!m->g_f32.ensure(f32_count * 4 * n) || !m->o_f32.ensure(static_cast<size_t>(rows) * W * 12))))
        return RT_ERR_HIP;
      if (hipEventRecord(m->ev[0], m->stream[0]) != hipSuccess) return RT_ERR_HIP;
    }
    if (R.group_start() != ncclSuccess) return RT_ERR_HIP;
    bool ok = true;
    for (int g = 0; g < n && ok; ++g) {
      if (out_ppm)
        ok = R.gather(m->u8[g].p, g == 0 ? m->g_u8.p : nullptr, u8_count, ncclUint8, 0, m->comm[g], m->stream[g]) == ncclSuccess;
      if (ok && out_rgb)
        ok = R.gather(m->f32[g].p, g == 0 ? m->g_f32.p : nullptr, f32_count, ncclFloat32, 0, m->comm[g], m->stream[g]) ==
             ncclSuccess;
    }
    if (R.group_end() != ncclSuccess || !ok) return RT_ERR_HIP;
    DeviceGuard guard(m->dev[0]);
    hipStream_t s0 = m->stream[0];
    if (out_ppm && rt::launch_unpermute(m->g_u8.p, m->o_u8.p, static_cast<uint32_t>(rows), static_cast<uint32_t>(n),
                                        static_cast<uint32_t>(max_rows), static_cast<uint32_t>(W) * 3u, s0) != hipSuccess)
      return RT_ERR_HIP;
    if (out_rgb && rt::launch_unpermute(m->g_f32.p, m->o_f32.p, static_cast<uint32_t>(rows), static_cast<uint32_t>(n),
                                        static_cast<uint32_t>(max_rows), static_cast<uint32_t>(W) * 12u, s0) != hipSuccess)
      return RT_ERR_HIP;
    if (hipEventRecord(m->ev[1], s0) != hipSuccess) return RT_ERR_HIP;
    if (out_ppm && hipMemcpyAsync(out_ppm, m->o_u8.p, static_cast<size_t>(rows) * W * 3, hipMemcpyDeviceToHost, s0) != hipSuccess)
      return RT_ERR_HIP;
    if (out_rgb && hipMemcpyAsync(out_rgb, m->o_f32.p, static_cast<size_t>(rows) * W * 12, hipMemcpyDeviceToHost, s0) != hipSuccess)
      return RT_ERR_HIP;
    if (hipStreamSynchronize(s0) != hipSuccess) return RT_ERR_HIP;
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, m->ev[0], m->ev[1]) == hipSuccess) acc.gather_ms = ms;
  }
  acc.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (stats) *stats = acc;
  return RT_OK;
}

int rt_render_devices(const rt_scene *scene, const rt_camera *cam, const rt_params *p, const int *devices, int n,
                      float *out_rgb, uint8_t *out_ppm, rt_stats *stats) {
  const auto t0 = std::chrono::steady_clock::now();
  rt_multi *m = nullptr;
  int st = rt_multi_create(scene, devices, n, &m);
  if (st != RT_OK) return st;
  st = rt_multi_render(m, cam, p, out_rgb, out_ppm, stats);
  rt_multi_destroy(m);
  if (st == RT_OK && stats)
    stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return st;
}

}  // extern "C"
