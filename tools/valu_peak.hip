// valu_peak.hip — measured VALU issue rates of one MI355X, for the roofline peak of bench.py.
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_peak.hip -o tools/valu_peak && tools/valu_peak
// Each thread runs 16 independent chains of one instruction kind, 8 waves per SIMD; prints the
// lane-instructions per second of each kind and the ratio to 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kChains = 16, kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void op_kernel(float *out, float a, float b) {
  float x[kChains];
  uint32_t u[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) { x[c] = threadIdx.x * 1e-3f + c; u[c] = threadIdx.x * 2654435761u + c; }
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0) x[c] = __builtin_fmaf(x[c], a, b);          // v_fma_f32
      else if (OP == 1) x[c] = x[c] + a;                       // v_add_f32
      else if (OP == 2) x[c] = x[c] * a;                       // v_mul_f32
      else if (OP == 4) x[c] = (c & 1) ? x[c] * a : x[c] + b;  // mul/add mix
    }
    if (OP == 5) {                                              // v_pk_fma_f32: 2 f32 fmas per lane
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 *y = reinterpret_cast<f2 *>(x);
      const f2 a2 = {a, a}, b2 = {b, b};
#pragma unroll
      for (int c = 0; c < kChains / 2; ++c) y[c] = __builtin_elementwise_fma(y[c], a2, b2);
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += x[c] + static_cast<float>(u[c]);
  if (s == 12345.678f) out[threadIdx.x] = s;   // keeps the chains live
}

template <int OP>
double rate(float *out, int blocks, double ops_per_step) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  op_kernel<OP><<<blocks, 256>>>(out, 0.999f, 0.001f);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    (void)hipEventRecord(e0);
    op_kernel<OP><<<blocks, 256>>>(out, 0.999f, 0.001f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return static_cast<double>(blocks) * 256 * kChains * kIters * ops_per_step / (best * 1e-3);
}

int main() {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) { std::printf("{\"error\": \"no device\"}\n"); return 1; }
  float *out = nullptr;
  if (hipMalloc(&out, 4096) != hipSuccess) return 1;
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;   // 8 blocks x 4 waves per CU = 8 waves per SIMD
  const double spec = static_cast<double>(cus) * 4 * 32 * 2.4e9;
  const double r[5] = {rate<0>(out, blocks, 1), rate<1>(out, blocks, 1), rate<2>(out, blocks, 1),
                       rate<4>(out, blocks, 1), rate<5>(out, blocks, 1)};
  const char *names[5] = {"v_fma_f32", "v_add_f32", "v_mul_f32", "v_mul_f32/v_add_f32", "v_pk_fma_f32 (2 fma/lane)"};
  std::printf("{\"cus\": %d, \"clock_mhz\": %d, \"spec_lane_ops_per_s\": %.4e, \"rates\": {", cus, prop.clockRate / 1000, spec);
  for (int k = 0; k < 5; ++k)
    std::printf("%s\"%s\": {\"lane_ops_per_s\": %.4e, \"fraction_of_spec\": %.4f}", k ? ", " : "", names[k], r[k], r[k] / spec);
  std::printf("}}\n");
  (void)hipFree(out);
  return 0;
}
