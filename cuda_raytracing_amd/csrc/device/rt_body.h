// rt_body.h — device code of the per-pixel render path (gfx950).
//
// Replaces cuda_calc (raytracing.cu:1543-1589) + ray_color (:1333-1371) + hit (:1079-1251) +
// materials/textures/Perlin (:356-502, perlin_noise.cpp).  Compiled twice: offline by hipcc
// (rt_device.hip: generic per-lane / packet traversal) and at run time by hipRTC (rt_jit.cpp: the
// traversal of one specific scene expanded into straight-line code).  It therefore includes nothing
// but rt_layout.h; the including translation unit provides the HIP device runtime.
//
// Arithmetic is the reference's, op for op: built with -ffp-contract=off and correctly rounded f32
// divide/sqrt, ternary MIN/MAX semantics, the same RNG draw order — bit-exact against the oracle.
#pragma once
// RT_PRIM_LISTS=0 (RT_JIT_OPTS=-DRT_PRIM_LISTS=0) compiles the verified walk without the camera-ray list path (A/B)
#ifndef RT_PRIM_LISTS
#define RT_PRIM_LISTS 1
#endif
#include "rt_layout.h"

#ifndef RT_UNWIND_BATCH
#define RT_UNWIND_BATCH 8   // HBM colour-stack levels loaded per batch in the deep-path unwind
#endif
#ifndef RT_UNWIND_LDS
#define RT_UNWIND_LDS 3     // LDS colour-stack levels loaded per batch in the unwind
#endif
#ifndef RT_UNWIND_LDS_DEEP
// ... in deep-path kernels (max_bounces > kDeepBounces).  5 since round 5: the Cornell and 4K scene-0 d50 kernels then
// fit 80 VGPRs (6 waves) without spilling (8: 87 VGPRs, 5 waves); same box: Cornell -4.5 %, 4K -7 %, Perlin level
// (profiles/r05_ab_s29_*.jsonl)
#define RT_UNWIND_LDS_DEEP 5
#endif

namespace rt {

// [scene image (LDS variant)] [colour-stack levels 0..rc_lds_levels-1] [per-lane traversal stacks]
extern __shared__ uint32_t g_lds[];

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 scale(float s, f3 v) { return mk(v.x * s, v.y * s, v.z * s); }
__device__ __forceinline__ f3 flip(f3 v) { return mk(-v.x, -v.y, -v.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float length(f3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ f3 unit(f3 v) {              // vec3.h:106-114 (three divisions)
  float l = length(v);
  if (l == 0.0f) return mk(0.0f, 0.0f, 0.0f);
  return mk(v.x / l, v.y / l, v.z / l);
}
__device__ __forceinline__ f3 line_at(f3 o, float t, f3 d) { return add(o, scale(t, d)); }
__device__ __forceinline__ float tmin_(float a, float b) { return (a < b) ? a : b; }   // utility.h:6
__device__ __forceinline__ float tmax_(float a, float b) { return (a < b) ? b : a; }   // utility.h:7
__device__ __forceinline__ float asf(uint32_t u) { return __uint_as_float(u); }

// |denom| >= 1e-8 (a double literal, raytracing.cu:1064) <=> |denom| >= the smallest float >= 1e-8
constexpr float kDenomEps = 1.00000008274037099e-08f;   // 0x322BCC78
static_assert(kDenomEps > 1e-8 && (kDenomEps - 1e-8) < 1e-15, "denominator threshold");
constexpr float kTmin = 0.001f;                          // ray_tmin (raytracing.cu:1341)

// ---------------------------------------------------------------------------------------------
// scene memory: one word image, either in LDS or in HBM (read-only)
// ---------------------------------------------------------------------------------------------
template <bool LDS>
struct Mem {
  const uint32_t *__restrict__ g;
  __device__ __forceinline__ uint32_t w(uint32_t i) const { return LDS ? g_lds[i] : g[i]; }
  __device__ __forceinline__ float f(uint32_t i) const { return asf(w(i)); }
  __device__ __forceinline__ uint4 w4(uint32_t i) const {   // i % 4 == 0
    return LDS ? *reinterpret_cast<const uint4 *>(&g_lds[i]) : *reinterpret_cast<const uint4 *>(&g[i]);
  }
  __device__ __forceinline__ uint32_t byte(uint32_t word_base, uint32_t b) const {
    return LDS ? reinterpret_cast<const uint8_t *>(&g_lds[word_base])[b]
               : reinterpret_cast<const uint8_t *>(&g[word_base])[b];
  }
  __device__ __forceinline__ uint32_t half(uint32_t word_base, uint32_t k) const {
    return LDS ? reinterpret_cast<const uint16_t *>(&g_lds[word_base])[k]
               : reinterpret_cast<const uint16_t *>(&g[word_base])[k];
  }
};

// ---------------------------------------------------------------------------------------------
// device checks (RT_DEVICE_CHECKS builds; rt_layout.h CheckSite): RT_CHECK(A, cond, site, index, capacity) is true when
// cond holds; otherwise the first failing site of the launch, its index and capacity go to work words kCheckWord..+2,
// and the caller skips the access.  Without RT_DEVICE_CHECKS it is the constant true and compiles away.
// ---------------------------------------------------------------------------------------------
__device__ __noinline__ bool check_fail(const RenderArgs &A, uint32_t site, uint32_t index, uint32_t cap) {
  // the address and the values through VGPRs: with wave-uniform operands the instruction selector may otherwise pick a
  // scalar-memory atomic (LLVM 22 did, and then failed to encode it for gfx950); these are vector (global) atomics
  uint32_t *w = A.work + kCheckWord;
  asm volatile("" : "+v"(w), "+v"(site), "+v"(index), "+v"(cap));
  if (atomicCAS(w, 0u, site) == 0u) {
    atomicExch(w + 1, index);
    atomicExch(w + 2, cap);
  }
  return false;
}
#ifdef RT_DEVICE_CHECKS
#define RT_CHECK(A, cond, site, index, cap) \
  (__builtin_expect(!!(cond), 1) ? true : check_fail((A), (site), static_cast<uint32_t>(index), static_cast<uint32_t>(cap)))
#else
#define RT_CHECK(A, cond, site, index, cap) true
#endif

// ---------------------------------------------------------------------------------------------
// RNG: rocRAND XORWOW (replaces cuRAND)
// ---------------------------------------------------------------------------------------------
// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96); LLVM does not form it for
// 32-bit xor chains by itself
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// x <- P x through the nibble table of P (kRngNibTableWords at byte tb of the buffer rs): 40 lookups of 5 words,
// XOR-summed.  Raw buffer loads (scalar descriptor + one 32-bit offset VGPR per gather) in twenty groups of two
// (a rolled loop: one group's gathers in flight together, without the registers of a fully unrolled product;
// this runs once per tile pickup, not per sample)
__device__ __forceinline__ void rng_jump_nib(__amdgpu_buffer_rsrc_t rs, uint32_t tb, uint32_t &x0, uint32_t &x1,
                                             uint32_t &x2, uint32_t &x3, uint32_t &x4) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
#pragma unroll 1
  for (uint32_t g = 0; g < 20; ++g) {
    const uint32_t w = g >> 2;
    const uint32_t xw = (w == 0 ? x0 : (w == 1 ? x1 : (w == 2 ? x2 : (w == 3 ? x3 : x4)))) >> ((g & 3u) * 8u);
#pragma unroll
    for (uint32_t q = 0; q < 2; ++q) {
      const uint32_t e = (g * 2 + q) * 16 + ((xw >> (4 * q)) & 15u);
      const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, tb + e * 16u, 0, 0);
      r0 ^= a.x; r1 ^= a.y; r2 ^= a.z; r3 ^= a.w;
      r4 ^= __builtin_amdgcn_raw_buffer_load_b32(rs, tb + 40u * 16u * 16u + e * 4u, 0, 0);
    }
  }
  x0 = r0; x1 = r1; x2 = r2; x3 = r3; x4 = r4;
}

struct Rng {
  uint32_t d, x0, x1, x2, x3, x4;
  __device__ __forceinline__ uint32_t next() {
    uint32_t t = x0 ^ (x0 >> 2);
    x0 = x1; x1 = x2; x2 = x3; x3 = x4;
    x4 = xor3(x4, x4 << 4, t) ^ (t << 1);
    d += 362437u;
    return d + x4;
  }
  // rocrand_uniform: inv + f*inv with f = (float)v, inv = 2^-32 — in (0, 1].  f*inv is exact (a
  // power-of-two scale of a float >= 1), so one fma with the same operands rounds identically to the
  // reference's multiply-then-add: this is an exact rewrite, not a contraction.
  __device__ __forceinline__ float uniform() {
    const float inv = 2.3283064e-10f;
    return __builtin_fmaf(static_cast<float>(next()), inv, inv);
  }
  __device__ __forceinline__ float bound(float lo, float hi) { return lo + (hi - lo) * uniform(); }
  // bound(-1, 1) = -1 + 2*uniform(); 2*uniform() = fl(2inv + f*2inv) exactly (scaling by 2 commutes
  // with rounding), again a single exact fma
  __device__ __forceinline__ float sym() {
    const float inv2 = 4.6566129e-10f;   // 2^-31
    return -1.0f + __builtin_fmaf(static_cast<float>(next()), inv2, inv2);
  }
};

// ---------------------------------------------------------------------------------------------
// correctly rounded f32 division, split so that one denominator's reciprocal can serve several
// numerators.  The compiler's a/b (-fhip-fp32-correctly-rounded-divide-sqrt) is
//   b' = div_scale(b), a' = div_scale(a), r0 = rcp(b'), r = fma(fma(-b', r0, 1), r0, r0),
//   q = a'*r, q = fma(fma(-b', q, a'), r, q), q = div_fmas(fma(-b', q, a'), r, q), div_fixup(q, b, a).
// When neither div_scale scales (b and 1/b normal, a not tiny, exponent gap < 96, quotient normal)
// div_scale returns its operand, div_fmas is a plain fma and div_fixup returns q: rcp_ref + div_ref
// below are then that very instruction sequence minus the identities, i.e. bit-identical to a/b.
// Callers use them only where the operands of every lane whose result matters are in that range.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float rcp_ref(float b) {
  const float r0 = __builtin_amdgcn_rcpf(b);
  return __builtin_fmaf(__builtin_fmaf(-b, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ float div_ref(float a, float b, float r) {   // r = rcp_ref(b)
  float q = a * r;
  q = __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
  return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}
// |b| in [2^-60, 2^60]: 1/b by div_ref equals 1.0f/b (NaN and 0 fail the test)
__device__ __forceinline__ bool recip_safe(float b) {
  const float a = fabsf(b);
  return (a >= 8.67361737988403547206e-19f) & (a <= 1.15292150460684697600e+18f);
}

// sinf substitute (identical algorithm in the oracle: float rounding of a double sine)
__device__ __forceinline__ float rt_sinf(float xf) {
  double x = static_cast<double>(xf);
  if (!(fabs(x) < 1.0e6)) return static_cast<float>(sin(x));
  const double two_over_pi = 6.36619772367581382433e-01;
  const double p1 = 1.57079632673412561417e+00;
  const double p2 = 6.07710050630396597660e-11;
  const double p3 = 2.02226624871116645580e-21;
  double k = floor(x * two_over_pi + 0.5);
  double r = ((x - k * p1) - k * p2) - k * p3;
  long q = static_cast<long>(k) & 3;
  double r2 = r * r;
  double s = r + r * r2 * (-1.66666666666666666667e-01 + r2 * (8.33333333333333333333e-03 +
             r2 * (-1.98412698412698412698e-04 + r2 * (2.75573192239858906526e-06 +
             r2 * (-2.50521083854417187751e-08 + r2 * (1.60590438368216145994e-10 +
             r2 * (-7.64716373181981647590e-13 + r2 * 2.81145725434552076320e-15)))))));
  double c = 1.0 + r2 * (-0.5 + r2 * (4.16666666666666666667e-02 + r2 * (-1.38888888888888888889e-03 +
             r2 * (2.48015873015873015873e-05 + r2 * (-2.75573192239858906526e-07 +
             r2 * (2.08767569878680989792e-09 + r2 * (-1.14707455977297247139e-11 +
             r2 * 4.77947733238738529744e-14)))))));
  double res = (q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c;
  return static_cast<float>(res);
}

__device__ __forceinline__ float rt_pow5f(float xf) {   // powf(x, 5.0f) substitute
  double x = static_cast<double>(xf);
  double x2 = x * x;
  double x4 = x2 * x2;
  return static_cast<float>(x4 * x);
}

// acosf / atan2f substitutes (sphere_get_uv, :583-590; only image textures read u,v): the float
// rounding of a double evaluation built from + - * and float seeds only, so the oracle and the HIP
// kernel (device/rt_body.h, the same operations) produce identical bits.  atan on [0,1]: anchor
// c = k/8, r = (t - c)/(1 + t c) (|r| <= 1/16), odd Taylor series to r^15 (error < 3e-22).
__device__ constexpr double RT_ATAN_K8[9] = {0.0, 0.12435499454676144, 0.24497866312686414, 0.35877067027057225,
                                     0.4636476090008061, 0.5585993153435624, 0.6435011087932844,
                                     0.7188299996216245, 0.7853981633974483};
__device__ __forceinline__ double rt_recip_d(double x) {            /* 1/x, x in [2^-60, 2^60]: float seed + 2 Newton steps */
  double y = (double)(1.0f / (float)x);
  y = y * (2.0 - x * y);
  y = y * (2.0 - x * y);
  return y;
}
__device__ __forceinline__ double rt_atan01_d(double t) {           /* t in [0, 1] */
  int k = (int)(t * 8.0 + 0.5);
  double c = (double)k * 0.125;
  double r = (t - c) * rt_recip_d(1.0 + t * c);
  double r2 = r * r;
  double p = r * (1.0 + r2 * (-1.0 / 3.0 + r2 * (1.0 / 5.0 + r2 * (-1.0 / 7.0 + r2 * (1.0 / 9.0 +
             r2 * (-1.0 / 11.0 + r2 * (1.0 / 13.0 + r2 * (-1.0 / 15.0))))))));
  return RT_ATAN_K8[k] + p;
}
__device__ __forceinline__ double rt_atan2_d(double y, double x) {  /* finite, not both zero */
  const double pi = 3.141592653589793, half_pi = 1.5707963267948966;
  double ax = fabs(x), ay = fabs(y);
  double m = ax > ay ? ax : ay;
  if (m < 8.673617379884035e-19) { ax *= 1.2676506002282294e30; ay *= 1.2676506002282294e30; }   /* 2^-60, 2^100 */
  else if (m > 1.152921504606847e18) { ax *= 7.888609052210118e-31; ay *= 7.888609052210118e-31; } /* 2^60, 2^-100 */
  double a;
  if (ay <= ax) a = rt_atan01_d(ay * rt_recip_d(ax));
  else a = half_pi - rt_atan01_d(ax * rt_recip_d(ay));
  if (x < 0.0 || (x == 0.0 && __builtin_signbit(x))) a = pi - a;
  return __builtin_signbit(y) ? -a : a;
}
__device__ __forceinline__ float rt_atan2f(float yf, float xf) {
  const double pi = 3.141592653589793;
  if (__builtin_isnan(xf) || __builtin_isnan(yf)) return xf + yf;
  double x = (double)xf, y = (double)yf, r;
  if (x == 0.0 && y == 0.0) r = __builtin_signbit(x) ? pi : 0.0;
  else if (__builtin_isinf(xf) && __builtin_isinf(yf)) r = x > 0.0 ? 0.7853981633974483 : 2.356194490192345;
  else if (__builtin_isinf(xf)) r = x > 0.0 ? 0.0 : pi;
  else if (__builtin_isinf(yf)) r = 1.5707963267948966;
  else return (float)rt_atan2_d(y, x);
  return (float)(__builtin_signbit(y) ? -r : r);
}
__device__ __forceinline__ float rt_acosf(float xf) {
  if (!(fabsf(xf) <= 1.0f)) return (xf - xf) / (xf - xf);   /* NaN */
  double x = (double)xf;
  double s = (1.0 - x) * (1.0 + x);
  double q = 0.0;
  if (s > 0.0) {
    double r = (double)(1.0f / sqrtf((float)s));
    r = r * (1.5 - 0.5 * s * r * r);
    r = r * (1.5 - 0.5 * s * r * r);
    q = s * r;
  }
  if (q == 0.0) return xf > 0.0f ? 0.0f : 3.14159274101257324f;   /* acos(1) = 0, acos(-1) = pi */
  return (float)rt_atan2_d(q, x);
}

// ---------------------------------------------------------------------------------------------
// textures + Perlin (raytracing.cu:343-398, perlin_noise.cpp:1-46,72-85)
// ---------------------------------------------------------------------------------------------
template <bool LDS>
__device__ float perlin_noise(const Mem<LDS> &S, uint32_t tb, f3 p) {
  float fx = floorf(p.x), fy = floorf(p.y), fz = floorf(p.z);
  float u = p.x - fx, v = p.y - fy, w = p.z - fz;
  int32_t i = static_cast<int32_t>(fx), j = static_cast<int32_t>(fy), k = static_cast<int32_t>(fz);
  // perm_x[i & 255] and perm_x[(i + 1) & 255] from one u16 of the pair table
  const uint32_t pb = tb + kPerlinPerm2Word;
  const uint32_t qi = S.half(pb, i & 255), qj = S.half(pb, j & 255), qk = S.half(pb, k & 255);
  uint32_t pi0 = qi & 255u, pi1 = qi >> 8;
  uint32_t pj0 = qj & 255u, pj1 = qj >> 8;
  uint32_t pk0 = qk & 255u, pk1 = qk >> 8;
  float uu = u * u * (3 - 2 * u);
  float vv = v * v * (3 - 2 * v);
  float ww = w * w * (3 - 2 * w);
  // (a*uu + (1-a)*(1-uu)) is exactly uu or 1-uu for every finite uu (and NaN either way)
  float wu[2] = {1 - uu, uu}, wv[2] = {1 - vv, vv}, wwk[2] = {1 - ww, ww};
  float du[2] = {u, u - 1.0f}, dv[2] = {v, v - 1.0f}, dw[2] = {w, w - 1.0f};
  uint32_t pi[2] = {pi0, pi1}, pj[2] = {pj0, pj1}, pk[2] = {pk0, pk1};
  float accum = 0.0f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        uint32_t g = (pi[a] ^ pj[b] ^ pk[c]) & 255;
        uint4 gr = S.w4(tb + 4 * g);
        f3 grad = mk(asf(gr.x), asf(gr.y), asf(gr.z));
        accum += wu[a] * wv[b] * wwk[c] * dot(grad, mk(du[a], dv[b], dw[c]));
      }
  return accum;
}

// TM: texture kinds present (bit T_*); the dispatch keeps only those
template <bool LDS, bool COUNT, bool NOISE, bool UV, uint32_t TM = 0xfu>
__device__ f3 texture_color(const Mem<LDS> &S, const RenderArgs &A, uint32_t ti, float u, float v, f3 p,
                            uint32_t &perlin_count) {
  if (TM == (1u << T_SOLID)) {   // solid colours only: no dispatch
    const uint4 t0 = S.w4(A.off_texs + ti * kTexWords);
    return mk(asf(t0.y), asf(t0.z), asf(t0.w));
  }
  for (int guard = 0; guard < 64; ++guard) {
    const uint32_t b = A.off_texs + ti * kTexWords;
    uint4 t0 = S.w4(b);
    if (!(TM & (1u << T_CHECKER)) && !(TM & (1u << T_IMAGE)) && !(TM & (1u << T_NOISE)))
      return mk(asf(t0.y), asf(t0.z), asf(t0.w));
    switch (t0.x) {
      case T_SOLID:
        return mk(asf(t0.y), asf(t0.z), asf(t0.w));
      case T_CHECKER: {
        if (!(TM & (1u << T_CHECKER))) return mk(0, 0, 0);
        float inv = asf(t0.w);
        int32_t x = static_cast<int32_t>(floorf(inv * p.x));
        int32_t y = static_cast<int32_t>(floorf(inv * p.y));
        int32_t z = static_cast<int32_t>(floorf(inv * p.z));
        bool even = ((x + y + z) & 1) == 0;
        ti = even ? t0.y : t0.z;
      } break;
      case T_IMAGE: {
        if (!(TM & (1u << T_IMAGE))) return mk(0, 0, 0);
        if (!UV) return mk(1, 0, 1);        // no pixels anywhere in the scene (host-checked)
        uint4 t1 = S.w4(b + 4);
        if (t1.x == 0) return mk(1, 0, 1);
        int32_t wd = static_cast<int32_t>(t0.y), ht = static_cast<int32_t>(t0.z);
        float cu = (u < 0) ? 0 : ((u > 1) ? 1 : u);
        float cv = 1.0f - ((v < 0) ? 0 : ((v > 1) ? 1 : v));
        int32_t x = static_cast<int32_t>(cu * wd), y = static_cast<int32_t>(cv * ht);
        x = (x < 0) ? 0 : ((x > wd) ? wd : x);
        y = (y < 0) ? 0 : ((y > ht) ? ht : y);
        uint64_t wo = static_cast<uint64_t>(t0.w) + 3ull * (static_cast<uint64_t>(y) * wd + x);
        if (wo + 3 > A.pixel_words) return mk(0, 0, 0);
        uint32_t o = A.off_pixels + static_cast<uint32_t>(wo);
        return mk(S.f(o), S.f(o + 1), S.f(o + 2));
      }
      case T_NOISE: {
        if (!NOISE || !(TM & (1u << T_NOISE))) return mk(0, 0, 0);   // host selects a NOISE variant
        if (COUNT) perlin_count++;
        const uint32_t tb = A.off_perlin + t0.y * kPerlinWords;
        float accum = 0.0f, weight = 1.0f;
        f3 q = p;
        // unrolled: the octaves' table reads are independent, so their LDS latencies overlap (a
        // path trapped between the noise spheres runs alone on its SIMD at the end of the frame)
#ifndef RT_NOISE_UNROLL
#define RT_NOISE_UNROLL 7
#endif
#define RT_STR_(x) #x
#define RT_UNROLL_(n) _Pragma(RT_STR_(unroll n))
        RT_UNROLL_(RT_NOISE_UNROLL)
        for (int oct = 0; oct < 7; ++oct) {
          accum += weight * perlin_noise(S, tb, q);
          weight *= 0.5f;
          q = mk(q.x * 2, q.y * 2, q.z * 2);
        }
        float turb = fabsf(accum);
        float s = 1 + rt_sinf(asf(t0.w) * p.z + 10 * turb);
        return mk(0.5f * s, 0.5f * s, 0.5f * s);
      }
      default:
        return mk(0, 0, 0);
    }
  }
  return mk(0, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// compact colour stack (rt_layout.h kRcRecTag): a level holds a code of its attenuation
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rc_rec(uint32_t r, bool wide) { return wide ? (kRcRecTag | r) : r; }
// a wide code is a grey unless it is a record (exponent field all ones) or a texel (sign bit)
__device__ __forceinline__ bool rc_is_grey(uint32_t w) { return (w & kRcTexelTag) == 0 && (w & kRcRecTag) != kRcRecTag; }

// texture_color's resolution (checker recursion, image clamp, noise) returning the colour-stack code of
// the Lambertian attenuation instead of the colour: rc_decode(code) == texture_color(...) bit for bit
template <bool LDS, bool COUNT, bool NOISE, bool UV, uint32_t TM, bool WIDE>
__device__ uint32_t texture_code(const Mem<LDS> &S, const RenderArgs &A, uint32_t ti, float u, float v, f3 p,
                                 uint32_t &perlin_count) {
  if (TM == (1u << T_SOLID)) return rc_rec(A.rc_tex0 + ti, WIDE);   // solid colours only: no load
  for (int guard = 0; guard < 64; ++guard) {
    const uint32_t b = A.off_texs + ti * kTexWords;
    const uint4 t0 = S.w4(b);
    if (!(TM & (1u << T_CHECKER)) && !(TM & (1u << T_IMAGE)) && !(TM & (1u << T_NOISE)))
      return rc_rec(A.rc_tex0 + ti, WIDE);
    switch (t0.x) {
      case T_SOLID:
        return rc_rec(A.rc_tex0 + ti, WIDE);
      case T_CHECKER: {
        if (!(TM & (1u << T_CHECKER))) return rc_rec(A.rc_consts + RC_BLACK, WIDE);
        float inv = asf(t0.w);
        int32_t x = static_cast<int32_t>(floorf(inv * p.x));
        int32_t y = static_cast<int32_t>(floorf(inv * p.y));
        int32_t z = static_cast<int32_t>(floorf(inv * p.z));
        bool even = ((x + y + z) & 1) == 0;
        ti = even ? t0.y : t0.z;
      } break;
      case T_IMAGE: {
        if (!(TM & (1u << T_IMAGE))) return rc_rec(A.rc_consts + RC_BLACK, WIDE);
        if (!UV) return rc_rec(A.rc_consts + RC_MAGENTA, WIDE);   // no pixels anywhere (host-checked)
        uint4 t1 = S.w4(b + 4);
        if (t1.x == 0) return rc_rec(A.rc_consts + RC_MAGENTA, WIDE);
        int32_t wd = static_cast<int32_t>(t0.y), ht = static_cast<int32_t>(t0.z);
        float cu = (u < 0) ? 0 : ((u > 1) ? 1 : u);
        float cv = 1.0f - ((v < 0) ? 0 : ((v > 1) ? 1 : v));
        int32_t x = static_cast<int32_t>(cu * wd), y = static_cast<int32_t>(cv * ht);
        x = (x < 0) ? 0 : ((x > wd) ? wd : x);
        y = (y < 0) ? 0 : ((y > ht) ? ht : y);
        uint64_t wo = static_cast<uint64_t>(t0.w) + 3ull * (static_cast<uint64_t>(y) * wd + x);
        if (wo + 3 > A.pixel_words) return rc_rec(A.rc_consts + RC_BLACK, WIDE);
        return kRcTexelTag | static_cast<uint32_t>(wo);   // UV kernels are wide; pixel pool < 2^31 words
      }
      case T_NOISE: {
        if (!NOISE || !(TM & (1u << T_NOISE))) return rc_rec(A.rc_consts + RC_BLACK, WIDE);
        if (COUNT) perlin_count++;
#ifdef RT_DBG_CHEAP_NOISE   // timing experiment only (RT_JIT_OPTS): the paths do not depend on albedo
        return __float_as_uint(0.5f);
#endif
        const uint32_t tb = A.off_perlin + t0.y * kPerlinWords;
        float accum = 0.0f, weight = 1.0f;
        f3 q = p;
#pragma unroll
        for (int oct = 0; oct < 7; ++oct) {
          accum += weight * perlin_noise(S, tb, q);
          weight *= 0.5f;
          q = mk(q.x * 2, q.y * 2, q.z * 2);
        }
        float turb = fabsf(accum);
        float s = 1 + rt_sinf(asf(t0.w) * p.z + 10 * turb);
        const uint32_t g = __float_as_uint(0.5f * s);   // attenuation (g, g, g); NOISE kernels are wide
        return ((g & kRcRecTag) == kRcRecTag) ? (kRcRecTag | (A.rc_consts + RC_NAN)) : g;
      }
      default:
        return rc_rec(A.rc_consts + RC_BLACK, WIDE);
    }
  }
  return rc_rec(A.rc_consts + RC_BLACK, WIDE);
}

// code -> attenuation (the record's words 1..3, the texel, or the grey)
template <bool LDS, bool WIDE, bool NOISE, bool UV>
__device__ __forceinline__ f3 rc_decode(const Mem<LDS> &S, const RenderArgs &A, uint32_t w) {
  const bool grey = NOISE && rc_is_grey(w);   // a grey reads record 0 (in bounds), unused
  if (!WIDE || !UV) {
    const uint32_t r = grey ? 0u : (WIDE ? (w & kRcPayload) : w);
    const uint4 q = S.w4(A.off_mats + r * kRecWords);
    return grey ? mk(asf(w), asf(w), asf(w)) : mk(asf(q.y), asf(q.z), asf(q.w));
  }
  const bool texel = (w & kRcTexelTag) != 0;
  const uint32_t o = grey ? A.off_mats : (texel ? A.off_pixels + (w & kRcTexelPayload) : A.off_mats + (w & kRcPayload) * kRecWords + 1);
  const f3 c = mk(S.f(o), S.f(o + 1), S.f(o + 2));
  return grey ? mk(asf(w), asf(w), asf(w)) : c;
}

// a batch of codes: in kernels with noise textures the record loads are skipped when every code of the
// batch is a grey in every lane (wave-uniform test) — a deep path between noise surfaces is all greys
template <bool LDS, bool WIDE, bool NOISE, bool UV, int N>
__device__ __forceinline__ void rc_decode_batch(const Mem<LDS> &S, const RenderArgs &A, const uint32_t (&cw)[N],
                                                f3 (&at)[N]) {
  if (NOISE) {
    bool rec = false;
#pragma unroll
    for (int i = 0; i < N; ++i) rec |= !rc_is_grey(cw[i]);
    if (__ballot(rec) == 0) {
#pragma unroll
      for (int i = 0; i < N; ++i) at[i] = mk(asf(cw[i]), asf(cw[i]), asf(cw[i]));
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) at[i] = rc_decode<LDS, WIDE, NOISE, UV>(S, A, cw[i]);
}

// ---------------------------------------------------------------------------------------------
// traversal state and the per-node operations of hit() (raytracing.cu:1079-1251)
// ---------------------------------------------------------------------------------------------
struct Ray { f3 o, d; float time; };
// n is the OUTWARD normal and fd = dot(dir, n) at hit time; the face test (fd < 0) and the flip of
// hit_record_set_face_normal (:983-987) are applied when shading (hit_normal) — exact, because the
// y-rotation cleanup that may transform n in between is linear and odd (R(-n) == -R(n) bitwise)
struct Hit { f3 p, n; float t, u, v, fd; uint32_t mat; };
__device__ __forceinline__ bool hit_front(const Hit &h) { return h.fd < 0.0f; }
__device__ __forceinline__ f3 hit_normal(const Hit &h) { return hit_front(h) ? h.n : flip(h.n); }
struct Visits { uint32_t k[7]; uint32_t max_sp; uint32_t xn, xp; };   // xn / xp: executed SAH node visits / leaf tests

// Kernel arguments read where they are used: every render kernel takes RenderArgs as its only argument (kernarg
// offset 0), and a pointer to it whose provenance an empty asm hides makes each use a scalar load instead of a value
// the compiler holds in SGPRs across the render loop (held, the excess spilled into VGPR lanes: DESIGN §5f).
// RT_JIT_OPTS=-DRT_KARGS_HOLD restores the held form (A/B).
#ifndef RT_KARGS_HOLD
typedef const __attribute__((address_space(4))) RenderArgs *KArgsPtr;
__device__ __forceinline__ KArgsPtr kargs(const RenderArgs &) {
  KArgsPtr K = (KArgsPtr)(__builtin_amdgcn_kernarg_segment_ptr());
  asm volatile("" : "+s"(K));
  return K;
}
#else
__device__ __forceinline__ const RenderArgs *kargs(const RenderArgs &A) { return &A; }
#endif

// locals of hit() (:1082-1088) plus a cached 1/dir
struct Trav {
  f3 inv;          // 1/dir, refreshed whenever the ray direction changes (y-rotation enter/exit)
  f3 rcp;          // rcp_ref(dir) (scene-specialised folded traversal: shared by axis-aligned planes)
  float tmax;      // shrinking ray_tmax (closest hit so far)
  int sp;          // per-lane hit-stack depth (0 = traversal finished)
  int tc, yc;      // translation / y-rotation cleanup counters
  uint32_t was_last;   // 0/1 in a VGPR (a bool becomes per-join SALU lane-mask merges)
  // the walk's hit flag, 0/1 in a VGPR.  It outlives a round in a paused walk (the lane skips shading with `continue`
  // and resumes next round); held as a bool — a wave-wide lane mask merged with exec at every join — the 4-wide
  // verified walk built for 6 waves (80 VGPRs, SGPR spills into VGPR lanes) lost it for paused lanes and mis-rendered
  // random sphere worlds in some pixels, nondeterministically; as a word it is carried like the rest of the
  // paused state (round-5 diagnosis: DESIGN §2, profiles/r05_w4_diag.txt)
  uint32_t result;
  // verified traversal paused at the end of a round (resumed next round, shading skipped meanwhile)
  uint32_t active;     // 1 = walk in progress
  uint32_t anode, abest, atie;
  int asp;
};

__device__ __forceinline__ void trav_reset(Trav &T, const Ray &r) {
  T.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  T.tmax = __builtin_huge_valf();
  T.sp = 0;
  T.tc = 0; T.yc = 0;
  T.was_last = 0; T.result = false;
}

// 1/dir through the shared reciprocals (folded scene-specialised traversal); a lane with a tiny,
// zero or huge component takes the exact division (wave-uniform branch, normally never taken)
__device__ __forceinline__ void dir_rcp(Trav &T, const Ray &r) {
  T.rcp = mk(rcp_ref(r.d.x), rcp_ref(r.d.y), rcp_ref(r.d.z));
  T.inv = mk(div_ref(1.0f, r.d.x, T.rcp.x), div_ref(1.0f, r.d.y, T.rcp.y), div_ref(1.0f, r.d.z, T.rcp.z));
  const bool bad = !(recip_safe(r.d.x) && recip_safe(r.d.y) && recip_safe(r.d.z));
  if (__ballot(bad) != 0) {
    asm volatile("" ::: "memory");   // keep the exact divisions off the common path
    if (bad) T.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  }
}

// the same without 1/dir (scene-specialised traversal: computed lazily before box tests)
__device__ __forceinline__ void trav_reset_dir(Trav &T) {
  T.tmax = __builtin_huge_valf();
  T.sp = 0;
  T.tc = 0; T.yc = 0;
  T.was_last = 0; T.result = false;
}

// aabb_hit (:990-1025) with the cached 1/dir; the three early returns folded into one flag
__device__ __forceinline__ bool box_hit(const Trav &T, const Ray &r, float x0, float x1, float y0, float y1,
                                        float z0, float z1) {
  // t0 starts at tmin > 0 and MAX(t0, x) = (t0 < x) ? x : t0 never lets a NaN in, so t0 stays a
  // positive non-NaN and the ternary equals fmaxf (v_max_f32).  t1 keeps the ternary MIN: a NaN
  // slab value does replace it (utility.h:6).
  float t0 = kTmin, t1 = T.tmax;
  float a = (x0 - r.o.x) * T.inv.x, c = (x1 - r.o.x) * T.inv.x;
  if (T.inv.x < 0.0f && a > c) { float s = a; a = c; c = s; }
  t0 = fmaxf(t0, a); t1 = tmin_(t1, c);
  bool miss = t1 <= t0;
  a = (y0 - r.o.y) * T.inv.y; c = (y1 - r.o.y) * T.inv.y;
  if (T.inv.y < 0.0f && a > c) { float s = a; a = c; c = s; }
  t0 = fmaxf(t0, a); t1 = tmin_(t1, c);
  miss |= t1 <= t0;
  a = (z0 - r.o.z) * T.inv.z; c = (z1 - r.o.z) * T.inv.z;
  if (T.inv.z < 0.0f && a > c) { float s = a; a = c; c = s; }
  t0 = fmaxf(t0, a); t1 = tmin_(t1, c);
  miss |= t1 <= t0;
  return !miss;
}

// triangle / quad branch (:1131-1175) over geom_calc_hit (:1060-1077); in_xf: inside a transform
__device__ __forceinline__ void planar_hit(Trav &T, const Ray &r, Hit &h, bool tri, uint32_t mat, f3 n, float dd,
                                           f3 q, f3 uu, f3 vv, f3 ww, bool in_xf) {
  float denom = dot(n, r.d);
  if (fabsf(denom) >= kDenomEps) {
    float t = (dd - dot(n, r.o)) / denom;
    if (kTmin <= t && t <= T.tmax) {
      f3 p = line_at(r.o, t, r.d);
      f3 pq = sub(p, q);
      float alpha = dot(ww, cross(pq, vv));
      float beta = dot(ww, cross(uu, pq));
      // same predicate as (0 <= a && a <= 1) && (0 <= b && b <= 1) (NaN fails every compare), written
      // with non-short-circuit ands so it stays four compares on the lane mask
      bool inside = (0.0f <= alpha) & (alpha <= 1.0f) & (0.0f <= beta) & (beta <= 1.0f);
      if (tri) inside = inside & (alpha + beta <= 1.0f);
      if (inside) {
        h.u = alpha; h.v = beta; h.t = t; h.p = p; h.mat = mat;
        h.fd = dot(r.d, n);
        h.n = n;
        T.tmax = t;
        T.result = true;
        if (in_xf) T.was_last = 1;
      }
    }
  }
}

// sphere branch (:1093-1123) + sphere_get_uv (:583-590, image textures only)
template <bool UV>
__device__ __forceinline__ bool sphere_hit(Trav &T, const Ray &r, Hit &h, uint32_t mat, f3 c0, f3 mv, float rad2,
                                           float inv_rad, bool in_xf, bool need_uv = true) {
  bool acc = false;
  f3 center = line_at(c0, r.time, mv);
  f3 oc = sub(center, r.o);
  float a = dot(r.d, r.d);
  float b = -2.0f * dot(r.d, oc);
  float c = dot(oc, oc) - rad2;
  float disc = b * b - 4 * a * c;
  if (disc >= 0) {
    float sq = sqrtf(disc);
    float root = (-b - sq) / (2.0f * a);
    if (kTmin >= root || root >= T.tmax) root = (-b + sq) / (2.0f * a);
    if (kTmin < root && root < T.tmax) {
      h.t = root;
      h.p = line_at(r.o, root, r.d);
      h.mat = mat;
      f3 outward = scale(inv_rad, sub(h.p, center));
      if (UV && need_uv) {
        const float pi = 3.1415926535897932385f;
        float theta = rt_acosf(-outward.y);
        float phi = rt_atan2f(-outward.z, outward.x) + pi;
        h.u = phi / (2 * pi);
        h.v = theta / pi;
      }
      h.fd = dot(r.d, outward);
      h.n = outward;
      T.tmax = h.t;
      T.result = true;
      if (in_xf) T.was_last = 1;
      acc = true;
    }
  }
  return acc;
}

// sphere with a constant centre (scene_codegen.cpp folds c + mv*time when mv = +-0)
template <bool UV>
__device__ __forceinline__ void sphere_hit_static(Trav &T, const Ray &r, Hit &h, uint32_t mat, f3 center, float rad2,
                                                  float inv_rad, bool in_xf) {
  f3 oc = sub(center, r.o);
  float a = dot(r.d, r.d);
  float b = -2.0f * dot(r.d, oc);
  float c = dot(oc, oc) - rad2;
  float disc = b * b - 4 * a * c;
  if (disc >= 0) {
    float sq = sqrtf(disc);
    float root = (-b - sq) / (2.0f * a);
    if (kTmin >= root || root >= T.tmax) root = (-b + sq) / (2.0f * a);
    if (kTmin < root && root < T.tmax) {
      h.t = root;
      h.p = line_at(r.o, root, r.d);
      h.mat = mat;
      f3 outward = scale(inv_rad, sub(h.p, center));
      if (UV) {
        const float pi = 3.1415926535897932385f;
        float theta = rt_acosf(-outward.y);
        float phi = rt_atan2f(-outward.z, outward.x) + pi;
        h.u = phi / (2 * pi);
        h.v = theta / pi;
      }
      h.fd = dot(r.d, outward);
      h.n = outward;
      T.tmax = h.t;
      T.result = true;
      if (in_xf) T.was_last = 1;
    }
  }
}

// translation enter / cleanup (:1176-1191)
__device__ __forceinline__ void translate_enter(Trav &T, Ray &r, f3 off) {
  T.was_last = 0;
  r.o = sub(r.o, off);
}
__device__ __forceinline__ void translate_exit(Trav &T, Ray &r, Hit &h, f3 off) {
  r.o = add(r.o, off);
  if (T.was_last) h.p = add(h.p, off);
}

// y-rotation enter / cleanup (:1192-1237): the ray is rotated in place and back (ulp drift kept)
__device__ __forceinline__ void rotate_enter(Trav &T, Ray &r, float sn, float cs) {
  T.was_last = 0;
  const f3 o = r.o, d = r.d;
  r.o = mk((cs * o.x) - (sn * o.z), o.y, (sn * o.x) + (cs * o.z));
  r.d = mk((cs * d.x) - (sn * d.z), d.y, (sn * d.x) + (cs * d.z));
  T.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
}
__device__ __forceinline__ void rotate_exit(Trav &T, Ray &r, Hit &h, float sn, float cs) {
  const f3 o = r.o, d = r.d;
  r.o = mk((cs * o.x) + (sn * o.z), o.y, (-sn * o.x) + (cs * o.z));
  r.d = mk((cs * d.x) + (sn * d.z), d.y, (-sn * d.x) + (cs * d.z));
  T.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
  if (T.was_last) {
    const f3 p = h.p, n = h.n;
    h.p = mk((cs * p.x) + (sn * p.z), p.y, (-sn * p.x) + (cs * p.z));
    h.n = mk((cs * n.x) + (sn * n.z), n.y, (-sn * n.x) + (cs * n.z));
  }
}

// y-rotation enter / cleanup without the 1/dir refresh (scene-specialised traversal)
__device__ __forceinline__ void rotate_enter_dir(Trav &T, Ray &r, float sn, float cs) {
  T.was_last = 0;
  const f3 o = r.o, d = r.d;
  r.o = mk((cs * o.x) - (sn * o.z), o.y, (sn * o.x) + (cs * o.z));
  r.d = mk((cs * d.x) - (sn * d.z), d.y, (sn * d.x) + (cs * d.z));
}
__device__ __forceinline__ void rotate_exit_dir(Trav &T, Ray &r, Hit &h, float sn, float cs) {
  const f3 o = r.o, d = r.d;
  r.o = mk((cs * o.x) + (sn * o.z), o.y, (-sn * o.x) + (cs * o.z));
  r.d = mk((cs * d.x) + (sn * d.z), d.y, (-sn * d.x) + (cs * d.z));
  if (T.was_last) {
    const f3 p = h.p, n = h.n;
    h.p = mk((cs * p.x) + (sn * p.z), p.y, (-sn * p.x) + (cs * p.z));
    h.n = mk((cs * n.x) + (sn * n.z), n.y, (-sn * n.x) + (cs * n.z));
  }
}

// ---------------------------------------------------------------------------------------------
// traversal policy 1: per-lane DFS with a lane-interleaved LDS stack (any scene)
// ---------------------------------------------------------------------------------------------
// One iteration of hit()'s while loop (:1089-1249): pop one record and process it.
// KM: kinds that can occur in the scene (bit K_*); the run-time compiled lane kernels drop the others
// ALL: load the whole 80-B record at once (one memory latency per step instead of the kind word, then
// the rest: the main per-lane walk of large scenes); the verified walk's rare fallback keeps the
// two-step load, which needs fewer registers
// TRACK: an accepted sphere also leaves its record index in T.abest (| kBestRecord): the verified sphere walk's
// fallback, whose hit record is rebuilt at shading time (AccelTraceK::materialize)
constexpr uint32_t kBestRecord = 0x80000000u;
template <bool LDS, bool COUNT, bool UV, uint32_t KM = 0x7fu, bool ALL = true, bool TRACK = false>
__device__ __forceinline__ void trav_step(const Mem<LDS> &S, Trav &T, Ray &r, Hit &h, uint16_t *stk, Visits &vc) {
  int sp = T.sp - 1;
  const uint32_t idx = stk[sp * 64];
  const uint32_t nb = idx * kNodeWords;
  const uint4 w0 = S.w4(nb);
  uint4 w1, w2, w3, w4;
  if (ALL) { w1 = S.w4(nb + 4); w2 = S.w4(nb + 8); w3 = S.w4(nb + 12); w4 = S.w4(nb + 16); }
  const uint32_t kind = w0.x;
  if (COUNT) { vc.k[kind < 7 ? kind : 0]++; }
  const bool in_xf = T.tc || T.yc;
  if ((KM & (1u << K_BVH)) && kind == K_BVH) {                             // :1124-1130
    if (!ALL) w1 = S.w4(nb + 4);
    if (box_hit(T, r, asf(w0.z), asf(w0.w), asf(w1.x), asf(w1.y), asf(w1.z), asf(w1.w))) {
      stk[sp * 64] = static_cast<uint16_t>(w0.y >> 16);      // right
      stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);      // left (popped first)
      sp += 2;
    }
  } else if ((KM & ((1u << K_QUAD) | (1u << K_TRIANGLE))) && (kind == K_QUAD || kind == K_TRIANGLE)) {
    if (!ALL) { w1 = S.w4(nb + 4); w2 = S.w4(nb + 8); w3 = S.w4(nb + 12); w4 = S.w4(nb + 16); }
    planar_hit(T, r, h, kind == K_TRIANGLE, w0.y, mk(asf(w0.z), asf(w0.w), asf(w1.x)), asf(w1.y),
               mk(asf(w1.z), asf(w1.w), asf(w2.x)), mk(asf(w2.y), asf(w2.z), asf(w2.w)),
               mk(asf(w3.x), asf(w3.y), asf(w3.z)), mk(asf(w3.w), asf(w4.x), asf(w4.y)), in_xf);
  } else if ((KM & (1u << K_SPHERE)) && kind == K_SPHERE) {
    if (!ALL) { w1 = S.w4(nb + 4); w2 = S.w4(nb + 8); }
    if (sphere_hit<UV>(T, r, h, w0.y, mk(asf(w0.z), asf(w0.w), asf(w1.x)), mk(asf(w1.y), asf(w1.z), asf(w1.w)),
                       asf(w2.y), asf(w2.z), in_xf) && TRACK)
      T.abest = idx | kBestRecord;
  } else if ((KM & (1u << K_TRANSLATE)) && kind == K_TRANSLATE) {
    if (!ALL) w1 = S.w4(nb + 4);
    const f3 off = mk(asf(w0.z), asf(w0.w), asf(w1.x));
    if (T.tc == 0) {
      translate_enter(T, r, off);
      stk[sp * 64] = static_cast<uint16_t>(idx);
      stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);
      sp += 2;
      T.tc++;
    } else {
      T.tc--;
      translate_exit(T, r, h, off);
    }
  } else if ((KM & (1u << K_YROTATE)) && kind == K_YROTATE) {
    if (T.yc == 0) {
      rotate_enter(T, r, asf(w0.z), asf(w0.w));
      stk[sp * 64] = static_cast<uint16_t>(idx);
      stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);
      sp += 2;
      T.yc++;
    } else {
      T.yc--;
      rotate_exit(T, r, h, asf(w0.z), asf(w0.w));
    }
  } else if ((KM & (1u << K_GROUP)) && kind == K_GROUP) {               // :1238-1247
    const uint32_t first = w0.y, n = w0.z;
    for (uint32_t i = 0; i < n; ++i) stk[(sp + i) * 64] = static_cast<uint16_t>(first + i);
    sp += n;
  }
  if (COUNT && static_cast<uint32_t>(sp) > vc.max_sp) vc.max_sp = sp;
  T.sp = sp;
}

// PAUSE: the walk may stop at the end of a round with its state kept in T and the LDS stack (as in
// AccelTraceK: the round's walk ends once at most A.defer_trace lanes, <= 1/4 of the starters, are
// still walking after A.trace_min_iters steps); the walk resumes next round with shading skipped.
template <uint32_t KM, bool PAUSE = false, bool ALL = true, bool TRACK = false>
struct LaneTraceK {
  template <bool LDS, bool COUNT, bool UV>
  __device__ __forceinline__ static void run(const Mem<LDS> &S, const RenderArgs &A, bool busy, uint64_t, uint32_t,
                                             uint16_t *stk, Trav &T, Ray &r, Hit &h, Visits &vc) {
    if (!busy) return;
    if (!PAUSE || !T.active) {
      trav_reset(T, r);
      // the root through a scalar operand: under the verified walk's 80-VGPR budget the allocator otherwise kept this
      // uniform value in a VGPR and spilled it to scratch (round 5)
      uint32_t root = A.root;
      asm volatile("" : "+s"(root));
      stk[0] = static_cast<uint16_t>(root);
      T.sp = 1;
    }
    // the walk's share of the lane's stack: the verified sphere walk's fallback (TRACK) runs below its parked pixel sum
    [[maybe_unused]] const uint32_t cap = A.stack_cap - (TRACK ? kSumEntries : 0u);
    if (!PAUSE) {
      while (T.sp > 0) {
        trav_step<LDS, COUNT, UV, KM, ALL, TRACK>(S, T, r, h, stk, vc);
        if (!RT_CHECK(A, T.sp <= cap, CHK_LANE_STACK, T.sp, cap)) T.sp = 0;
      }
      return;
    }
    const uint32_t started = static_cast<uint32_t>(__popcll(__ballot(true)));
    for (uint32_t it = 1;; ++it) {
      if (T.sp > 0) {
        trav_step<LDS, COUNT, UV, KM, ALL>(S, T, r, h, stk, vc);
        if (!RT_CHECK(A, T.sp <= cap, CHK_LANE_STACK, T.sp, cap)) T.sp = 0;
      }
      const uint64_t left = __ballot(T.sp > 0);
      if (left == 0) break;
      const uint32_t nl = static_cast<uint32_t>(__popcll(left));
      if (it >= A.trace_min_iters && nl <= A.defer_trace && 4 * nl <= started) break;
    }
    T.active = T.sp > 0 ? 1u : 0u;
  }
};
using LaneTrace = LaneTraceK<0x7fu>;

// ---------------------------------------------------------------------------------------------
// traversal policy 4: verified sphere traversal (all-sphere worlds, sphere_accel.cpp)
// ---------------------------------------------------------------------------------------------
// For a world of spheres the record hit() returns does not depend on the order of the tests, only on
// which spheres the walk reaches: a sphere contributes its first root in (tmin, inf) and is accepted
// iff that root is below the running tmax (:1100-1110), so the closest-so-far only ever shrinks to
// the minimum over the reached spheres — unless two spheres yield the same root bitwise (then the
// first one tested wins).  The reference reaches a sphere iff the slab test (:990-1025) of every BVH
// ancestor passes with the tmax of that moment, which is >= the final t*.  Hence, for a ray, if
//   (1) a walk of ANY tree over the same spheres reaches every sphere the reference could accept
//       (conservative boxes, below), and finds the minimum t* at sphere P with no other root == t*,
//   (2) the reference's tests of P's BVH ancestors pass with tmax = t* (then with any larger tmax);
//       ancestors contain P's deepest ancestor box B exactly (unions of boxes, :571-580) and the
//       rounded slab values are monotone in the box bounds, so it suffices that the computed hit point
//       lies inside B with a margin that absorbs the rounding of the slab test,
// then the reference returns P's record at t*, and the record computed here from P and the same ray is
// bit-identical.  Rays failing (1)'s preconditions, with a tie, or failing (2) are re-traced with the
// reference's own walk (LaneTraceK).  Conservative boxes: a computed root can lie off the sphere —
// disc = b^2 - 4ac cancels — but within sqrt(r^2 + 32u|oc|^2) of the centre (u = 2^-24), i.e. within
// r + 2^-9 |oc| (|oc| <= |o|_1 + M, M bounding |centre| + r over a subtree); boxes are padded by that
// (slab test on the padded box, NaN-tolerant), so no sphere the reference could accept is culled.
// The box arrives padded by the subtree's share kAccelKappa * M; the ray's share kAccelKappa * |o|_1
// is added in t (pinv = that pad * |1/d| per axis).  Slab values by fma with oinv = o * (1/d): this
// test only has to be conservative, and its rounding (~u |o| in space) is far inside the padding.
// Per ray: which slab plane is the near one on each axis (sign of 1/d) and the t offsets with the ray's
// padding share folded in: near t = fma(x_near, 1/d, on), far t = fma(x_far, 1/d, of), on/of =
// -o/d -+ pad |1/d| (one more rounding of ~u |o/d|, again far inside the padding).
struct SlabRay {
  f3 on, of;
  bool nx, ny, nz;   // 1/d < 0: the near plane is the box's max
};
__device__ __forceinline__ SlabRay slab_ray(const Trav &T, f3 oinv, f3 pinv) {
  SlabRay s;
  s.on = mk(-oinv.x - pinv.x, -oinv.y - pinv.y, -oinv.z - pinv.z);
  s.of = mk(-oinv.x + pinv.x, -oinv.y + pinv.y, -oinv.z + pinv.z);
  s.nx = T.inv.x < 0.0f; s.ny = T.inv.y < 0.0f; s.nz = T.inv.z < 0.0f;
  return s;
}
__device__ __forceinline__ bool accel_box(const Trav &T, const SlabRay &R, float x0, float x1, float y0, float y1,
                                          float z0, float z1, float *tnear) {
  const float nx = __builtin_fmaf(R.nx ? x1 : x0, T.inv.x, R.on.x), fx = __builtin_fmaf(R.nx ? x0 : x1, T.inv.x, R.of.x);
  const float ny = __builtin_fmaf(R.ny ? y1 : y0, T.inv.y, R.on.y), fy = __builtin_fmaf(R.ny ? y0 : y1, T.inv.y, R.of.y);
  const float nz = __builtin_fmaf(R.nz ? z1 : z0, T.inv.z, R.on.z), fz = __builtin_fmaf(R.nz ? z0 : z1, T.inv.z, R.of.z);
  const float t0 = fmaxf(fmaxf(nx, ny), fmaxf(nz, kTmin)), t1 = fminf(fminf(fx, fy), fminf(fz, T.tmax));
  *tnear = t0;
  return !(t1 < t0);
}

// sphere branch of hit() with the record commit of sphere_hit<UV>; also reports a root equal to tmax.
// a = dot(d, d) and 2 * a are the same for every sphere of the walk (the ray is not transformed in an
// all-sphere world): computed once per ray by the caller, the same IEEE operations.
// FAST: the roots' division by 2a goes through the ray's reciprocal ra2 = rcp_ref(2a) (div_ref, exact
// when 2a is in [2^-40, 2^60]: the numerator -b -+ sqrt(disc) of a walkable ray is below 2^43 in
// magnitude, so the exponent gap stays < 96 and the quotient normal; a numerator too small for
// div_ref's preconditions gives a quotient below 2^-86, rejected as < tmin either way).
// The record of the accepted sphere is a function of (root, ray, sphere) only, so the walk commits it once
// after the last step (sphere_commit, from the closest sphere's index) instead of at every acceptance:
// the same operations on the same values, outside the loop.
template <bool UV>
__device__ __forceinline__ void sphere_commit(const Trav &T, const Ray &r, Hit &h, uint32_t mat, f3 c0, f3 mv, float inv_rad,
                                              bool need_uv = true) {
  const f3 center = line_at(c0, r.time, mv);
  h.t = T.tmax;
  h.p = line_at(r.o, h.t, r.d);
  h.mat = mat;
  f3 outward = scale(inv_rad, sub(h.p, center));
  if (UV && need_uv) {
    const float pi = 3.1415926535897932385f;
    float theta = rt_acosf(-outward.y);
    float phi = rt_atan2f(-outward.z, outward.x) + pi;
    h.u = phi / (2 * pi);
    h.v = theta / pi;
  }
  h.fd = dot(r.d, outward);
  h.n = outward;
}

template <bool UV, bool FAST, bool COMMIT = true>
__device__ __forceinline__ bool sphere_hit_tie(Trav &T, const Ray &r, Hit &h, uint32_t mat, f3 c0, f3 mv, float rad2,
                                               float inv_rad, float a2, float ra2, bool &tie) {
  f3 center = line_at(c0, r.time, mv);
  f3 oc = sub(center, r.o);
  float b = -2.0f * dot(r.d, oc);
  float c = dot(oc, oc) - rad2;
  float disc = b * b - (2.0f * a2) * c;   // 4 * a == 2 * (2 * a) exactly
  if (!(disc >= 0)) return false;
  float sq = sqrtf(disc);
  float root = FAST ? div_ref(-b - sq, a2, ra2) : (-b - sq) / a2;
  tie |= root == T.tmax;
  if (kTmin >= root || root >= T.tmax) {
    root = FAST ? div_ref(-b + sq, a2, ra2) : (-b + sq) / a2;
    tie |= root == T.tmax;
  }
  if (!(kTmin < root && root < T.tmax)) return false;
  if (!COMMIT) {
    T.tmax = root;
    T.result = true;
    return true;
  }
  h.t = root;
  h.p = line_at(r.o, root, r.d);
  h.mat = mat;
  f3 outward = scale(inv_rad, sub(h.p, center));
  if (UV) {
    const float pi = 3.1415926535897932385f;
    float theta = rt_acosf(-outward.y);
    float phi = rt_atan2f(-outward.z, outward.x) + pi;
    h.u = phi / (2 * pi);
    h.v = theta / pi;
  }
  h.fd = dot(r.d, outward);
  h.n = outward;
  T.tmax = h.t;
  T.result = true;
  return true;
}

// sort network on 4 keys (ascending)
__device__ __forceinline__ void sort4(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  uint32_t t;
  t = min(a, b); b = max(a, b); a = t;
  t = min(c, d); d = max(c, d); c = t;
  t = min(a, c); c = max(a, c); a = t;
  t = min(b, d); d = max(b, d); b = t;
  t = min(b, c); c = max(b, c); b = t;
}

// W4: the 4-wide form of the tree (rt_layout.h kAccel4*, accel::collapse_wide) — the same padded child boxes
// and leaves, about half the node steps (each testing four boxes): the nearest hit inner child is visited next,
// the others pushed far to near, the spheres of every hit leaf child tested in the step (one per-lane loop).
// Every sphere is culled by exactly the box the 2-wide walk would test for it, so the record, the tie flag and
// the reach proof are those of the 2-wide walk.
// Q: the quantised 4-wide nodes (rt_layout.h kAccel4Q*, accel::quantize_wide): one 64-B line per node, the planes
// as bytes over a per-axis origin and power-of-two step; plane t = fma(q, 2^e / d, fma(o, 1/d, on)) — the boxes
// contain the float ones widened for this evaluation's rounding, so the culling stays conservative (any tree
// that reaches every sphere the reference could accept gives the same record: the verified walk above).
template <uint32_t KM, bool W4 = false, bool Q = false>
struct AccelTraceK {
  template <bool LDS, bool COUNT, bool UV>
  __device__ __forceinline__ static void run(const Mem<LDS> &S, const RenderArgs &A, bool busy, uint64_t lanes,
                                             uint32_t lane, uint16_t *stk, Trav &T, Ray &r, Hit &h, Visits &vc) {
    if (!busy) return;
    const bool resume = T.active != 0;
    if (!resume) trav_reset(T, r);
    const float ao = fabsf(r.o.x) + fabsf(r.o.y) + fabsf(r.o.z);
    const float dmin = fminf(fminf(fabsf(r.d.x), fabsf(r.d.y)), fabsf(r.d.z));
    const float dmax = fmaxf(fmaxf(fabsf(r.d.x), fabsf(r.d.y)), fabsf(r.d.z));
    // bounded, finite rays with no tiny direction component (finite 1/dir); the counting variant
    // walks the reference tree so that the op model counts the reference's visits
    // (and 2|d|^2 >= 2^-40, so that the roots' division by 2a can use the ray's reciprocal, sphere_hit_tie)
    // (and max |d_i| >= 7e-7, so 2|d|^2 >= 2^-40 and the roots' division by 2a can use the ray's
    // reciprocal, sphere_hit_tie)
    // The counting variant runs the walk on copies (never pausing) only to count its executed node visits
    // and leaf tests (vc.xn / vc.xp: the op model's second, executed-work frac), then walks the
    // reference tree for the record so that the op model also counts the reference's visits.
    bool nice = (ao <= 1.0e6f) && (dmin >= 1.0e-20f) && (dmax <= 1.0e6f) && (dmax >= 7.0e-7f);
    const Trav tsave = T;
    const Hit hsave = h;
    bool tie = resume && (T.anode >> 31) != 0;
    uint32_t best = resume ? T.abest : 0u;
    const uint4 *N = reinterpret_cast<const uint4 *>(A.scene + (W4 ? A.accel_wide : A.accel_nodes));
    const uint4 *P = reinterpret_cast<const uint4 *>(A.scene + A.accel_prims);
    bool walking = nice;
    if (nice) {
      const float pad_o = kAccelKappa * ao;
      const f3 oinv = mk(r.o.x * T.inv.x, r.o.y * T.inv.y, r.o.z * T.inv.z);
      const f3 pinv = mk(pad_o * fabsf(T.inv.x), pad_o * fabsf(T.inv.y), pad_o * fabsf(T.inv.z));
      const SlabRay sr = slab_ray(T, oinv, pinv);
      const float sa2 = 2.0f * dot(r.d, r.d);   // sphere_hit_tie's per-ray terms
      const float sra2 = rcp_ref(sa2);
      uint32_t node = resume ? (T.anode & 0xffffu) : (W4 ? 0u : A.accel_root);
      int sp = resume ? static_cast<int>((T.anode >> 16) & 0x7fffu) : 0;
      // Wave-uniform loop, one node per walking lane per step.  Rays differ wildly in length (the
      // horizon of a sphere field vs a close hit), so instead of every lane waiting for the longest
      // walk, the round's walk ends once few lanes remain (A.defer_trace, after A.trace_min_iters
      // steps); those lanes keep node, stack and best hit and resume next round, skipping shading
      // meanwhile.  A walk's steps and order are unchanged, so the record is the same.
      // A camera ray of a tile with a candidate list (RenderArgs::prim_lists, T.atie = tile + 1): the list's spheres
      // in ascending order of their axial lower bound instead of the walk — any set of spheres holding every one
      // the ray could accept gives the same record ((1) above), and a sphere whose lower bound lies beyond the
      // ray's axial reach below tmax (|o - centre| + tmax |d|, rounded up) cannot yield a root below tmax, nor
      // can any later one; the reach proof and the fallback below apply unchanged
      if (RT_PRIM_LISTS && !resume && T.atie != 0u) {
        const uint32_t tile = T.atie - 1u;
        const uint32_t n = A.prim_counts[tile];
        const uint32_t cap = A.prim_cap;
        if (n <= cap) {
          walking = false;
          const float dl = sqrtf(dot(r.d, r.d));
          const float rho = A.prim_rho;
          // 8-B entries (SAH prim index, axial bound); the sphere's centre, motion and r^2 from the tree's prims (the
          // walk's own leaf words, L2-resident): entry k+1 is loaded under entry k's test (32-B entries with the
          // sphere inline evicted the frame's lines from L2 before their tiles had filled them: twice the memory
          // writes)
          const uint2 *L = reinterpret_cast<const uint2 *>(A.prim_lists) + static_cast<size_t>(tile) * cap;
#ifdef RT_NT_LISTS   // A/B (RT_JIT_OPTS=-DRT_NT_LISTS): list entries read with the non-temporal hint (L2 streaming)
          auto entry = [&](uint32_t k) -> uint2 {
            const unsigned long long v = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long *>(L + k));
            return make_uint2(static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32));
          };
#else
          auto entry = [&](uint32_t k) -> uint2 { return L[k]; };
#endif
          uint2 c1 = n > 0 ? entry(0) : make_uint2(0, 0);
          for (uint32_t k = 0; k < n; ++k) {
            const uint2 c = c1;
            if (__uint_as_float(c.y) > __builtin_fmaf(T.tmax, dl, rho) * 1.0000010f) break;
            const uint4 a0 = P[c.x * 4], a1 = P[c.x * 4 + 1];
            if (k + 1 < n) c1 = entry(k + 1);
            if (COUNT) vc.xp++;
            if (sphere_hit_tie<UV, true, false>(T, r, h, 0u, mk(asf(a0.x), asf(a0.y), asf(a0.z)),
                                                mk(asf(a0.w), asf(a1.x), asf(a1.y)), asf(a1.z), 0.0f, sa2, sra2, tie))
              best = c.x;
          }
        }
      }
      const uint32_t started = static_cast<uint32_t>(__popcll(__ballot(walking)));
      // the top of the tree from LDS (A.accel_lds_nodes breadth-first nodes), the rest from HBM / L2
      // (two explicit loads rather than one generic pointer: flat loads would wait on both counters)
      uint4 q0, q1, q2, q3;
      auto load_node = [&](uint32_t nd) {
        if (nd < A.accel_lds_nodes) {
          const uint4 *L = reinterpret_cast<const uint4 *>(g_lds);
          q0 = L[nd * 4]; q1 = L[nd * 4 + 1]; q2 = L[nd * 4 + 2]; q3 = L[nd * 4 + 3];
        } else {
          q0 = N[nd * 4]; q1 = N[nd * 4 + 1]; q2 = N[nd * 4 + 2]; q3 = N[nd * 4 + 3];
        }
      };
      for (uint32_t it = 1;; ++it) {
        if (W4 && walking) {
          // planes x0 x1 y0 y1 z0 z1 of the four children and their refs, 16 B each, from one base address with
          // immediate offsets (LDS for the staged top of the tree, else global: two explicit loads, not a flat one)
          // (address-space-typed pointers: merged into one generic pointer, the two paths become flat loads)
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          constexpr int NV = Q ? 4 : 7, NS = Q ? 4 : 8;
          u32x4 v[NV];
          if (node < A.accel_lds_nodes) {
            const __attribute__((address_space(3))) u32x4 *L =
                (const __attribute__((address_space(3))) u32x4 *)(static_cast<uintptr_t>(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(g_lds)))) + node * NS;
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] = L[k];
          } else {
            const __attribute__((address_space(1))) u32x4 *G =
                (const __attribute__((address_space(1))) u32x4 *)(reinterpret_cast<uintptr_t>(N)) + node * NS;
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] = G[k];
          }
          if (COUNT) vc.xn += 2;   // four boxes: two 2-wide steps' worth (the op model's per-step weight)
          uint32_t key[4], cnt[4], rr[4];
          if constexpr (Q) {
            // per axis: scale 2^e / d and the offsets fma(o, 1/d, on / of); near / far plane bytes by the octant
            const uint32_t meta = v[0].w;
            const float sx = __builtin_amdgcn_ldexpf(T.inv.x, static_cast<int>(meta & 0xffu) - 127);
            const float sy = __builtin_amdgcn_ldexpf(T.inv.y, static_cast<int>((meta >> 8) & 0xffu) - 127);
            const float sz = __builtin_amdgcn_ldexpf(T.inv.z, static_cast<int>((meta >> 16) & 0xffu) - 127);
            const float bnx = __builtin_fmaf(asf(v[0].x), T.inv.x, sr.on.x), bfx = __builtin_fmaf(asf(v[0].x), T.inv.x, sr.of.x);
            const float bny = __builtin_fmaf(asf(v[0].y), T.inv.y, sr.on.y), bfy = __builtin_fmaf(asf(v[0].y), T.inv.y, sr.of.y);
            const float bnz = __builtin_fmaf(asf(v[0].z), T.inv.z, sr.on.z), bfz = __builtin_fmaf(asf(v[0].z), T.inv.z, sr.of.z);
            const uint32_t xn = sr.nx ? v[1].y : v[1].x, xf = sr.nx ? v[1].x : v[1].y;
            const uint32_t yn = sr.ny ? v[1].w : v[1].z, yf = sr.ny ? v[1].z : v[1].w;
            const uint32_t zn = sr.nz ? v[2].y : v[2].x, zf = sr.nz ? v[2].x : v[2].y;
            rr[0] = v[2].z; rr[1] = v[2].w; rr[2] = v[3].x; rr[3] = v[3].y;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float tnx = __builtin_fmaf(static_cast<float>((xn >> (8 * c)) & 0xffu), sx, bnx);
              const float tfx = __builtin_fmaf(static_cast<float>((xf >> (8 * c)) & 0xffu), sx, bfx);
              const float tny = __builtin_fmaf(static_cast<float>((yn >> (8 * c)) & 0xffu), sy, bny);
              const float tfy = __builtin_fmaf(static_cast<float>((yf >> (8 * c)) & 0xffu), sy, bfy);
              const float tnz = __builtin_fmaf(static_cast<float>((zn >> (8 * c)) & 0xffu), sz, bnz);
              const float tfz = __builtin_fmaf(static_cast<float>((zf >> (8 * c)) & 0xffu), sz, bfz);
              const float t0 = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, kTmin)), t1 = fminf(fminf(tfx, tfy), fminf(tfz, T.tmax));
              const bool hit = !(t1 < t0) && ((meta >> (24 + c)) & 1u);
              const bool leaf = (rr[c] & kAccelLeaf) != 0;
              key[c] = (hit && !leaf) ? ((__float_as_uint(t0) & 0xffff0000u) | rr[c]) : 0xffffffffu;
              cnt[c] = (hit && leaf) ? ((rr[c] >> 24) & 0x7fu) + 1u : 0u;
            }
          } else {
          const uint4 X0 = make_uint4(v[0].x, v[0].y, v[0].z, v[0].w), X1 = make_uint4(v[1].x, v[1].y, v[1].z, v[1].w);
          const uint4 Y0 = make_uint4(v[2].x, v[2].y, v[2].z, v[2].w), Y1 = make_uint4(v[3].x, v[3].y, v[3].z, v[3].w);
          const uint4 Z0 = make_uint4(v[4].x, v[4].y, v[4].z, v[4].w), Z1 = make_uint4(v[5].x, v[5].y, v[5].z, v[5].w);
          const uint4 R4 = make_uint4(v[NV - 1].x, v[NV - 1].y, v[NV - 1].z, v[NV - 1].w);
          // near / far plane per axis by the ray's octant (the near plane is the max one when 1/d < 0)
          const uint4 XN = sr.nx ? X1 : X0, XF = sr.nx ? X0 : X1, YN = sr.ny ? Y1 : Y0, YF = sr.ny ? Y0 : Y1;
          const uint4 ZN = sr.nz ? Z1 : Z0, ZF = sr.nz ? Z0 : Z1;
          const uint32_t xn[4] = {XN.x, XN.y, XN.z, XN.w}, xf[4] = {XF.x, XF.y, XF.z, XF.w};
          const uint32_t yn[4] = {YN.x, YN.y, YN.z, YN.w}, yf[4] = {YF.x, YF.y, YF.z, YF.w};
          const uint32_t zn[4] = {ZN.x, ZN.y, ZN.z, ZN.w}, zf[4] = {ZF.x, ZF.y, ZF.z, ZF.w};
          rr[0] = R4.x; rr[1] = R4.y; rr[2] = R4.z; rr[3] = R4.w;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            // accel_box with the planes already in near / far order
            const float tnx = __builtin_fmaf(asf(xn[c]), T.inv.x, sr.on.x), tfx = __builtin_fmaf(asf(xf[c]), T.inv.x, sr.of.x);
            const float tny = __builtin_fmaf(asf(yn[c]), T.inv.y, sr.on.y), tfy = __builtin_fmaf(asf(yf[c]), T.inv.y, sr.of.y);
            const float tnz = __builtin_fmaf(asf(zn[c]), T.inv.z, sr.on.z), tfz = __builtin_fmaf(asf(zf[c]), T.inv.z, sr.of.z);
            const float t0 = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, kTmin)), t1 = fminf(fminf(tfx, tfy), fminf(tfz, T.tmax));
            const bool hit = !(t1 < t0);
            const bool leaf = (rr[c] & kAccelLeaf) != 0;
            // inner children: sortable key = the entry t's high bits (t >= tmin > 0: monotone as an integer)
            // with the node index in the low 16 bits (only the visit order depends on the truncation)
            key[c] = (hit && !leaf) ? ((__float_as_uint(t0) & 0xffff0000u) | rr[c]) : 0xffffffffu;
            cnt[c] = (hit && leaf) ? ((rr[c] >> 24) & 0x7fu) + 1u : 0u;
          }
          }
          // the hit leaves' spheres, in one per-lane loop below: sphere k of the concatenated ranges
          const uint32_t p1 = cnt[0], p2 = p1 + cnt[1], p3 = p2 + cnt[2], tot = p3 + cnt[3];
          const uint32_t b0 = rr[0] & 0xffffffu, b1 = (rr[1] & 0xffffffu) - p1, b2 = (rr[2] & 0xffffffu) - p2,
                         b3 = (rr[3] & 0xffffffu) - p3;
          // next node first (the order does not depend on the leaves): the nearest hit inner child, the others
          // pushed far to near (the nearest of them on top); none: pop
          sort4(key[0], key[1], key[2], key[3]);
          if (key[0] != 0xffffffffu) {
            const int n_in = 1 + (key[1] != 0xffffffffu) + (key[2] != 0xffffffffu) + (key[3] != 0xffffffffu);
            if (n_in >= 4) stk[(sp + n_in - 4) * 64] = static_cast<uint16_t>(key[3]);
            if (n_in >= 3) stk[(sp + n_in - 3) * 64] = static_cast<uint16_t>(key[2]);
            if (n_in >= 2) stk[(sp + n_in - 2) * 64] = static_cast<uint16_t>(key[1]);
            sp += n_in - 1;
            if (!RT_CHECK(A, static_cast<uint32_t>(sp) <= A.stack_cap - kSumEntries, CHK_ACCEL_STACK, sp, A.stack_cap - kSumEntries)) sp = 0;
            node = key[0] & 0xffffu;
          } else if (sp == 0) {
            walking = false;
          } else {
            --sp;
            node = stk[sp * 64];
          }
          for (uint32_t k = 0; k < tot; ++k) {
            const uint32_t pr = (k < p1 ? b0 : (k < p2 ? b1 : (k < p3 ? b2 : b3))) + k;
            if (COUNT) vc.xp++;
            const uint4 p0 = P[pr * 4], pw1 = P[pr * 4 + 1], pw2 = P[pr * 4 + 2];
            if (sphere_hit_tie<UV, true, false>(T, r, h, pw2.x, mk(asf(p0.x), asf(p0.y), asf(p0.z)),
                                                mk(asf(p0.w), asf(pw1.x), asf(pw1.y)), asf(pw1.z), asf(pw1.w), sa2, sra2, tie))
              best = pr;
          }
        }
        if (!W4 && walking) {
        load_node(node);
        if (COUNT) vc.xn++;
        float n0, n1;
        bool h0 = accel_box(T, sr, asf(q0.x), asf(q0.y), asf(q0.z), asf(q0.w), asf(q1.x), asf(q1.y), &n0);
        bool h1 = accel_box(T, sr, asf(q1.z), asf(q1.w), asf(q2.x), asf(q2.y), asf(q2.z), asf(q2.w), &n1);
        const bool near0 = n0 <= n1;
        const uint32_t rn = near0 ? q3.x : q3.y, rf = near0 ? q3.y : q3.x;
        bool hn = near0 ? h0 : h1, hf = near0 ? h1 : h0;
        // the hit leaves' spheres, near leaf first, in ONE per-lane loop (the wave runs the longest
        // lane's count once, not the near and the far leaf's maxima one after the other)
        const bool ln = hn && (rn & kAccelLeaf), lf = hf && (rf & kAccelLeaf);
        const uint32_t c1 = ln ? ((rn >> 24) & 0x7fu) + 1u : 0u, c2 = lf ? ((rf >> 24) & 0x7fu) + 1u : 0u;
        const uint32_t f1 = rn & 0xffffffu, f2 = (rf & 0xffffffu) - c1;
        for (uint32_t k = 0; k < c1 + c2; ++k) {
          const uint32_t pr = (k < c1 ? f1 : f2) + k;
          if (COUNT) vc.xp++;
          const uint4 p0 = P[pr * 4], p1 = P[pr * 4 + 1], p2 = P[pr * 4 + 2];
          if (sphere_hit_tie<UV, true, false>(T, r, h, p2.x, mk(asf(p0.x), asf(p0.y), asf(p0.z)), mk(asf(p0.w), asf(p1.x), asf(p1.y)),
                                       asf(p1.z), asf(p1.w), sa2, sra2, tie))
            best = pr;
        }
        hn = hn && !ln;
        hf = hf && !lf;
        if (hn && hf) {
          stk[sp * 64] = static_cast<uint16_t>(rf);
          ++sp;
          if (!RT_CHECK(A, static_cast<uint32_t>(sp) <= A.stack_cap - kSumEntries, CHK_ACCEL_STACK, sp, A.stack_cap - kSumEntries)) sp = 0;
          node = rn;
        } else if (hn | hf) {
          node = hn ? rn : rf;
        } else if (sp == 0) {
          walking = false;
        } else {
          --sp;
          node = stk[sp * 64];
        }
        }
        const uint64_t left = __ballot(walking);
        if (left == 0) break;
        const uint32_t nl = static_cast<uint32_t>(__popcll(left));
        if (!COUNT && it >= A.trace_min_iters && nl <= A.defer_trace && 4 * nl <= started) break;
      }
      if (walking) {   // paused: resume next round
        // one VGPR for node (< 2^16, u16 stack entries), depth and the tie flag
        T.active = 1; T.anode = node | (static_cast<uint32_t>(sp) << 16) | (tie ? 0x80000000u : 0u); T.abest = best;
        return;
      }
    }
    T.active = 0;
    if (COUNT) {   // counted; the record comes from the reference walk below
      T = tsave;
      h = hsave;
      nice = false;
    }
    bool need_ref = !nice || tie;
    T.abest = best;   // the record is rebuilt from it at shading time (materialize)
    if (nice && T.result) {
      // (2): the hit point (sphere_commit's: line_at(o, t, d)) inside P's deepest reference BVH ancestor box with
      // a margin of 2^-19 of the magnitudes the slab test and the hit point round (|o|, |p|, |t d| per axis):
      // the reference's slab values err by <= 3u |x - o| and p by <= 2u (|o| + |t d|), u = 2^-24
      const float t = T.tmax;
      const f3 hp = line_at(r.o, t, r.d);
      const uint4 b0 = P[best * 4 + 2], b1 = P[best * 4 + 3];
      const float bx0 = asf(b0.z), bx1 = asf(b0.w), by0 = asf(b1.x), by1 = asf(b1.y), bz0 = asf(b1.z), bz1 = asf(b1.w);
      const float m = 1.9073486328125e-06f;   // 2^-19
      const float dx = m * (fabsf(r.o.x) + fabsf(hp.x) + fabsf(t * r.d.x)) + 1.0e-30f;
      const float dy = m * (fabsf(r.o.y) + fabsf(hp.y) + fabsf(t * r.d.y)) + 1.0e-30f;
      const float dz = m * (fabsf(r.o.z) + fabsf(hp.z) + fabsf(t * r.d.z)) + 1.0e-30f;
      const bool inside = (hp.x - bx0 >= dx) & (bx1 - hp.x >= dx) & (hp.y - by0 >= dy) & (by1 - hp.y >= dy) &
                          (hp.z - bz0 >= dz) & (bz1 - hp.z >= dz);
      need_ref |= !inside;
    }
    const uint64_t fb = __ballot(need_ref);
    if (fb != 0) {   // rare: the reference walk for those lanes (it leaves the accepted record's index in T.abest)
      asm volatile("" ::: "memory");
      if (!COUNT && lane == static_cast<uint32_t>(__builtin_ctzll(fb))) atomicAdd(A.accel_fallbacks, static_cast<uint32_t>(__popcll(fb)));
      LaneTraceK<KM, false, false, true>::template run<LDS, COUNT, UV>(S, A, need_ref, lanes, lane, stk, T, r, h, vc);
    }
  }

  // The hit record, rebuilt at shading time from (T.abest, T.tmax, the ray) for EVERY lane (values of lanes
  // without a hit are never read): the record of a sphere hit is a function of the sphere, the root and the ray
  // only (sphere_commit performs sphere_hit's record operations, :1093-1123), so the walk keeps two words per
  // lane instead of the record, and no record is carried across the walk or across rounds (a lane resuming its
  // rejection sampling rebuilds the same record from the same words).  T.abest: a SAH prim, or | kBestRecord a
  // reference record (the fallback walk's hit).
  static constexpr bool kLazyHit = true;
  static constexpr bool kPrimLists = true;   // camera rays may take their tile's candidate list (T.atie)
  // random_test (drawn before the scatter's rejection, read by a dielectric after it) waits in the lane's traversal
  // stack (dead from the end of the walk to the next trace) instead of a register: at this kernel's 80-VGPR budget the
  // allocator otherwise spilled it to scratch once per bounce (scratch stores reach HBM: 10k config)
  static constexpr bool kParkRandomTest = true;
  // the pixel's running sum (used once per sample) waits in the kSumEntries top entries of the lane's stack, above the
  // walk's (the host adds them to stack_cap): three registers fewer across the walk, which then fits 80 VGPRs (6 waves)
  // without spilling (round 5: default builds never spill VGPRs)
  static constexpr bool kParkSum = true;
  template <bool LDS, bool UV>
  __device__ __forceinline__ static void materialize(const Mem<LDS> &S, const RenderArgs &A, const Trav &T, const Ray &r,
                                                     Hit &h) {
    const uint32_t b = T.abest;
    uint4 w0, w1, w2;
    uint32_t mat;
    float inv_rad;
    if (b & kBestRecord) {   // reference record: w1 material, w2..4 centre, w5..7 motion, w10 1/r
      const uint32_t nb = (b & 0xffffu) * kNodeWords;
      w0 = S.w4(nb); w1 = S.w4(nb + 4); w2 = S.w4(nb + 8);
      mat = w0.y;
      inv_rad = asf(w2.z);
      w0 = make_uint4(w0.z, w0.w, w1.x, w1.y);   // centre x y z, motion x
      w1 = make_uint4(w1.z, w1.w, 0u, 0u);       // motion y z
    } else {                  // SAH prim: centre 0..2, motion 3..5, 1/r 7, material 8
      const uint4 *P = reinterpret_cast<const uint4 *>(A.scene + A.accel_prims) + b * 4;
      w0 = P[0]; w2 = P[1];
      const uint4 w3 = P[2];
      mat = w3.x;
      inv_rad = asf(w2.w);
      w1 = make_uint4(w2.x, w2.y, 0u, 0u);
    }
    sphere_commit<UV>(T, r, h, mat, mk(asf(w0.x), asf(w0.y), asf(w0.z)), mk(asf(w0.w), asf(w1.x), asf(w1.y)),
                      inv_rad, T.result);
  }
};

// Traces whose hit record is rebuilt at shading time (kLazyHit) — detected without <type_traits> (hipRTC)
template <class TR> __device__ constexpr auto lazy_hit(int) -> decltype(TR::kLazyHit, bool()) { return TR::kLazyHit; }
template <class TR> __device__ constexpr bool lazy_hit(long) { return false; }
template <class TR> __device__ constexpr auto carry_point(int) -> decltype(TR::kCarryPoint, bool()) { return TR::kCarryPoint; }
template <class TR> __device__ constexpr bool carry_point(long) { return false; }
template <class TR> __device__ constexpr auto prim_lists(int) -> decltype(TR::kPrimLists, bool()) { return TR::kPrimLists; }
template <class TR> __device__ constexpr bool prim_lists(long) { return false; }
template <class TR> __device__ constexpr auto park_random_test(int) -> decltype(TR::kParkRandomTest, bool()) { return TR::kParkRandomTest; }
template <class TR> __device__ constexpr bool park_random_test(long) { return false; }
template <class TR> __device__ constexpr auto park_sum(int) -> decltype(TR::kParkSum, bool()) { return TR::kParkSum; }
template <class TR> __device__ constexpr bool park_sum(long) { return false; }

// ---------------------------------------------------------------------------------------------
// traversal policy 5: verified traversal of mixed worlds (mixed_accel.cpp)
// ---------------------------------------------------------------------------------------------
// The reference's own DFS (LaneTrace) above the macro roots — transforms, their in-place ray drift and
// the visit order included — and, at a macro root whose box test passes (W_MACRO), one SAH walk over its
// transform-free primitives instead of the reference's walk of that subtree.  Inside a macro the ray is
// never modified (static macro: no transform below; dynamic macro: entered only when the reference's
// slab test on W_XFBOX, the union of the boxes of the BVH nodes with a transform child below, fails —
// those nodes then fail too at their visit: smaller box, smaller tmax, same ray, and the rounded slab
// values are monotone in the bounds for finite 1/dir).  So the subtree's effect on the record is that of
// its closest acceptable primitive the reference reaches, unless two candidates tie.  Per primitive the
// candidate value v does not depend on tmax (sphere: the root hit() would accept for any tmax > v;
// quad / triangle: the plane t when the point is inside), and the reference accepts it iff v < tmax
// (sphere) or v <= tmax (quad, triangle: :1066).  The walk keeps
//   best    the smallest v below min(best, tmax_in), with its deepest reference BVH ancestor A below the
//           macro root (its "group": every primitive under that node shares it),
//   tie     a second candidate equal to the final min(best, tmax_in) (the reference's order would decide
//           which one it keeps; equal candidates above the final value are all replaced by it),
//   second  a lower bound on v over the primitives outside best's group (pruning bound included),
// and proves reach: the reference visits A with the tmax of that moment, T_A = min(tmax_in, v of the
// primitives it accepted before A), all outside A's subtree, so T_A >= lb = min(tmax_in, second, bound);
// the reference's own slab test of A with tmax = lb passing implies it passes at T_A, and then every
// ancestor of A passes too (their boxes contain A's, their tmax is larger).  A ray that fails a check
// (tie, reach, or a non-finite / unbounded ray) takes the reference's walk of that subtree instead.
// Culling is conservative as in AccelTraceK (boxes padded by kAccelKappa (M + |o|_1)); the pruning bound
// exceeds best by 2^-16 best so that the reach test's near-boundary cases (a box face hit, where A's
// entry slab value and the plane t are two roundings of one number) see every competitor.
constexpr float kMixBoundRel = 1.52587890625e-05f;   // 2^-16

__device__ __forceinline__ bool mix_box(const Trav &T, const SlabRay &R, float x0, float x1, float y0, float y1, float z0,
                                        float z1, float bound, float *tnear) {
  // the octant from 1/d's signs (SlabRay's flags, recomputed: three registers fewer across the mixed walk)
  const bool sx = T.inv.x < 0.0f, sy = T.inv.y < 0.0f, sz = T.inv.z < 0.0f;
  const float nx = __builtin_fmaf(sx ? x1 : x0, T.inv.x, R.on.x), fx = __builtin_fmaf(sx ? x0 : x1, T.inv.x, R.of.x);
  const float ny = __builtin_fmaf(sy ? y1 : y0, T.inv.y, R.on.y), fy = __builtin_fmaf(sy ? y0 : y1, T.inv.y, R.of.y);
  const float nz = __builtin_fmaf(sz ? z1 : z0, T.inv.z, R.on.z), fz = __builtin_fmaf(sz ? z0 : z1, T.inv.z, R.of.z);
  const float t0 = fmaxf(fmaxf(nx, ny), fmaxf(nz, kTmin)), t1 = fminf(fminf(fx, fy), fminf(fz, bound));
  *tnear = t0;
  return !(t1 < t0);
}

// candidate value of a quad / triangle (geom_calc_hit, :1060-1077, + the inside test of :1131-1175): the
// plane t when t >= tmin and the point is inside; ok = false otherwise.  Same operations as planar_hit.
// lim: a plane t above it cannot change the walk's result (the caller's bound), so its inside test is skipped
__device__ __forceinline__ float planar_value(const Ray &r, bool tri, f3 n, float dd, f3 q, f3 uu, f3 vv, f3 ww, bool &ok,
                                              float lim = __builtin_huge_valf()) {
  ok = false;
  float t = 0.0f;
  const float denom = dot(n, r.d);
  if (fabsf(denom) >= kDenomEps) {
    t = (dd - dot(n, r.o)) / denom;
    if (kTmin <= t && t <= lim) {
      const f3 p = line_at(r.o, t, r.d);
      const f3 pq = sub(p, q);
      const float alpha = dot(ww, cross(pq, vv));
      const float beta = dot(ww, cross(uu, pq));
      bool inside = (0.0f <= alpha) & (alpha <= 1.0f) & (0.0f <= beta) & (beta <= 1.0f);
      if (tri) inside = inside & (alpha + beta <= 1.0f);
      ok = inside;
    }
  }
  return t;
}

// candidate value of a sphere (:1093-1110): the root hit() accepts for any tmax above it
__device__ __forceinline__ float sphere_value(const Ray &r, f3 c0, f3 mv, float rad2, bool &ok) {
  const f3 center = line_at(c0, r.time, mv);
  const f3 oc = sub(center, r.o);
  const float a = dot(r.d, r.d);
  const float b = -2.0f * dot(r.d, oc);
  const float c = dot(oc, oc) - rad2;
  const float disc = b * b - 4 * a * c;
  ok = false;
  if (!(disc >= 0)) return 0.0f;
  const float sq = sqrtf(disc);
  float root = (-b - sq) / (2.0f * a);
  if (kTmin >= root || root >= __builtin_huge_valf()) root = (-b + sq) / (2.0f * a);
  ok = kTmin < root && root < __builtin_huge_valf();
  return root;
}

// PAUSE: as in LaneTraceK, the round's walk may stop once few lanes still walk; it stops only between two
// reference steps (no lane inside a macro walk), where the whole walk state is T, the ray (drift included),
// the hit record and the LDS stack, all of which outlive the round.
template <uint32_t KM, bool PAUSE = false>
struct MixedTraceK {
  template <bool LDS, bool COUNT, bool UV>
  __device__ __forceinline__ static void run(const Mem<LDS> &S, const RenderArgs &A, bool busy, uint64_t lanes,
                                             uint32_t lane, uint16_t *stk, Trav &T, Ray &r, Hit &h, Visits &vc) {
    if (COUNT) {   // the counting variant walks the reference tree (the op model counts its visits)
      LaneTraceK<KM, false, true>::template run<LDS, COUNT, UV>(S, A, busy, lanes, lane, stk, T, r, h, vc);
      return;
    }
    if (!busy) return;
    if (!PAUSE || !T.active) {
      trav_reset(T, r);
      stk[0] = static_cast<uint16_t>(A.root);
      T.sp = 1;
    }
    T.active = 0;
    const uint4 *N = reinterpret_cast<const uint4 *>(A.scene + A.mix_nodes);
    const uint4 *P = reinterpret_cast<const uint4 *>(A.scene + A.mix_prims);
    bool walking = true, in_macro = false;
    uint32_t mroot = 0, mnode = 0, bprim = 0, bgroup = 0;
    int msp = 0;
    float best = __builtin_huge_valf(), second = __builtin_huge_valf();
    bool tie = false;
    SlabRay sr;
    sr.on = mk(0, 0, 0); sr.of = mk(0, 0, 0); sr.nx = sr.ny = sr.nz = false;
#ifdef RT_MIX_DIAG
    // diagnostic build (RT_JIT_OPTS=-DRT_MIX_DIAG): wave trips, lanes per phase, reference steps by kind;
    // every value is wave-uniform (ballots at the top of a trip, where all the wave's walkers are active)
    unsigned long long dg[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    dg[9] = __popcll(__ballot(true));
#endif
    const uint32_t started = PAUSE ? static_cast<uint32_t>(__popcll(__ballot(true))) : 0u;
    uint32_t it = 0;
    for (;;) {
      const uint64_t wl = __ballot(walking);
      if (wl == 0) break;
      if (PAUSE) {
        const uint32_t nl = static_cast<uint32_t>(__popcll(wl));
        if (++it >= A.trace_min_iters && nl <= A.defer_trace && 4 * nl <= started && __ballot(in_macro) == 0) {
          T.active = walking && T.sp > 0 ? 1u : 0u;   // resumes next round with shading skipped
          break;
        }
      }
#ifdef RT_MIX_DIAG
      {
        const bool rs = walking && !in_macro && T.sp != 0;
        const uint64_t rl = __ballot(rs), ml = __ballot(walking && in_macro);
        const uint32_t k = rs ? S.w4(stk[(T.sp - 1) * 64] * kNodeWords).x : 0xffu;
        const uint64_t bv = __ballot(k == K_BVH), qd = __ballot(k == K_QUAD || k == K_TRIANGLE),
                       ch = __ballot(k == K_TRANSLATE || k == K_YROTATE);
        dg[0]++;
        dg[1] += __popcll(rl);
        dg[2] += __popcll(ml);
        dg[3] += (rl != 0 && ml != 0) ? 1u : 0u;
        dg[4] += (rl != 0) ? 1u : 0u;
        dg[5] += __popcll(bv); dg[6] += __popcll(qd); dg[7] += __popcll(ch);
        dg[8] += (bv != 0) + (qd != 0) + (ch != 0) + ((rl & ~(bv | qd | ch)) != 0);
      }
#endif
      if (!walking) continue;
#ifdef RT_MIX_KIND
      // kind-scheduled trips (A/B: RT_JIT_OPTS=-DRT_MIX_KIND=1): the step each walking lane would take next is one of
      // four classes — a reference BVH node, a transform (a fused / packed chain or an enter / exit), any other
      // reference record, a step of a macro's SAH walk — and a trip runs one class only, the one most lanes hold (ties:
      // the lower class), so the wave issues one step body per trip instead of one per class present.  The other
      // lanes wait a trip; every lane still takes its own steps in its own order, with its own in-place drift.
      if (!in_macro && T.sp == 0) { walking = false; continue; }
      {
        uint32_t cls = 3u;
        if (!in_macro) {
          const uint32_t k = S.w4(static_cast<uint32_t>(stk[(T.sp - 1) * 64]) * kNodeWords).x;
          cls = k == K_BVH ? 0u : ((k == K_TRANSLATE || k == K_YROTATE) ? 1u : 2u);
        }
        const uint32_t n0 = static_cast<uint32_t>(__popcll(__ballot(cls == 0u)));
        const uint32_t n1 = static_cast<uint32_t>(__popcll(__ballot(cls == 1u)));
        const uint32_t n2 = static_cast<uint32_t>(__popcll(__ballot(cls == 2u)));
        const uint32_t n3 = static_cast<uint32_t>(__popcll(__ballot(cls == 3u)));
        uint32_t sel = 0u, best_n = n0;
        if (n1 > best_n) { sel = 1u; best_n = n1; }
        if (n2 > best_n) { sel = 2u; best_n = n2; }
        if (n3 > best_n) sel = 3u;
        if (cls != sel) continue;
      }
#endif
      if (!in_macro) {
        if (T.sp == 0) { walking = false; continue; }
        // ---- one step of the reference walk (trav_step), macro roots aside ----
        int sp = T.sp - 1;
        const uint32_t idx = stk[sp * 64];
        const uint32_t nb = idx * kNodeWords;
        const uint4 w0 = S.w4(nb), w1 = S.w4(nb + 4), w2 = S.w4(nb + 8), w3 = S.w4(nb + 12), w4 = S.w4(nb + 16);
        const uint32_t kind = w0.x;
        const bool in_xf = T.tc || T.yc;
        bool expand = false;   // a BVH node whose box passed / a group: push its children (unless a macro)
        // dispatch: the two common steps (a BVH node; a fused chain ending in a packed sphere) first, every
        // other kind in one block, so a trip whose lanes hold only common steps skips the rest with one
        // branch (each divergent `if` costs exec-mask bookkeeping on every trip)
        const bool xf_kind = kind == K_TRANSLATE || kind == K_YROTATE;
        constexpr bool packed_chain_ok = (KM & ((1u << K_TRANSLATE) | (1u << K_YROTATE))) && (KM & (1u << K_SPHERE));
        const bool packed_chain = packed_chain_ok && xf_kind &&
                                  (w3.x & (kChainFused | kChainPacked)) == (kChainFused | kChainPacked) &&
                                  (kind == K_TRANSLATE ? T.tc : T.yc) == 0;
        // translate -> [y-rotate ->] sphere, or y-rotate -> sphere, packed into the head record
        // (mixed_accel.cpp): the reference's enter, enter, test, cleanup, cleanup steps (:1176-1237) at once
        auto packed_step = [&](uint4 v0, uint4 v1, uint4 v2, uint4 v3, uint4 v4) {
          const bool tr = v0.x == K_TRANSLATE;
          const bool rot = !tr || (v3.x & kChainRotate);
          const f3 off = mk(asf(v0.z), asf(v0.w), asf(v1.x));
          const float sn = asf(v3.y), cs = asf(v3.z);
          if (tr) translate_enter(T, r, off);
          if (rot) rotate_enter_dir(T, r, sn, cs);   // no box test inside: 1/dir is refreshed at the exit
          sphere_hit<UV>(T, r, h, v1.y, mk(asf(v1.z), asf(v1.w), asf(v4.x)), mk(asf(v4.y), asf(v4.z), asf(v4.w)),
                         asf(v2.y), asf(v2.z), true, v2.w != 0u);
          if (rot) rotate_exit(T, r, h, sn, cs);
          if (tr) translate_exit(T, r, h, off);
        };
        if ((KM & (1u << K_BVH)) && kind == K_BVH) {
          expand = box_hit(T, r, asf(w0.z), asf(w0.w), asf(w1.x), asf(w1.y), asf(w1.z), asf(w1.w));
        } else if (packed_chain) {
          packed_step(w0, w1, w2, w3, w4);
        } else if ((KM & (1u << K_GROUP)) && kind == K_GROUP) {
          expand = true;
        } else if ((KM & ((1u << K_QUAD) | (1u << K_TRIANGLE))) && (kind == K_QUAD || kind == K_TRIANGLE)) {
          planar_hit(T, r, h, kind == K_TRIANGLE, w0.y, mk(asf(w0.z), asf(w0.w), asf(w1.x)), asf(w1.y),
                     mk(asf(w1.z), asf(w1.w), asf(w2.x)), mk(asf(w2.y), asf(w2.z), asf(w2.w)),
                     mk(asf(w3.x), asf(w3.y), asf(w3.z)), mk(asf(w3.w), asf(w4.x), asf(w4.y)), in_xf);
        } else if ((KM & (1u << K_SPHERE)) && kind == K_SPHERE) {
          sphere_hit<UV>(T, r, h, w0.y, mk(asf(w0.z), asf(w0.w), asf(w1.x)), mk(asf(w1.y), asf(w1.z), asf(w1.w)),
                         asf(w2.y), asf(w2.z), in_xf, w2.w != 0u);
        } else if ((KM & ((1u << K_TRANSLATE) | (1u << K_YROTATE))) && (kind == K_TRANSLATE || kind == K_YROTATE)) {
          const bool tr = kind == K_TRANSLATE;
          const uint32_t chain = w3.x;   // W_MACRO: fused chain marker
          if ((tr ? T.tc : T.yc) == 0 && (chain & kChainFused)) {
            // translate -> [y-rotate ->] primitive, or y-rotate -> primitive: the reference's enter, enter,
            // test, cleanup, cleanup steps (:1176-1237, in this order, nothing else runs in between) at once
            const f3 off = mk(asf(w0.z), asf(w0.w), asf(w1.x));
            const bool rot = !tr || (chain & kChainRotate);
            float sn = asf(w0.z), cs = asf(w0.w);
            if (tr) {
              translate_enter(T, r, off);
              if (rot) { const uint4 c0 = S.w4(w0.y * kNodeWords); sn = asf(c0.z); cs = asf(c0.w); }
            }
            if (rot) rotate_enter_dir(T, r, sn, cs);   // no box test inside: 1/dir is refreshed at the exit
            const uint32_t gb = (chain & kChainPrimMask) * kNodeWords;
            const uint4 g0 = S.w4(gb), g1 = S.w4(gb + 4), g2 = S.w4(gb + 8), g3 = S.w4(gb + 12), g4 = S.w4(gb + 16);
            if ((KM & (1u << K_SPHERE)) && g0.x == K_SPHERE)
              sphere_hit<UV>(T, r, h, g0.y, mk(asf(g0.z), asf(g0.w), asf(g1.x)), mk(asf(g1.y), asf(g1.z), asf(g1.w)),
                             asf(g2.y), asf(g2.z), true, g2.w != 0u);
            else
              planar_hit(T, r, h, g0.x == K_TRIANGLE, g0.y, mk(asf(g0.z), asf(g0.w), asf(g1.x)), asf(g1.y),
                         mk(asf(g1.z), asf(g1.w), asf(g2.x)), mk(asf(g2.y), asf(g2.z), asf(g2.w)),
                         mk(asf(g3.x), asf(g3.y), asf(g3.z)), mk(asf(g3.w), asf(g4.x), asf(g4.y)), true);
            if (rot) rotate_exit(T, r, h, sn, cs);
            if (tr) translate_exit(T, r, h, off);
          } else if (tr) {
            const f3 off = mk(asf(w0.z), asf(w0.w), asf(w1.x));
            if (T.tc == 0) {
              translate_enter(T, r, off);
              stk[sp * 64] = static_cast<uint16_t>(idx);
              stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);
              sp += 2;
              T.tc++;
            } else {
              T.tc--;
              translate_exit(T, r, h, off);
            }
          } else {
            if (T.yc == 0) {
              rotate_enter(T, r, asf(w0.z), asf(w0.w));
              stk[sp * 64] = static_cast<uint16_t>(idx);
              stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);
              sp += 2;
              T.yc++;
            } else {
              T.yc--;
              rotate_exit(T, r, h, asf(w0.z), asf(w0.w));
            }
          }
        }
        if (expand) {
          const uint32_t mw = w3.x;   // W_MACRO
          bool macro = (mw & (kMacroStatic | kMacroDynamic)) != 0;
          if (macro) {
            // bounded, finite rays only (finite 1/dir: the slab arithmetic stays monotone, the conservative
            // boxes hold); a dynamic macro only when the ray misses W_XFBOX in the reference's own test
            const float ao = fabsf(r.o.x) + fabsf(r.o.y) + fabsf(r.o.z);
            const float dmin = fminf(fminf(fabsf(r.d.x), fabsf(r.d.y)), fabsf(r.d.z));
            const float dmax = fmaxf(fmaxf(fabsf(r.d.x), fabsf(r.d.y)), fabsf(r.d.z));
            macro = (ao <= 1.0e6f) && (dmin >= 1.0e-20f) && (dmax <= 1.0e6f);
            if (macro && (mw & kMacroDynamic))
              macro = !box_hit(T, r, asf(w3.y), asf(w3.z), asf(w3.w), asf(w4.x), asf(w4.y), asf(w4.z));
            if (macro) {
              in_macro = true;
              mroot = idx;
              mnode = mw & kMacroRootMask;
              msp = 0;
              best = __builtin_huge_valf();
              second = __builtin_huge_valf();
              bprim = 0; bgroup = kMixNoGroup;
              tie = false;
#ifndef RT_MIX_SLAB_RECOMPUTE
              const float pad_o = kAccelKappa * ao;
              const f3 oinv = mk(r.o.x * T.inv.x, r.o.y * T.inv.y, r.o.z * T.inv.z);
              const f3 pinv = mk(pad_o * fabsf(T.inv.x), pad_o * fabsf(T.inv.y), pad_o * fabsf(T.inv.z));
              sr = slab_ray(T, oinv, pinv);
#endif
            }
          }
          if (!macro) {
            if (kind == K_BVH) {
              stk[sp * 64] = static_cast<uint16_t>(w0.y >> 16);      // right
              stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);      // left (popped first)
              sp += 2;
            } else {
              const uint32_t first = w0.y, n = w0.z;
              for (uint32_t i = 0; i < n; ++i) stk[(sp + i) * 64] = static_cast<uint16_t>(first + i);
              sp += n;
            }
          }
        }
        if (!RT_CHECK(A, static_cast<uint32_t>(sp) <= A.stack_cap, CHK_MIXED_STACK, sp, A.stack_cap)) sp = 0;
        T.sp = sp;
        continue;
      }
      // ---- one step of the macro's SAH walk ----
#ifdef RT_MIX_SLAB_RECOMPUTE
      // A/B (RT_JIT_OPTS=-DRT_MIX_SLAB_RECOMPUTE): the padded slab offsets recomputed every step from the ray (unchanged
      // inside a macro: the same operations on the same values as at the entry) instead of held — six registers fewer,
      // so that RT_JIT_WAVES=4 builds the walk at 128 VGPRs without spilling
      {
        const float ao = fabsf(r.o.x) + fabsf(r.o.y) + fabsf(r.o.z);
        const float pad_o = kAccelKappa * ao;
        const f3 oinv = mk(r.o.x * T.inv.x, r.o.y * T.inv.y, r.o.z * T.inv.z);
        const f3 pinv = mk(pad_o * fabsf(T.inv.x), pad_o * fabsf(T.inv.y), pad_o * fabsf(T.inv.z));
        sr = slab_ray(T, oinv, pinv);
      }
#endif
      const float cur = fminf(best, T.tmax);
      const float bound = best < __builtin_huge_valf() ? fminf(T.tmax, best + best * kMixBoundRel) : T.tmax;
      const uint4 q0 = N[mnode * 4], q1 = N[mnode * 4 + 1], q2 = N[mnode * 4 + 2], q3 = N[mnode * 4 + 3];
      float n0, n1;
      bool h0 = mix_box(T, sr, asf(q0.x), asf(q0.y), asf(q0.z), asf(q0.w), asf(q1.x), asf(q1.y), bound, &n0);
      bool h1 = mix_box(T, sr, asf(q1.z), asf(q1.w), asf(q2.x), asf(q2.y), asf(q2.z), asf(q2.w), bound, &n1);
      const bool near0 = n0 <= n1;
      const uint32_t rn = near0 ? q3.x : q3.y, rf = near0 ? q3.y : q3.x;
      bool hn = near0 ? h0 : h1, hf = near0 ? h1 : h0;
      const bool ln = hn && (rn & kAccelLeaf), lf = hf && (rf & kAccelLeaf);
      const uint32_t c1 = ln ? ((rn >> 24) & 0x7fu) + 1u : 0u, c2 = lf ? ((rf >> 24) & 0x7fu) + 1u : 0u;
      const uint32_t f1 = rn & 0xffffffu, f2 = (rf & 0xffffffu) - c1;
      float cur_k = cur;
      for (uint32_t k = 0; k < c1 + c2; ++k) {
        const uint32_t pr = (k < c1 ? f1 : f2) + k;
        const uint4 *pw = P + static_cast<size_t>(pr) * (kMixPrimWords / 4);
        const uint4 p0 = pw[0], p1 = pw[1], p2 = pw[2];
        bool ok;
        float v;
        if ((KM & (1u << K_SPHERE)) && p0.x == K_SPHERE) {
          v = sphere_value(r, mk(asf(p0.z), asf(p0.w), asf(p1.x)), mk(asf(p1.y), asf(p1.z), asf(p1.w)), asf(p2.y), ok);
        } else {
          const uint4 p3 = pw[3], p4 = pw[4];
          // a candidate matters only at or below the running value (best / tie) or below min(second, T.tmax)
          // (the reach proof reads second only through that minimum): others skip the inside test
          v = planar_value(r, p0.x == K_TRIANGLE, mk(asf(p0.z), asf(p0.w), asf(p1.x)), asf(p1.y),
                           mk(asf(p1.z), asf(p1.w), asf(p2.x)), mk(asf(p2.y), asf(p2.z), asf(p2.w)),
                           mk(asf(p3.x), asf(p3.y), asf(p3.z)), mk(asf(p3.w), asf(p4.x), asf(p4.y)), ok,
                           fmaxf(cur_k, fminf(second, T.tmax)));
        }
        if (ok) {
          const uint32_t g = pw[5].x;   // MP_GROUP
          if (v < cur_k) {
            if (best < __builtin_huge_valf() && g != bgroup) second = fminf(second, best);
            best = v; bprim = pr; bgroup = g;
            cur_k = v;
            tie = false;   // a tie at a larger value no longer matters: the reference ends on this one
          } else if (v == cur_k) {
            tie = true;
          } else if (g != bgroup) {
            second = fminf(second, v);
          }
        }
      }
      hn = hn && !ln;
      hf = hf && !lf;
      if (hn && hf) {
        stk[(T.sp + msp) * 64] = static_cast<uint16_t>(rf);
        ++msp;
        if (!RT_CHECK(A, T.sp + msp <= A.stack_cap, CHK_MIXED_STACK, T.sp + msp, A.stack_cap)) msp = 0;
        mnode = rn;
        continue;
      }
      if (hn | hf) { mnode = hn ? rn : rf; continue; }
      if (msp > 0) { --msp; mnode = stk[(T.sp + msp) * 64]; continue; }
      // ---- walk done: prove the record, commit it, or hand the subtree to the reference walk ----
      in_macro = false;
      bool ok = !tie && !A.mix_no_proof;
      const uint4 *bw = P + static_cast<size_t>(bprim) * (kMixPrimWords / 4);
      if (ok && best < __builtin_huge_valf() && bgroup != kMixNoGroup) {
        const float bnd = fminf(T.tmax, best + best * kMixBoundRel);
        const uint4 g0 = bw[5], g1 = bw[6];
        Trav tt = T;
        tt.tmax = fminf(fminf(T.tmax, second), bnd);
        ok = box_hit(tt, r, asf(g0.y), asf(g0.z), asf(g0.w), asf(g1.x), asf(g1.y), asf(g1.z));
      }
      if (ok) {
        if (best < __builtin_huge_valf()) {
          const uint4 p0 = bw[0], p1 = bw[1], p2 = bw[2], p3 = bw[3], p4 = bw[4];
          if ((KM & (1u << K_SPHERE)) && p0.x == K_SPHERE) {
            T.tmax = best;
            sphere_commit<UV>(T, r, h, p0.y, mk(asf(p0.z), asf(p0.w), asf(p1.x)), mk(asf(p1.y), asf(p1.z), asf(p1.w)), asf(p2.z),
                              p2.w != 0u);
          } else {
            // planar_hit's record at t = best (tmax = best: the same plane test accepts it)
            T.tmax = best;
            planar_hit(T, r, h, p0.x == K_TRIANGLE, p0.y, mk(asf(p0.z), asf(p0.w), asf(p1.x)), asf(p1.y),
                       mk(asf(p1.z), asf(p1.w), asf(p2.x)), mk(asf(p2.y), asf(p2.z), asf(p2.w)),
                       mk(asf(p3.x), asf(p3.y), asf(p3.z)), mk(asf(p3.w), asf(p4.x), asf(p4.y)), false);
          }
          T.result = true;
          if (T.tc || T.yc) T.was_last = 1;
        }
      } else {   // the reference's own expansion of the macro root (its box test already passed)
        if (A.mix_fallbacks) {   // rare (diagnostic): total, then by reason (tie | reach) in the next words
          atomicAdd(A.mix_fallbacks, 1u);
          atomicAdd(A.mix_fallbacks - 9 + (tie ? 0 : 1), 1u);
        }
        const uint32_t nb = mroot * kNodeWords;
        const uint4 w0 = S.w4(nb);
        int sp = T.sp;
        if (w0.x == K_BVH) {
          stk[sp * 64] = static_cast<uint16_t>(w0.y >> 16);
          stk[(sp + 1) * 64] = static_cast<uint16_t>(w0.y);
          sp += 2;
        } else {
          for (uint32_t i = 0; i < w0.z; ++i) stk[(sp + i) * 64] = static_cast<uint16_t>(w0.y + i);
          sp += w0.z;
        }
        if (!RT_CHECK(A, static_cast<uint32_t>(sp) <= A.stack_cap, CHK_MIXED_STACK, sp, A.stack_cap)) sp = 0;
        T.sp = sp;
      }
    }
#ifdef RT_MIX_DIAG
    if (A.mix_fallbacks && __builtin_amdgcn_readfirstlane(lane) == lane) {
      unsigned long long *d = reinterpret_cast<unsigned long long *>(A.mix_fallbacks + 5);
      for (int i = 0; i < 10; ++i) atomicAdd(d + i, dg[i]);
    }
#endif
  }
};

// ---------------------------------------------------------------------------------------------
// traversal policy 2: one DFS per wave with per-entry lane masks
// ---------------------------------------------------------------------------------------------
// The reference's DFS order is fixed by the scene, not by the ray: a hit BVH node pushes right then
// left (:1127-1128), a group pushes its children in index order (:1243-1245), a transform pushes
// itself then its child (:1181-1182, :1207-1208).  So all rays of a wave can share ONE stack whose
// entries carry the set of lanes that pushed them: restricted to lane L, the shared stack IS lane L's
// own stack at every moment, and lane L processes exactly its own node sequence in its own order.
// Each popped node is processed once for all its lanes; its kind and data are wave-uniform (scalar
// loads, scalar branches) and the stack lives in three VGPRs used as 64-entry lane-indexed arrays.
typedef const __attribute__((address_space(4))) uint32_t *cnode_ptr;

struct WStack {          // wave-uniform stack: entry e lives in lane e of each register
  uint32_t node, mlo, mhi;
  int sp;
};

__device__ __forceinline__ void wpush(WStack &W, uint32_t lane, uint32_t node, uint64_t mask) {
  const bool here = lane == static_cast<uint32_t>(W.sp);   // write entry sp into lane sp
  W.node = here ? node : W.node;
  W.mlo = here ? static_cast<uint32_t>(mask) : W.mlo;
  W.mhi = here ? static_cast<uint32_t>(mask >> 32) : W.mhi;
  W.sp++;
}

struct PacketTrace {
  template <bool LDS, bool COUNT, bool UV>
  __device__ __forceinline__ static void run(const Mem<LDS> &, const RenderArgs &A, bool busy, uint64_t lanes,
                                             uint32_t lane, uint16_t *, Trav &T, Ray &r, Hit &h, Visits &vc) {
    cnode_ptr nodes = (cnode_ptr)(reinterpret_cast<uintptr_t>(A.scene));
    if (busy) trav_reset(T, r);   // a lane resuming its rejection sampling keeps its hit
    WStack W{0, 0, 0, 0};
    wpush(W, lane, A.root, lanes);
    int depth_seen = 1;
    while (W.sp > 0) {
      W.sp--;
      // readlane returns int: go through uint32_t so the low half is not sign-extended
      const uint32_t node = static_cast<uint32_t>(__builtin_amdgcn_readlane(W.node, W.sp));
      const uint32_t mlo = static_cast<uint32_t>(__builtin_amdgcn_readlane(W.mlo, W.sp));
      const uint32_t mhi = static_cast<uint32_t>(__builtin_amdgcn_readlane(W.mhi, W.sp));
      const uint64_t mask = (static_cast<uint64_t>(mhi) << 32) | mlo;
      const bool active = (mask >> lane) & 1ull;
      const uint32_t nb = node * kNodeWords;
      const uint32_t kind = nodes[nb + W_KIND];
      const uint32_t aux = nodes[nb + W_AUX];
      const bool in_xf = T.tc || T.yc;
      if (COUNT && active) vc.k[kind < 7 ? kind : 0]++;
      if (kind == K_BVH) {
        const float x0 = asf(nodes[nb + 2]), x1 = asf(nodes[nb + 3]), y0 = asf(nodes[nb + 4]);
        const float y1 = asf(nodes[nb + 5]), z0 = asf(nodes[nb + 6]), z1 = asf(nodes[nb + 7]);
        bool hit = false;
        if (active) hit = box_hit(T, r, x0, x1, y0, y1, z0, z1);
        const uint64_t hm = __ballot(hit);
        if (hm) {
          wpush(W, lane, aux >> 16, hm);        // right
          wpush(W, lane, aux & 0xffffu, hm);    // left (popped first)
        }
      } else if (kind == K_QUAD || kind == K_TRIANGLE) {
        const f3 n = mk(asf(nodes[nb + W_NORMAL]), asf(nodes[nb + W_NORMAL + 1]), asf(nodes[nb + W_NORMAL + 2]));
        const f3 q = mk(asf(nodes[nb + W_Q]), asf(nodes[nb + W_Q + 1]), asf(nodes[nb + W_Q + 2]));
        const f3 uu = mk(asf(nodes[nb + W_U]), asf(nodes[nb + W_U + 1]), asf(nodes[nb + W_U + 2]));
        const f3 vv = mk(asf(nodes[nb + W_V]), asf(nodes[nb + W_V + 1]), asf(nodes[nb + W_V + 2]));
        const f3 ww = mk(asf(nodes[nb + W_W]), asf(nodes[nb + W_W + 1]), asf(nodes[nb + W_W + 2]));
        const float dd = asf(nodes[nb + W_D]);
        if (active) planar_hit(T, r, h, kind == K_TRIANGLE, aux, n, dd, q, uu, vv, ww, in_xf);
      } else if (kind == K_SPHERE) {
        const f3 c0 = mk(asf(nodes[nb + W_CENTER]), asf(nodes[nb + W_CENTER + 1]), asf(nodes[nb + W_CENTER + 2]));
        const f3 mv = mk(asf(nodes[nb + W_MOTION]), asf(nodes[nb + W_MOTION + 1]), asf(nodes[nb + W_MOTION + 2]));
        const float rad2 = asf(nodes[nb + W_RADIUS2]), inv_rad = asf(nodes[nb + W_INV_RADIUS]);
        if (active) sphere_hit<UV>(T, r, h, aux, c0, mv, rad2, inv_rad, in_xf);
      } else if (kind == K_TRANSLATE) {
        const f3 off = mk(asf(nodes[nb + W_OFFSET]), asf(nodes[nb + W_OFFSET + 1]), asf(nodes[nb + W_OFFSET + 2]));
        bool enter = false;
        if (active) {
          if (T.tc == 0) { enter = true; translate_enter(T, r, off); T.tc++; }
          else { T.tc--; translate_exit(T, r, h, off); }
        }
        const uint64_t em = __ballot(enter);
        if (em) { wpush(W, lane, node, em); wpush(W, lane, aux, em); }
      } else if (kind == K_YROTATE) {
        const float sn = asf(nodes[nb + W_SIN]), cs = asf(nodes[nb + W_COS]);
        bool enter = false;
        if (active) {
          if (T.yc == 0) { enter = true; rotate_enter(T, r, sn, cs); T.yc++; }
          else { T.yc--; rotate_exit(T, r, h, sn, cs); }
        }
        const uint64_t em = __ballot(enter);
        if (em) { wpush(W, lane, node, em); wpush(W, lane, aux, em); }
      } else if (kind == K_GROUP) {
        const uint32_t n = nodes[nb + W_COUNT];
        for (uint32_t i = 0; i < n; ++i) wpush(W, lane, (aux + i) & 0xffffu, mask);
      }
      if (COUNT && W.sp > depth_seen) depth_seen = W.sp;
    }
    if (COUNT && static_cast<uint32_t>(depth_seen) > vc.max_sp) vc.max_sp = depth_seen;
  }
};

// ---------------------------------------------------------------------------------------------
// cooperative Perlin turbulence (perlin_noise.cpp:72-85 through texture_get_color's noise case,
// raytracing.cu:386-395): the 7 octaves of the lanes in M spread over K lanes each
// ---------------------------------------------------------------------------------------------
// Lane L serves the noise lane of rank L / K (the (L / K)-th set bit of M) and evaluates its octaves
// o = L % K, L % K + K, ... < 7 at q = p * 2^o — bit-identical to the reference's repeated doubling
// (scaling by a power of two is exact, and overflows exactly when the doubling does).  Each noise lane
// then gathers its 7 values and sums them in the reference's order.  Every lane of the wave must be
// active.  Returns the colour-stack code of the attenuation for the lanes in M (unused elsewhere).
template <int K, bool LDS>
__device__ __forceinline__ uint32_t coop_noise_code(const Mem<LDS> &S, const RenderArgs &A, uint64_t M, uint32_t lane,
                                                    uint64_t lt_mask, f3 p, uint32_t tb, float scale) {
  const uint32_t grp = lane / K, slot = lane % K;
  uint32_t pos = 0, r = grp;   // select the grp-th set bit of M
#pragma unroll
  for (uint32_t s = 32; s >= 1; s >>= 1) {
    const uint32_t c = static_cast<uint32_t>(__popcll((M >> pos) & ((1ull << s) - 1ull)));
    if (r >= c) { r -= c; pos += s; }
  }
  const bool serve = grp < static_cast<uint32_t>(__popcll(M));
  const int own = static_cast<int>(serve ? pos : lane);
  const float px = __shfl(p.x, own), py = __shfl(p.y, own), pz = __shfl(p.z, own);
  const uint32_t otb = static_cast<uint32_t>(__shfl(static_cast<int>(tb), own));
  constexpr int NI = (7 + K - 1) / K;
  float nv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const uint32_t o = slot + static_cast<uint32_t>(i * K);
    nv[i] = 0.0f;
    if (serve && o < 7u) {
      const float sc = __uint_as_float((127u + o) << 23);   // 2^o
      nv[i] = perlin_noise(S, otb, mk(px * sc, py * sc, pz * sc));
    }
  }
  const int rank = static_cast<int>(__popcll(M & lt_mask));
  float accum = 0.0f, weight = 1.0f;
#pragma unroll
  for (int o = 0; o < 7; ++o) {
    accum += weight * __shfl(nv[o / K], rank * K + (o % K));
    weight *= 0.5f;
  }
  const float turb = fabsf(accum);
  const float sv = 1 + rt_sinf(scale * p.z + 10 * turb);
  const uint32_t g = __float_as_uint(0.5f * sv);
  return ((g & kRcRecTag) == kRcRecTag) ? (kRcRecTag | (A.rc_consts + RC_NAN)) : g;
}

// linear -> P6 byte of pixels_to_ppm (raytracing.cu:1391-1395, 1419-1431): sqrt gamma (0 for
// non-positive), clamp to [0, 0.999], (u8)(256 x) — the conversion of rt_tonemap / tonemap_kernel
__device__ __forceinline__ uint8_t ppm_byte(float c) {
  const float g = c > 0 ? sqrtf(c) : 0.0f;
  const float k = (g < 0.0f) ? 0.0f : ((g > 0.999f) ? 0.999f : g);
  return static_cast<uint8_t>(static_cast<uint32_t>(256 * k) & 0xffu);
}

// ---------------------------------------------------------------------------------------------
// the render body (cuda_calc + ray_color)
// ---------------------------------------------------------------------------------------------
// Each loop iteration is one "round": lanes without a pixel take the next pixels of their wave's
// 8x8 tile (ballot + prefix count: active-path compaction), every lane with a pixel traces one path
// segment (Trace policy), then shades it.  A lane whose path ended unwinds, accumulates and
// immediately starts its next camera sample, so every lane traces every round.  A lane owns one pixel
// and runs that pixel's samples strictly in order (one XORWOW stream per pixel), so scheduling never
// changes what a lane computes.
template <int F, class Trace>
__device__ __forceinline__ void render_body(const RenderArgs &A) {
  constexpr bool LDS = (F & kVarLds) != 0, COUNT = (F & kVarCount) != 0;
  constexpr bool NOISE = (F & kVarNoise) != 0, UV = (F & kVarUv) != 0;
  constexpr bool TRACE = (F & kVarTrace) != 0;   // per-wave timeline into A.wave_trace (diagnostics)
  constexpr bool DEEP = (F & kVarDeep) != 0;     // batched unwind of HBM colour-stack levels
  constexpr bool COOP = NOISE && (F & kVarCoop) != 0;   // cooperative noise octaves
  // schedule probe launch (1-spp throwaway paths, costs per tile): fixed at compile time in the run-time
  // compiled kernels, read from RenderArgs::probe_cost in the offline ones
  const bool probe = (F & kVarProbe) != 0 || ((F & kVarNoProbe) == 0 && A.probe_cost != nullptr);
  constexpr uint32_t MM = ((F >> kVarMatShift) & 15) ? ((F >> kVarMatShift) & 15) : 15u;   // material kinds
  constexpr uint32_t TM = ((F >> kVarTexShift) & 15) ? ((F >> kVarTexShift) & 15) : 15u;   // texture kinds
  // kernel-only span (A.span): the start is the earliest first wave of blocks 0..7 — one block per XCD (workgroups go
  // round-robin over the 8 XCDs, and block 0's XCD need not start first) — recorded at once rather than
  // held in registers to the end.  (A start atomic from every wave serialised ~6k same-address device atomics ahead
  // of the first barrier: scene 0 +8 ms, profiles/r04_ab_v17_scene0.jsonl; eight are noise.)
  if (A.span && blockIdx.x < 8u && threadIdx.x == 0)
    atomicMax(A.span, static_cast<unsigned long long>(~__builtin_amdgcn_s_memrealtime()));
  Mem<LDS> S{A.scene};
  // kargs() reads RenderArgs from the kernarg segment's start: every kernel must take it as its only argument
  [[maybe_unused]] const bool kargs_ok = RT_CHECK(A, kargs(A)->scene == A.scene && kargs(A)->n_ids == A.n_ids &&
                                                        kargs(A)->spp == A.spp, CHK_KARGS, 0u, 1u);
  if (LDS) {
    const uint32_t n4 = A.scene_words / 4;
    const uint4 *src = reinterpret_cast<const uint4 *>(A.scene);
    uint4 *dst = reinterpret_cast<uint4 *>(g_lds);
    for (uint32_t i = threadIdx.x; i < n4; i += kBlock) dst[i] = src[i];
    __syncthreads();
  } else if (A.accel_lds_nodes) {   // the verified walk's top nodes (A.accel_node_u4 uint4 each)
    const uint4 *src = reinterpret_cast<const uint4 *>(A.scene + (A.accel_wide ? A.accel_wide : A.accel_nodes));
    uint4 *dst = reinterpret_cast<uint4 *>(g_lds);
    const uint32_t n4 = A.accel_lds_nodes * A.accel_node_u4;
    for (uint32_t i = threadIdx.x; i < n4; i += kBlock) dst[i] = src[i];
    __syncthreads();
  }
  const uint32_t lane = __lane_id();
  const uint32_t wave = threadIdx.x >> 6;
  const uint32_t gtid = blockIdx.x * kBlock + threadIdx.x;
  uint16_t *stk = reinterpret_cast<uint16_t *>(g_lds + A.stack_lds_word) + wave * A.stack_cap * 64 + lane;
  // colour stack (codes, rt_layout.h): level k < rc_lds_levels in LDS, lane-interleaved (conflict-free) —
  // wide: rcw[k * 64]; narrow: two levels per word, rch[(k >> 1) * 128 + (k & 1)] (rc_lds_levels even) —
  // deeper levels in HBM at rc[gtid * max_bounces + k]
  constexpr bool WIDE = (F & kVarNarrow) == 0;
  constexpr bool BYTE = !WIDE && (F & kVarByte) != 0;   // 8-bit codes: four levels per word, rcb[(k >> 2) * 256 + (k & 3)]
  constexpr bool RC_LDS = (F & kVarRcLds) != 0;          // every level in LDS (host-checked): no HBM level code
  const uint32_t mb = static_cast<uint32_t>(A.max_bounces);
  uint32_t *rcw = g_lds + A.rc_lds_word + wave * A.rc_lds_levels * 64 + lane;
  uint16_t *rch = reinterpret_cast<uint16_t *>(g_lds + A.rc_lds_word + wave * (A.rc_lds_levels >> 1) * 64 + lane);
  uint8_t *rcb = reinterpret_cast<uint8_t *>(g_lds + A.rc_lds_word + wave * (A.rc_lds_levels >> 2) * 64 + lane);
  auto rc_lds_store = [&](uint32_t k, uint32_t code) {
    if (WIDE) rcw[k * 64] = code;
    else if (BYTE) rcb[(k >> 2) * 256 + (k & 3)] = static_cast<uint8_t>(code);
    else rch[(k >> 1) * 128 + (k & 1)] = static_cast<uint16_t>(code);
  };
  auto rc_lds_load = [&](uint32_t k) -> uint32_t {
    return WIDE ? rcw[k * 64] : (BYTE ? static_cast<uint32_t>(rcb[(k >> 2) * 256 + (k & 3)])
                                      : static_cast<uint32_t>(rch[(k >> 1) * 128 + (k & 1)]));
  };
  // HBM levels lane-contiguous (rc[gtid * max_bounces + k]): a deep path's successive levels fill the same
  // cache lines, which reach HBM whole instead of as one 4-byte piece per line
  auto rc_at = [&](uint32_t k) -> size_t {
#ifdef RT_RC_INTERLEAVED   // A/B: level-major (rc[k * threads + gtid])
    return static_cast<size_t>(k) * A.threads + gtid;
#else
    return static_cast<size_t>(gtid) * mb + k;
#endif
  };
  auto rc_hbm_store = [&](uint32_t k, uint32_t code) {
    const size_t i = rc_at(k);
    if (WIDE) static_cast<uint32_t *>(A.rc)[i] = code;
    else if (BYTE) static_cast<uint8_t *>(A.rc)[i] = static_cast<uint8_t>(code);
    else static_cast<uint16_t *>(A.rc)[i] = static_cast<uint16_t>(code);
  };
  auto rc_hbm_load = [&](uint32_t k) -> uint32_t {
    const size_t i = rc_at(k);
    return WIDE ? static_cast<const uint32_t *>(A.rc)[i]
                : (BYTE ? static_cast<uint32_t>(static_cast<const uint8_t *>(A.rc)[i])
                        : static_cast<uint32_t>(static_cast<const uint16_t *>(A.rc)[i]));
  };
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  // Deep-level pool (kVarRcPool): levels [rc_lds_levels, mb) of a path go to one of its wave's LDS chunks when one is
  // free at the path's first such push (else to HBM, as without the pool); the chunk returns to the wave's free mask
  // when the path's unwind has read it.  Paths that deep are a few lanes of a wave at a time, so chunks for a fraction of
  // the lanes keep nearly every deep level out of HBM in far fewer LDS bytes than per-lane levels would take.  The mask
  // is wave-private (taken at the push, returned by LDS atomics at the unwind, program-ordered within the wave)
  constexpr bool POOL = !RC_LDS && (F & kVarRcPool) != 0;
  const uint32_t pool_stride = mb > A.rc_lds_levels ? mb - A.rc_lds_levels : 0u;
  uint32_t *const pool = g_lds + __builtin_amdgcn_readfirstlane(A.rc_pool_word + wave * (kRcPoolHead + A.rc_pool_chunks * pool_stride));
  // the lane's chunk (0xff: none) in a byte of the wave's pool header, not in a register carried through the traversal
  uint8_t *const pool_lane = reinterpret_cast<uint8_t *>(pool + 1) + lane;
  if (POOL) {
    if (lane == 0) pool[0] = A.rc_pool_chunks >= 32u ? 0xffffffffu : (1u << A.rc_pool_chunks) - 1u;
    *pool_lane = 0xffu;
    __threadfence_block();
  }
  auto rc_deep_store = [&](uint32_t k, uint32_t code) {
    if (!RT_CHECK(A, k < mb, CHK_RC_DEEP, k, mb)) return;
    if constexpr (POOL) {
      const uint32_t c = *pool_lane;
      if (c != 0xffu) {
        if (RT_CHECK(A, c < A.rc_pool_chunks, CHK_POOL_CHUNK, c, A.rc_pool_chunks))
          pool[kRcPoolHead + c * pool_stride + (k - A.rc_lds_levels)] = code;
        return;
      }
    }
    rc_hbm_store(k, code);
  };
  auto rc_deep_load = [&](uint32_t k) -> uint32_t {
    if constexpr (POOL) {
      const uint32_t c = *pool_lane;
      if (c != 0xffu) return pool[kRcPoolHead + c * pool_stride + (k - A.rc_lds_levels)];
    }
    return rc_hbm_load(k);
  };

  bool busy = false;                      // lane owns a pixel
  bool hot = false;                       // the pixel is one of the first A.prio_ids handed out
  uint32_t prio_now = 0;                  // wave-uniform: the s_setprio level in force
  uint32_t pxy = 0;                       // the pixel: local row << 16 | column (rt_capi.cpp: both < 65536)
  int32_t sample = 0;
  uint32_t depth = 0;                     // bounces of the current path (max_bounces, :1336)
  uint32_t rsp = 0;                       // colour-stack levels pushed (dielectric bounces push none)
  Rng rng{0, 0, 0, 0, 0, 0};
  Ray ray;
  ray.o = mk(0, 0, 0); ray.d = mk(0, 0, 0); ray.time = 0;
  f3 sum = mk(0, 0, 0);
  // kParkSum traces: the sum lives in the lane's stack entries stack_cap - kSumEntries .. stack_cap - 1 (u16 halves)
  constexpr bool kParkS = park_sum<Trace>(0);
  auto sum_put = [&](const f3 &v) {
    if constexpr (kParkS) {
      uint16_t *e = stk + (A.stack_cap - kSumEntries) * 64u;
      const uint32_t w[3] = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z)};
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        e[(2 * i) * 64] = static_cast<uint16_t>(w[i]);
        e[(2 * i + 1) * 64] = static_cast<uint16_t>(w[i] >> 16);
      }
      asm volatile("" ::: "memory");   // reloaded from LDS, not kept in registers
    } else {
      sum = v;
    }
  };
  auto sum_get = [&]() -> f3 {
    if constexpr (kParkS) {
      const uint16_t *e = stk + (A.stack_cap - kSumEntries) * 64u;
      float f[3];
#pragma unroll
      for (int i = 0; i < 3; ++i)
        f[i] = __uint_as_float(static_cast<uint32_t>(e[(2 * i) * 64]) | (static_cast<uint32_t>(e[(2 * i + 1) * 64]) << 16));
      return mk(f[0], f[1], f[2]);
    } else {
      return sum;
    }
  };
  Trav T;
  T.inv = mk(0, 0, 0); T.rcp = mk(0, 0, 0); T.tmax = 0; T.active = 0; T.anode = 0; T.abest = 0; T.atie = 0; T.asp = 0; T.sp = 0; T.tc = 0; T.yc = 0; T.was_last = 0; T.result = false;
  Hit h;
  h.u = 0; h.v = 0; h.t = 0; h.fd = 0; h.mat = 0; h.p = mk(0, 0, 0); h.n = mk(0, 0, 0);
  Visits vc{};
  uint32_t c_bounce = 0, c_shade = 0, c_perlin = 0, c_samples = 0;

  uint32_t chunk_pos = 0, chunk_end = 0;   // wave-uniform: ids of the wave's current tile
  // the wave's slot: a wave-uniform base (scalar registers; threadIdx.x >> 6 is not known to be uniform) and
  // 32-bit per-lane offsets
  // the wave's RNG slot in LDS (32-bit words, one per lane and state word)
  uint32_t *const rng_slot = g_lds + A.rng_slot_word + wave * kRngSlotWords;
  // tiles: tw = 1 << ts pixels wide, 64 / tw = 1 << tsh tall (pixel k of a tile at row k >> ts, column k & (tw - 1))
  constexpr uint32_t kTs = (static_cast<uint32_t>(F) >> kVarTileShift) & 7u;   // 0: the offline kernels read it
  const uint32_t ts = kTs ? kTs : A.tile_shift, tsh = 6u - ts, twm = (1u << ts) - 1u;
  constexpr bool STAGE = (F & kVarStage) != 0;
  // Output staging (coalesced tile writes to the HBM frame): a whole tile handed to a wave takes the wave's next
  // staging slot if it is free (else its pixels are stored when they end, as before).  A lane whose pixel ends parks
  // its floats in the slot (pixel k at 3 k) and sets bit k of the slot's done mask; the lane that sets the last bit
  // flags the slot, and at the top of the next round — every lane of the wave active — the wave stores the tile:
  // lane l writes floats l, l + 64, l + 128 of the tile, so each store instruction covers a contiguous run of a tile
  // row (a 32-pixel row of a 32-aligned frame: three whole 128-B lines), and the PPM bytes of the same floats
  // (pixels_to_ppm, fused) likewise.  A lane finds its pixel's slot by the tile id in the slot headers, so nothing
  // but the one-word "slot complete" flag is carried through the traversal.
  const uint32_t n_stage = (!STAGE || probe || A.out == nullptr) ? 0u : A.stage_slots;   // wave-uniform
  uint32_t *const stage = g_lds + __builtin_amdgcn_readfirstlane(A.stage_word + wave * (A.stage_slots * kStageSlotWords + 2u));
  uint32_t stage_next = 0;                 // wave-uniform: the slot the next whole tile may take
  // the wave's "slot complete" bits (bit q: slot q's last pixel ended), an LDS word after the slots: set by the lane that
  // completes a tile, read once per round (no per-lane register carried through the traversal)
  uint32_t *const stage_done = stage + A.stage_slots * kStageSlotWords;
  if (n_stage != 0u) {
    if (lane < n_stage) stage[lane * kStageSlotWords + kStageTile] = kStageFree;
    if (lane == 0) *stage_done = 0u;
    __threadfence_block();
  }
  // the tiles whose last pixel has ended are stored (whole lines per store instruction); every lane of the wave, at a
  // tile pickup and once the wave's last pixel has ended (no per-round check: nothing is carried through the traversal)
  auto stage_store = [&]() {
    uint32_t fm = __builtin_amdgcn_readfirstlane(*stage_done);
    if (fm == 0) return;
    // the lane id through a volatile asm: the per-lane entry indices below stay inside this rarely run block instead
    // of being hoisted out of the render loop (registers live across the whole traversal)
    uint32_t ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
    __threadfence_block();   // the floats parked and the done bits set before come first
    if (ln == 0) *stage_done = 0u;
    while (fm != 0) {
      const uint32_t q = static_cast<uint32_t>(__builtin_ctz(fm));
      fm &= fm - 1u;
      uint32_t *const sq = stage + q * kStageSlotWords;
      const uint32_t tile = __builtin_amdgcn_readfirstlane(sq[kStageTile]);
      // (readfirstlane returns an int: widened without the cast, the low word's bit 31 would sign-extend into the high
      // word and mark a partial tile's missing rows valid)
      const uint64_t valid = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(sq[kStageValid + 1]))) << 32) |
                             static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(sq[kStageValid]));
      const uint32_t ty = tile / A.tiles_x, tx = tile - ty * A.tiles_x;
      const uint32_t lr0 = ty << tsh, j0 = tx << ts;
      const float *sf = reinterpret_cast<const float *>(sq);
#pragma unroll
      for (uint32_t i = 0; i < 3; ++i) {
        const uint32_t e = ln + 64u * i, k = e / 3u, comp = e - 3u * k;
        if ((valid >> k) & 1ull) {
          const size_t pix = static_cast<size_t>(lr0 + (k >> ts)) * static_cast<uint32_t>(A.width) + j0 + (k & twm);
          const float v = sf[e];
          A.out[3 * pix + comp] = v;
          if (A.out8) A.out8[3 * pix + comp] = ppm_byte(v);
        }
      }
      __threadfence_block();   // the slot's reads above come before its release
      if (ln == 0) sq[kStageTile] = kStageFree;
    }
  };
  // XCD classes (A.cls_off): the wave's XCD, the queue it draws from (lane 0's count of drained queues) and the rank
  // in its class of the chunk being handed out
  const uint32_t xcd = A.cls_off ? (__builtin_amdgcn_s_getreg(20 | (15 << 11)) & (kXcdClasses - 1u)) : 0u;   // HW_REG_XCC_ID
  uint32_t cls_step = 0;
  bool chunk_hot = false;
  bool exhausted = false;
  bool prio_done = false;                  // wave-uniform: the split costliest tiles are all handed out
  uint32_t tiles_taken = 0, rounds = 0;
  uint32_t probe_tile = 0, probe_rounds = 0;
  bool probe_end = false;                  // probe: the lane's path ended in the last round
  uint64_t ph_refill = 0, ph_trace = 0, ph_rej = 0, ph_mat = 0, ph_shade = 0, ph_unwind = 0, ph_cam = 0, t_mark = 0;   // wave-trace clocks
  uint64_t busy_lane_rounds = 0;
  uint64_t ph_noise = 0, lph_noise = 0;                     // wave trace: cooperative noise (part of mat)
  uint64_t lph[7] = {0, 0, 0, 0, 0, 0, 0}, lone_rounds = 0;   // wave trace: the same phases over the rounds
  bool lone = false;                                         // with at most 2 busy lanes (the frame's tail)
  const uint64_t t_start = TRACE ? __builtin_amdgcn_s_memrealtime() : 0;

  uint32_t pending = 0;   // 1: the lane's rejection sampling continues next round (A.max_tries)
  float random_test = 0.0f;
  constexpr bool kParkRt = park_random_test<Trace>(0);   // random_test parked in the lane's LDS stack
  const uint32_t try_cap = A.max_tries ? A.max_tries : 0xffffffffu;
  // the pixel's viewport point (:1565-1567), recomputed per sample from pxy (a few ops and no division; three
  // fewer registers carried across the trace)
  // the camera's arguments (once per sample) and the tile / pixel pickup's (once per tile) are read where used (kargs):
  // held, they pushed the render loop's own SGPRs into VGPR lanes — scene 0 27 -> 7 spilled SGPRs, Perlin 120 -> 52
  auto cam = [&]() { return kargs(A); };
  auto pixel_point = [&]() -> f3 {
    const int32_t lr = static_cast<int32_t>(pxy >> 16), j = static_cast<int32_t>(pxy & 0xffffu);
    const int32_t i = A.row_offset + lr * A.row_stride;
    const auto C = cam();
    return add(mk(C->p00[0], C->p00[1], C->p00[2]),
             add(scale(static_cast<float>(i), mk(C->dv[0], C->dv[1], C->dv[2])),
                 scale(static_cast<float>(j), mk(C->du[0], C->du[1], C->du[2]))));
  };
  // the scene-specialised kernels (register room at 72-85 VGPRs) keep the point from the pixel's pickup instead of
  // recomputing it for every sample; the walks at a register budget (the verified sphere walk's 80, the mixed
  // walk's 160) recompute it (a few ops, no division)
  constexpr bool kCarryPoint = carry_point<Trace>(0);
  f3 pp = mk(0, 0, 0);
  auto camera_ray = [&]() {                                                 // :1561-1578
    const auto C = cam();
    if (C->defocus_angle <= 0) {
      ray.o = mk(C->center[0], C->center[1], C->center[2]);
    } else {                                                                // :1459-1476
      float x, y;
      for (;;) {
        y = rng.sym();    // bound(-1, 1); Vec3(x(), y(), 0): y drawn first
        x = rng.sym();
        float l = sqrtf(x * x + y * y + 0.0f * 0.0f);
        if (l * l < 1.0f) break;
      }
      f3 c = mk(C->center[0], C->center[1], C->center[2]);
      f3 u = mk(C->dfu[0], C->dfu[1], C->dfu[2]), v = mk(C->dfv[0], C->dfv[1], C->dfv[2]);
      ray.o = add(c, add(scale(x, u), scale(y, v)));
    }
    float xo = rng.uniform() - 0.5f;
    float yo = rng.uniform() - 0.5f;
    ray.d = sub(kCarryPoint ? pp : pixel_point(), ray.o);
    const auto D = cam();
    ray.d = add(ray.d, scale(xo, mk(D->du[0], D->du[1], D->du[2])));
    ray.d = add(ray.d, scale(yo, mk(D->dv[0], D->dv[1], D->dv[2])));
    ray.time = rng.uniform();
    depth = 0;
    rsp = 0;
  };

  for (;;) {
    if (TRACE) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if (t_mark) { ph_shade += t - t_mark; if (lone) lph[2] += t - t_mark; }
      t_mark = t;
    }
    if (probe) {
      // the lanes whose probe path ended last round add their rounds to their tile's cost: one atomic per
      // tile, the rounds summed across the wave first (all lanes are active here)
      uint64_t left = __ballot(probe_end);
      while (left) {
        const int leader = __builtin_ctzll(left);
        const uint32_t t = __builtin_amdgcn_readfirstlane(__shfl(probe_tile, leader));
        const bool mine = probe_end && probe_tile == t;
        uint32_t v = mine ? probe_rounds : 0u;
#pragma unroll
        for (int sh = 1; sh < 64; sh <<= 1) v += __shfl_xor(v, sh);
        if (lane == static_cast<uint32_t>(leader)) atomicAdd(A.probe_cost + t, v);
        left &= ~__ballot(mine);
      }
      probe_end = false;
    }
    // ---- lanes without a pixel take the next pixels of the wave's tile ----
    bool need = !busy;
    uint64_t m = __ballot(need);
    // sparse hot waves (A.prio_lanes < 64, split hand-out only): a wave holding pixels of the costliest
    // tiles takes at most prio_lanes of them and no other pixel until they are done, so the longest pixel
    // chains run in waves with few divergent lanes (the idle lanes share their noise octaves)
    const bool sparse = A.prio_lanes < static_cast<uint32_t>(kChunk);
    uint32_t nhot = sparse ? static_cast<uint32_t>(__popcll(__ballot(busy && hot))) : 0u;
    while (m != 0 && !exhausted) {
      const auto K = cam();   // tile / pixel pickup: kernel arguments read here (see cam)
      if (chunk_pos >= chunk_end) {
        if (n_stage != 0u) stage_store();   // the wave's finished tiles first (their slots become free)
        if (sparse && !K->prio_mix && (nhot >= K->prio_lanes || (nhot > 0 && prio_done))) break;
        // the costliest tiles (the first prio_ids ids of the longest-first order) may be handed out in
        // prio_chunk-pixel pieces from their own counter, so that their long pixel chains spread over
        // more waves; every other tile goes out whole.  Mixed (K->prio_mix): a wave holding prio_lanes of
        // those pixels takes ordinary tiles for its other lanes meanwhile.
        uint32_t base = 0, size = static_cast<uint32_t>(kChunk), hold = 0;
        const bool capped = K->prio_mix && nhot >= K->prio_lanes;
        const bool split = K->prio_chunk < static_cast<uint32_t>(kChunk) && !prio_done && !capped;
        if (lane == 0) {
          if (split) base = atomicAdd(K->work + 1, K->prio_chunk);
          if (!split || base >= K->prio_ids) {
            if (sparse && !K->prio_mix && nhot > 0) hold = 1;   // the last costly pixels are out: stay sparse
            else if (!K->cls_off) {
              base = atomicAdd(K->work, static_cast<uint32_t>(kChunk)) + (K->prio_chunk < static_cast<uint32_t>(kChunk) ? K->prio_ids : 0u);
              // the last tail_ids ids of the order go out in tail_chunk-pixel pieces from their own counter: a wave
              // then holds at most tail_chunk - 1 pixels it has not started when the queue drains, instead of up to 63
              // of a whole tile, so the waves' last pixels start (and the waves end) closer together
              if ((F & kVarTail) != 0 && K->tail_ids != 0u && base >= K->n_ids - K->tail_ids) {
                base = K->n_ids - K->tail_ids + atomicAdd(K->work + kTailWord, K->tail_chunk);
                size = K->tail_chunk;
              }
            }
          } else {
            size = K->prio_chunk;
          }
        }
        if (K->cls_off) {
          // XCD classes (whole tiles only): this wave's XCD queue — tiles whose frame lines no other XCD writes, so the
          // XCD's L2 merges their partial lines into whole ones — then, once it is drained, the other queues in turn.
          // Wave-uniform (scalar registers); lane 0 takes the ids
          for (;;) {
            const uint32_t q = (xcd + cls_step) & (kXcdClasses - 1u);
            const uint32_t lo = K->cls_off[q], hi = K->cls_off[q + 1];   // positions in the tile order
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(K->work + kClsWord + q, static_cast<uint32_t>(kChunk));
            b = __builtin_amdgcn_readfirstlane(b);
            if (b < (hi - lo) * static_cast<uint32_t>(kChunk)) {
              base = lo * static_cast<uint32_t>(kChunk) + b;
              // the chunk is among the costliest if its rank in its class is (each class holds ~1/8 of them)
              chunk_hot = b < K->prio_ids / kXcdClasses;
              break;
            }
            if (++cls_step == kXcdClasses) { base = K->n_ids; break; }
          }
        }
        base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
        size = __builtin_amdgcn_readfirstlane(__shfl(size, 0));
        hold = __builtin_amdgcn_readfirstlane(__shfl(hold, 0));
        if (size == static_cast<uint32_t>(kChunk) && !capped) prio_done = true;
        if (hold) break;
        // a capped mixed wave that finds the ordinary tiles gone waits for a hot lane to free (costly
        // pixels may still be queued); the queue is exhausted only when both counters are drained
        if (base >= K->n_ids) { if (!capped) exhausted = true; break; }
        if (K->reverse_tiles) base = K->n_ids - kChunk - base;   // whole tiles: n_ids is a multiple of 64
        tiles_taken++;
        chunk_pos = base;
        chunk_end = min(base + size, K->n_ids);
        if (!probe) {
          // RNG seeding of the chunk (init_gpu_data's curand_init, :1591-1606, subsequence = global pixel index
          // i * W + j): lane l takes id base + l, starts from the phase base of its pixel (the row's state jumped
          // over the column's low 3 bits, host) and applies the column table of its tile column (J^(8 (j >> 3))):
          // one nibble-table product per lane, the same table across the wave; the states wait in the wave's
          // slot for the lanes that take those pixels
          const uint32_t id = base + lane;
          uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0, x4 = 0, tcol = 0;
          uint32_t tile = id >> 6;
          bool valid = false;
          if (id < chunk_end) {
            const uint32_t kk = id & 63u;
            if (K->tile_order) tile = K->tile_order[tile];
            const uint32_t ty = tile / K->tiles_x, tx = tile - ty * K->tiles_x;
            const uint32_t lr = (ty << tsh) + (kk >> ts), j = (tx << ts) + (kk & twm);
            if (lr < K->rows && j < static_cast<uint32_t>(K->width)) {
              // phase base of (lr, j & (tw - 1)) and the column table of J^(tw (j >> ts)): one table per tile
              const uint32_t *pb = K->rng_rows + ((lr << ts) + (j & twm)) * 8;
              const uint4 rb = *reinterpret_cast<const uint4 *>(pb);
              x0 = rb.x; x1 = rb.y; x2 = rb.z; x3 = rb.w; x4 = pb[4];
              tcol = j >> ts;
              valid = true;
            }
          }
          // a whole tile takes the wave's next staging slot if that slot is free (else it is stored pixel by pixel)
          if (n_stage != 0u && size == static_cast<uint32_t>(kChunk)) {
            uint32_t *const sq = stage + stage_next * kStageSlotWords;
            const uint64_t vm = __ballot(valid);
            if (__builtin_amdgcn_readfirstlane(sq[kStageTile]) == kStageFree && vm != 0) {
              if (lane == 0) {
                sq[kStageDone] = 0u; sq[kStageDone + 1] = 0u;
                sq[kStageValid] = static_cast<uint32_t>(vm); sq[kStageValid + 1] = static_cast<uint32_t>(vm >> 32);
                sq[kStageTile] = __builtin_amdgcn_readfirstlane(tile);
              }
              stage_next = stage_next + 1u == n_stage ? 0u : stage_next + 1u;
            }
          }
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(K->rng_nib), 0,
                                                                              0x7fffffff, 0x00020000);
          // two table products (J^(tw (t & 15)), then J^(16 tw (t >> 4))): 16 + W / (16 tw) tables in all, so each
          // XCD's L2 fetches a few hundred KB of them instead of every column group's table
          rng_jump_nib(rs, (tcol & (kRngColLo - 1u)) * kRngNibTableWords * 4u, x0, x1, x2, x3, x4);
          rng_jump_nib(rs, (kRngColLo + (tcol >> kRngColLoBits)) * kRngNibTableWords * 4u, x0, x1, x2, x3, x4);
          // slot entry id & 63: a chunk is size-aligned (whole tiles, or prio_chunk pieces, a power of two <= 64),
          // so its ids take distinct entries and no chunk base is kept across rounds
          const uint32_t so = id & 63u;
          rng_slot[so] = x0;
          rng_slot[64u + so] = x1;
          rng_slot[128u + so] = x2;
          rng_slot[192u + so] = x3;
          rng_slot[256u + so] = x4;
          __threadfence_block();   // the stores reach the wave's later loads of other lanes' entries
        }
      }
      const uint32_t avail = chunk_end - chunk_pos;
      const uint32_t rank = __popcll(m & lt_mask);
      if (need && rank < avail) {
        // tile-major id -> (local row, column); ids past the shard edge are skipped
        const uint32_t id = chunk_pos + rank;
        uint32_t tile, k, salt = 0;
        if (probe) {                        // probe: probe_per_tile paths spread over the tile's pixels
          tile = id / K->probe_per_tile;
          const uint32_t q = id - tile * K->probe_per_tile;
          k = (q * 37u + 11u) & 63u;        // a permutation of the 64 pixels per 64 paths
          salt = q >> 6;                    // more than 64 paths per tile: another stream per pixel
        } else {
          tile = id >> 6;
          k = id & 63u;
          if (K->tile_order) tile = K->tile_order[tile];
        }
        const uint32_t ty = tile / K->tiles_x, tx = tile - ty * K->tiles_x;
        const uint32_t lr = (ty << tsh) + (k >> ts), j = (tx << ts) + (k & twm);
        if (lr < K->rows && j < static_cast<uint32_t>(K->width)) {
          pxy = (lr << 16) | j;
          if constexpr (kCarryPoint) pp = pixel_point();
          need = false;
          busy = true;
          hot = K->cls_off ? chunk_hot : id < K->prio_ids;
          if (probe) {                      // throwaway stream: the real ones are not consumed
            probe_tile = tile;
            probe_rounds = 0;
            uint32_t hsh = (lr * static_cast<uint32_t>(K->width) + j) * 0x9E3779B9u + 0x7F4A7C15u + salt * 0x632BE5ABu;
            hsh ^= hsh >> 16; hsh *= 0x85EBCA6Bu; hsh ^= hsh >> 13; hsh *= 0xC2B2AE35u; hsh ^= hsh >> 16;
            rng.d = hsh; rng.x0 = hsh ^ 0x2c7f967fu; rng.x1 = hsh * 3u + 1u; rng.x2 = ~hsh;
            rng.x3 = hsh ^ 0xa03697cbu; rng.x4 = hsh | 1u;
          } else {
            // the state seeded at the chunk's pickup (the slot entry of this id)
            const uint32_t so = id & 63u;
            rng.d = K->rng_d;
            rng.x0 = rng_slot[so];
            rng.x1 = rng_slot[64u + so];
            rng.x2 = rng_slot[128u + so];
            rng.x3 = rng_slot[192u + so];
            rng.x4 = rng_slot[256u + so];
          }
          sum_put(mk(0, 0, 0));
          sample = 0;
          camera_ray();
        }
      }
      chunk_pos += min(static_cast<uint32_t>(__popcll(m)), avail);
      m = __ballot(need);
      if (sparse) nhot = static_cast<uint32_t>(__popcll(__ballot(busy && hot)));
    }
    const uint64_t lanes = __ballot(busy);
    if (lanes == 0) break;   // queue exhausted and every lane idle
    // the slowest pixels bound the frame (a pixel's samples form one serial chain): waves holding
    // pixels of the costliest tiles get issue priority over the waves that have slack
    uint32_t want_prio = __ballot(busy && hot) != 0 ? 2u : 0u;
    // once the queue is drained the frame ends with the wave whose pixel has the most samples left; the
    // SIMD's arbiter otherwise favours the oldest waves (measured: 20 vs 28 us per round, first vs third
    // wave of a SIMD on the 10k scene), so the level grows with the least advanced pixel's remaining share
    if (A.tail_prio && exhausted) {
      // the level of the wave's largest remaining share, by ballots (each threshold holds for the maximum iff it holds
      // for some lane; no cross-lane shuffle, whose lane addresses the compiler would keep live across the loop)
      const uint32_t rem = busy ? static_cast<uint32_t>(A.spp - sample) : 0u, spp = static_cast<uint32_t>(A.spp);
      const uint32_t lvl = __ballot(4u * rem > 3u * spp) != 0 ? 3u
                         : __ballot(2u * rem > spp) != 0 ? 2u
                         : __ballot(4u * rem > spp) != 0 ? 1u : 0u;
      want_prio = max(want_prio, lvl);
    }
    if (want_prio != prio_now) {
      if (want_prio == 3u) __builtin_amdgcn_s_setprio(3);
      else if (want_prio == 2u) __builtin_amdgcn_s_setprio(2);
      else if (want_prio == 1u) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      prio_now = want_prio;
    }
    rounds++;
    busy_lane_rounds += static_cast<uint64_t>(__popcll(lanes));
    if (TRACE) {
      lone = __popcll(lanes) <= 2;
      lone_rounds += lone ? 1u : 0u;
    }
    if (TRACE) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph_refill += t - t_mark; if (lone) lph[0] += t - t_mark;
      t_mark = t;
    }

    // ---- trace one path segment per busy lane (hit(), :1340) ----
    const bool tracing = busy && !pending;   // a lane still resuming its rejection keeps its hit
    if constexpr (RT_PRIM_LISTS && prim_lists<Trace>(0)) {
      // a camera ray (no bounce yet, no paused walk) of a shard with candidate lists: its tile's list
      T.atie = 0u;
      if (A.prim_lists && tracing && depth == 0u && !T.active) {
        T.atie = (pxy >> (16u + tsh)) * A.tiles_x + ((pxy & 0xffffu) >> ts) + 1u;
      }
    }
    Trace::template run<LDS, COUNT, UV>(S, A, tracing, __ballot(tracing), lane, stk, T, ray, h, vc);
    if (T.active) continue;                   // walk paused (verified traversal): resumes next round
    if constexpr (lazy_hit<Trace>(0)) Trace::template materialize<LDS, UV>(S, A, T, ray, h);
#ifdef RT_DBG_PX   // diagnostics only (RT_JIT_OPTS=-DRT_DBG_PX=<row << 16 | column>): one pixel's path segments
    if (tracing && pxy == static_cast<uint32_t>(RT_DBG_PX))
      printf("dbg s %d d %u res %d t %08x best %08x o %08x %08x %08x dir %08x %08x %08x rng %08x\n", sample, depth,
             T.result ? 1 : 0, __float_as_uint(T.tmax), T.abest, __float_as_uint(ray.o.x), __float_as_uint(ray.o.y),
             __float_as_uint(ray.o.z), __float_as_uint(ray.d.x), __float_as_uint(ray.d.y), __float_as_uint(ray.d.z), rng.x4);
#endif
    if (TRACE) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph_trace += t - t_mark; if (lone) lph[1] += t - t_mark;
      t_mark = t;
    }
    // ---- shade (ray_color loop body, :1340-1359); in noise kernels lanes without a pixel stay to help
    // the cooperative noise evaluation below ----
    if (!COOP && !busy) continue;
    bool done = false;
    f3 res = mk(0, 0, 0);
    f3 ruv = mk(0, 0, 0);
    if (busy) probe_rounds++;
    if (busy && T.result) {
      // cuda_material_scatter: random_test first, then the unit vector by rejection, drawn (z, y, x)
      // (:497-502, vec3.h:152-161) — for every material, lights included.  With A.max_tries > 0 a lane
      // whose tries all fail keeps its hit and resumes the rejection next round (skipping that round's
      // traversal), so one unlucky lane no longer holds the whole wave in this loop.
      if (!pending) {
        if (COUNT) c_shade++;
        const float rtv = rng.uniform();
        if constexpr (kParkRt) {   // two u16 stack entries of the lane (the clobber: reloaded, not kept in registers)
          stk[0] = static_cast<uint16_t>(__float_as_uint(rtv));
          stk[64] = static_cast<uint16_t>(__float_as_uint(rtv) >> 16);
          asm volatile("" ::: "memory");
        } else {
          random_test = rtv;
        }
      }
      // Wave-uniform loop: one try per iteration for every lane still rejecting.  It ends when no
      // lane needs a try, after try_cap tries, or once at most A.defer_lanes lanes are left (those
      // resume next round): the wave no longer runs the maximum of 64 geometric try counts.
      bool want = true;
      // deferring only pays when the lanes that accepted outnumber the pending ones: a nearly empty
      // wave (the tail of the frame) keeps trying rather than spending a round per try
      const uint32_t started = static_cast<uint32_t>(__popcll(__ballot(true)));
      for (uint32_t k = 0;;) {
        if (want) {
          float z = rng.sym();   // bound(-1, 1)
          float y = rng.sym();
          float x = rng.sym();
          // accept iff fl(fl(sqrt(s))^2) in (0, 1] (vec3.h:152-161, `1e-50 < len2` == `len2 > 0`).
          // Decided on s itself except within 2^-20 of 1: s in (0, 1-2^-20] always passes, s >= 1+2^-20
          // always fails (components are 0 or >= 2^-31 in magnitude, so s > 0 => len2 > 0); the sqrt and
          // the division run once, after the loop, instead of on every try of every lane.
          const float s2 = x * x + y * y + z * z;
          bool acc = s2 > 0.0f && s2 <= 0.99999904632568359375f;           // 1 - 2^-20
          const bool near1 = s2 > 0.99999904632568359375f && s2 < 1.00000095367431640625f;
          if (__ballot(near1) != 0) {   // wave-uniform branch: keeps the rare exact test out of the loop
            asm volatile("" ::: "memory");   // not speculated (the compiler would if-convert the sqrt)
            const float l = sqrtf(s2);
            if (near1) acc = l * l <= 1.0f;
          }
          if (acc) { ruv = mk(x, y, z); want = false; }
        }
        const uint64_t left = __ballot(want);
        const uint32_t nleft = static_cast<uint32_t>(__popcll(left));
        if (left == 0 || ++k == try_cap || (nleft <= A.defer_lanes && 4 * nleft <= started)) break;
      }
      pending = want ? 1u : 0u;
    }
    if (TRACE) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph_rej += t - t_mark; if (lone) lph[4] += t - t_mark;
      t_mark = t;
    }
    // ---- cooperative noise (kernels with noise textures): a lane shading a Lambertian noise texture
    // spends most of its round in the 7 octaves of perlin_turbulence — a trapped-path straggler, alone
    // on its SIMD at the end of the frame, issues them one after the other.  When at most half of the
    // wave needs one, the octaves are spread over 2, 4 or 8 lanes per noise lane (coop_noise_code) ----
    bool coop = false;
    uint32_t coop_code = 0;
    const uint64_t t_noise0 = TRACE ? __builtin_amdgcn_s_memtime() : 0;
    if (COOP && !COUNT && (TM & (1u << T_NOISE))) {
      bool nz = false;
      uint32_t ntb = 0;
      float nsc = 0.0f;
      if (busy && T.result && !pending) {
        const uint4 mm = S.w4(A.off_mats + h.mat * kMatWords);
        if (mm.x == MAT_LAMBERTIAN) {
          const uint4 t0 = S.w4(A.off_texs + mm.y * kTexWords);
          if (t0.x == T_NOISE) { nz = true; ntb = A.off_perlin + t0.y * kPerlinWords; nsc = asf(t0.w); }
        }
      }
      const uint64_t nm = __ballot(nz);
      const uint32_t nb = static_cast<uint32_t>(__popcll(nm));
      if (nb != 0 && nb <= A.coop_noise && __ballot(true) == ~0ull) {
        // (the 2-lane share costs 17 VGPRs, 4 -> 3 waves/SIMD, and still wins 3 % on scenes 17 and 19)
        if (nb <= 8) coop_code = coop_noise_code<8>(S, A, nm, lane, lt_mask, h.p, ntb, nsc);
        else if (nb <= 16) coop_code = coop_noise_code<4>(S, A, nm, lane, lt_mask, h.p, ntb, nsc);
        else coop_code = coop_noise_code<2>(S, A, nm, lane, lt_mask, h.p, ntb, nsc);
        coop = nz;
      }
    }
    if (TRACE) {   // the cooperative noise block's share of the material phase
      const uint64_t dt = __builtin_amdgcn_s_memtime() - t_noise0;
      ph_noise += dt;
      if (lone) lph_noise += dt;
    }
    if (busy && T.result && !pending) {
      const uint32_t mbase = A.off_mats + h.mat * kMatWords;
      const uint4 m0 = S.w4(mbase), m1 = S.w4(mbase + 4);
      const uint32_t mkind = m0.x;
      f3 emit = mk(0, 0, 0);
      if ((MM & (1u << MAT_DIFFUSE_LIGHT)) && mkind == MAT_DIFFUSE_LIGHT)
        emit = texture_color<LDS, COUNT, NOISE, UV, TM>(S, A, m0.y, h.u, h.v, h.p, c_perlin);
      ruv = scale(1.0f / length(ruv), ruv);
      bool scattered = false;
      bool push = false;        // dielectrics push no level: their attenuation (1,1,1) is x*1 == x
      uint32_t code = 0;        // colour-stack code of the attenuation (rt_layout.h)
      f3 dir = mk(0, 0, 0);
      const bool hfront = hit_front(h);
      const f3 hn = hfront ? h.n : flip(h.n);
      if ((MM & (1u << MAT_LAMBERTIAN)) && mkind == MAT_LAMBERTIAN) {      // :458-465
        scattered = true;
        push = true;
        dir = add(hn, ruv);
        const float eps = 1e-8f;
        if (fabsf(dir.x) < eps && fabsf(dir.y) < eps && fabsf(dir.z) < eps) dir = hn;
        code = coop ? coop_code : texture_code<LDS, COUNT, NOISE, UV, TM, WIDE>(S, A, m0.y, h.u, h.v, h.p, c_perlin);
      } else if ((MM & (1u << MAT_METAL)) && mkind == MAT_METAL) {         // :466-472
        f3 rd = sub(ray.d, scale(2.0f * dot(ray.d, hn), hn));
        dir = add(unit(rd), scale(asf(m1.y), ruv));
        code = rc_rec(h.mat, WIDE);                                         // albedo: the material record
        scattered = dot(dir, hn) > 0;
        push = true;
      } else if ((MM & (1u << MAT_DIELECTRIC)) && mkind == MAT_DIELECTRIC) {   // :473-487
        const float ior = asf(m1.z);
        const float ri = hfront ? (1.0f / ior) : ior;
        const f3 ud = unit(ray.d);
        const float cos_t = fminf(dot(flip(ud), hn), 1.0f);
        const float sin_t = sqrtf(1.0f - cos_t * cos_t);
        bool reflect_it = ri * sin_t > 1.0f;
        if (!reflect_it) {
          float r0 = (1.0f - ri) / (1.0f + ri);
          r0 = r0 * r0;
          float rtest = random_test;
          if constexpr (kParkRt) rtest = __uint_as_float(static_cast<uint32_t>(stk[0]) | (static_cast<uint32_t>(stk[64]) << 16));
          reflect_it = (r0 + (1.0f - r0) * rt_pow5f(1.0f - cos_t)) > rtest;
        }
        if (reflect_it) {
          dir = sub(ud, scale(2.0f * dot(ud, hn), hn));
        } else {                                                            // refract (:416-422)
          float ct = fminf(dot(flip(ud), hn), 1.0f);
          f3 perp = scale(ri, add(ud, scale(ct, hn)));
          float pl = length(perp);
          f3 par = scale(-sqrtf(fabsf(1.0f - pl * pl)), hn);
          dir = add(perp, par);
        }
        scattered = true;
      }
      if (scattered) {
        // push the attenuation's code (the emission pushed with it is always 0: only lights emit and
        // lights never scatter, raytracing.cu:439-450 vs :457-488, so the unwind adds +0.0f per level)
        if (push) {
          if (RC_LDS || rsp < A.rc_lds_levels) {
            if (RT_CHECK(A, rsp < A.rc_lds_levels, CHK_RC_LDS, rsp, A.rc_lds_levels)) rc_lds_store(rsp, code);
          } else {
            if constexpr (POOL) {
              // the lanes starting their first deep level this round take the lowest free chunks, one each in lane order
              const bool first = rsp == A.rc_lds_levels;
              const uint64_t need = __ballot(first);
              if (need != 0) {
                // scalar loop over the needing lanes (few per round): lane l takes the lowest free chunk
                uint32_t fm = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(pool[0]));
                uint64_t nm = need;
                while (nm != 0 && fm != 0) {
                  const uint32_t l = static_cast<uint32_t>(__builtin_ctzll(nm));
                  if (lane == l) *pool_lane = static_cast<uint8_t>(__builtin_ctz(fm));
                  nm &= nm - 1ull;
                  fm &= fm - 1u;
                }
                pool[0] = fm;   // (every active lane stores the same word)
              }
            }
            rc_deep_store(rsp, code);
          }
#ifdef RT_DBG_PX
          if (pxy == static_cast<uint32_t>(RT_DBG_PX)) printf("dbgp s %d d %u rsp %u code %08x\n", sample, depth, rsp, code);
#endif
          rsp++;
        }
        depth++;
        if (COUNT) c_bounce++;
        ray.o = h.p;
        ray.d = dir;
        if (depth == mb) { done = true; res = mk(0, 0, 0); }           // max_bounces exhausted: black
      } else {
        done = true;
        res = emit;
      }
    } else if (busy && !T.result) {
      done = true;
      res = mk(A.bg[0], A.bg[1], A.bg[2]);
    }
    if (TRACE) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph_mat += t - t_mark; if (lone) lph[3] += t - t_mark;
      t_mark = t;
    }
    if (done) {
      // res = att_k * res + 0.0f from the deepest level (:1362-1368).  With res = (+-0,+-0,+-0) and
      // finite attenuations every level yields +0, so such paths (absorbed, depth-exhausted, escaped
      // into a black background) skip the stack reads; depth 0 keeps res itself.
      // The "+ 0.0f" of each level only turns a -0 into +0 (an underflowed product stays +-0 in every
      // later level) and sum = +0 + ... is never -0, so it is dropped (the pixel is bit-identical); the
      // same argument covers the dielectric levels, which are not pushed (att (1,1,1)).
      const bool rsp_deep = POOL && rsp > A.rc_lds_levels;   // the path pushed past its LDS levels
      if (A.black_skip && rsp > 0 && res.x == 0.0f && res.y == 0.0f && res.z == 0.0f) {
        res = mk(0.0f, 0.0f, 0.0f);
        rsp = 0;
      }
      // Levels past the LDS ones live in HBM/L2: their codes are loaded kUnwindBatch at a time, then
      // decoded together, ahead of the multiply chain (one memory latency per batch, not per level)
      int32_t k = static_cast<int32_t>(rsp) - 1;
      const int32_t kl = static_cast<int32_t>(A.rc_lds_levels);
      while (!RC_LDS && k >= kl) {
        constexpr int kUnwindBatch = DEEP ? RT_UNWIND_BATCH : 1;
        uint32_t cw[kUnwindBatch];
#pragma unroll
        for (int i = 0; i < kUnwindBatch; ++i) cw[i] = rc_deep_load(static_cast<uint32_t>(max(k - i, kl)));
        f3 at[kUnwindBatch];
        rc_decode_batch<LDS, WIDE, NOISE, UV>(S, A, cw, at);
#pragma unroll
        for (int i = 0; i < kUnwindBatch; ++i)
          if (k - i >= kl) res = mk(at[i].x * res.x, at[i].y * res.y, at[i].z * res.z);
        k -= kUnwindBatch;
        if (k < kl) k = kl - 1;   // continue with the deepest LDS level
      }
      // LDS levels, kLdsBatch at a time: the code loads of a batch are issued together, then their
      // decodes (one LDS latency each per batch, not per level).  Levels below 0 read level 0 and
      // multiply by 1.0f instead (exact).
      constexpr int kLdsBatch = DEEP ? RT_UNWIND_LDS_DEEP : RT_UNWIND_LDS;
      for (; k >= 0; k -= kLdsBatch) {
        uint32_t cw[kLdsBatch];
#pragma unroll
        for (int i = 0; i < kLdsBatch; ++i) cw[i] = rc_lds_load(static_cast<uint32_t>(max(k - i, 0)));
        f3 at[kLdsBatch];
        rc_decode_batch<LDS, WIDE, NOISE, UV>(S, A, cw, at);
#pragma unroll
        for (int i = 0; i < kLdsBatch; ++i) {
          if (k - i < 0) at[i] = mk(1.0f, 1.0f, 1.0f);
          res = mk(at[i].x * res.x, at[i].y * res.y, at[i].z * res.z);
        }
      }
      if constexpr (POOL) {   // a deep path's pool chunk (read above, or skipped with a black path) is free again
        if (rsp_deep) {
          const uint32_t c = *pool_lane;
          if (c != 0xffu) {
            atomicOr(pool, 1u << c);
            *pool_lane = 0xffu;
          }
        }
      }
      if (TRACE) {   // the unwind's share of the done block (the rest: camera ray / pixel write)
        const uint64_t t = __builtin_amdgcn_s_memtime();
        ph_unwind += t - t_mark; if (lone) lph[5] += t - t_mark;
        t_mark = t;
      }
#ifdef RT_DBG_PX
      if (pxy == static_cast<uint32_t>(RT_DBG_PX))
        printf("dbgu s %d res %08x %08x %08x sum %08x %08x %08x\n", sample, __float_as_uint(res.x), __float_as_uint(res.y),
               __float_as_uint(res.z), __float_as_uint(sum_get().x), __float_as_uint(sum_get().y), __float_as_uint(sum_get().z));
#endif
      const f3 sum_now = add(sum_get(), res);
      sum_put(sum_now);
      sample++;
      if (COUNT) c_samples++;
      if (probe) {
        probe_end = true;   // its rounds are added to the tile's cost at the top of the next round
        busy = false;
      } else if (sample == A.spp) {
        const f3 c = mk(sum_now.x * A.sample_scale, sum_now.y * A.sample_scale, sum_now.z * A.sample_scale);
        uint32_t *sq = nullptr;   // the staging slot of the pixel's tile, if the wave still holds it
        const uint32_t plr = pxy >> 16, pj = pxy & 0xffffu;
        if (n_stage != 0u) {
          const uint32_t ptile = (plr >> tsh) * A.tiles_x + (pj >> ts);
          for (uint32_t q = 0; q < n_stage; ++q)
            if (stage[q * kStageSlotWords + kStageTile] == ptile) sq = stage + q * kStageSlotWords;
        }
        if (sq != nullptr) {   // parked in the tile's staging slot, stored with the whole tile
          const uint32_t k = ((plr & ((1u << tsh) - 1u)) << ts) | (pj & twm);
          float *const d = reinterpret_cast<float *>(sq) + 3u * k;
          d[0] = c.x;
          d[1] = c.y;
          d[2] = c.z;
          const uint64_t all = (static_cast<uint64_t>(sq[kStageValid + 1]) << 32) | sq[kStageValid];
          const uint64_t was = atomicOr(reinterpret_cast<unsigned long long *>(sq + kStageDone), 1ull << k);
          if (((was | (1ull << k)) & all) == all)   // the tile's last pixel: the wave stores it next round
            atomicOr(stage_done, 1u << static_cast<uint32_t>((sq - stage) / kStageSlotWords));
        } else if constexpr ((F & kVarTiledOut) != 0) {   // tile-major frame (untile_kernel writes rows and bytes)
          const uint32_t tile = (plr >> tsh) * A.tiles_x + (pj >> ts);
          const uint32_t k = ((plr & ((1u << tsh) - 1u)) << ts) | (pj & twm);
          float *o = A.out + static_cast<size_t>(tile) * 192u + 3u * k;
          if (RT_CHECK(A, tile * 64u + k < A.n_ids, CHK_PIXEL, tile * 64u + k, A.n_ids)) {
#ifdef RT_NT_FRAME   // A/B (RT_JIT_OPTS=-DRT_NT_FRAME): non-temporal stores of the tile frame
            __builtin_nontemporal_store(c.x, &o[0]);
            __builtin_nontemporal_store(c.y, &o[1]);
            __builtin_nontemporal_store(c.z, &o[2]);
#else
            o[0] = c.x;
            o[1] = c.y;
            o[2] = c.z;
#endif
          }
        } else if (RT_CHECK(A, plr < A.rows && pj < static_cast<uint32_t>(A.width), CHK_PIXEL, pxy, (A.rows << 16) | A.width)) {
          const size_t pix = static_cast<size_t>(plr) * static_cast<uint32_t>(A.width) + pj;
          float *o = A.out + 3 * pix;
          o[0] = c.x;
          o[1] = c.y;
          o[2] = c.z;
          if (A.out8) {   // pixels_to_ppm's bytes of the same floats (:1391-1395, 1419-1431), fused
            uint8_t *b = A.out8 + 3 * pix;
            b[0] = ppm_byte(c.x);
            b[1] = ppm_byte(c.y);
            b[2] = ppm_byte(c.z);
          }
        }
        busy = false;
      } else {
        camera_ray();
      }
      if (TRACE) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        ph_cam += t - t_mark; if (lone) lph[6] += t - t_mark;
        t_mark = t;
      }
    }
  }

  if (n_stage != 0u) stage_store();   // every pixel of the wave has ended: the tiles still parked
  if (A.span && lane == 0)   // vector atomics from one lane per wave: first start (above), last end of the launch
    atomicMax(A.span + 1, static_cast<unsigned long long>(__builtin_amdgcn_s_memrealtime()));
  if (TRACE && A.wave_trace && lane == 0) {
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_REG_HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));   // HW_REG_XCC_ID
    unsigned long long *w = A.wave_trace + kWaveTraceWords * static_cast<size_t>(blockIdx.x * kWavesPerBlock + wave);
    w[0] = t_start; w[1] = t_end; w[2] = tiles_taken; w[3] = (static_cast<uint64_t>(xcc) << 32) | hw;
    w[4] = rounds; w[5] = busy_lane_rounds;
    w[6] = ph_refill; w[7] = ph_trace; w[8] = ph_shade; w[9] = ph_mat; w[10] = ph_rej; w[11] = ph_unwind;
    w[12] = ph_cam;
    w[13] = lone_rounds;
    for (int k = 0; k < 7; ++k) w[14 + k] = lph[k];
    w[21] = ph_noise; w[22] = lph_noise;
  }
  if (COUNT) {
    uint32_t vals[CNT_SLOTS] = {0};
    for (int k = 0; k < 7; ++k) vals[k] = vc.k[k];
    vals[CNT_EXEC_NODE] = vc.xn;
    vals[CNT_EXEC_PRIM] = vc.xp;
    vals[CNT_BOUNCES] = c_bounce;
    vals[CNT_SHADES] = c_shade;
    vals[CNT_PERLIN] = c_perlin;
    vals[CNT_SAMPLES] = c_samples;
    for (int k = 0; k < CNT_SLOTS; ++k) {
      if (k == CNT_MAX_STACK || k == CNT_OVERFLOW || k == CNT_RNG) continue;
      unsigned long long v = vals[k];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0 && v) atomicAdd(&A.counters[k], v);
    }
    uint32_t ms = vc.max_sp;
    for (int off = 32; off > 0; off >>= 1) ms = max(ms, static_cast<uint32_t>(__shfl_xor(ms, off)));
    if (lane == 0) {
      atomicMax(&A.counters[CNT_MAX_STACK], static_cast<unsigned long long>(ms));
      // (kParkSum traces: the top kSumEntries entries hold the pixel sum, so the walk's own capacity is below them)
      if (ms > A.stack_cap - (kParkS ? kSumEntries : 0u)) atomicAdd(&A.counters[CNT_OVERFLOW], 1ull);
    }
  }
}

}  // namespace rt
