/*
 * oracle_rt.c — CPU restatement of luk-zm/cuda_raytracing's per-pixel render path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / CPU baseline — never as the product path.
 *
 * Parity status: "parity unpinned" against the reference binary.  The reference's path is CUDA
 * (src/raytracing.cu, nvcc + cuRAND) and cannot be built in this image without writing stand-ins
 * for CUDA/cuRAND headers, which this project does not do.  The reference has
 * no tests, fixtures or golden images.  What IS pinned:
 *   - the device RNG against rocRAND's own XORWOW (tests/golden/rng_kat.json, oracle/kat/);
 *   - the host RNG (glibc rand) against this image's libc;
 *   - analytic single-ray fixtures (tests/test_oracle.py).
 * Every function below cites the reference lines it restates, statement by statement: float
 * operations in source order, ternary MIN/MAX, g++ right-to-left argument evaluation for draws.
 * Build: gcc -O2 -ffp-contract=off (no FMA contraction, IEEE div/sqrt), see oracle/Makefile.
 *
 * Documented substitutions (identical in the HIP kernel):
 *   - cuRAND XORWOW -> rocRAND XORWOW (seed salting + uniform mapping differ);
 *   - sinf in the noise texture (raytracing.cu:389) -> rt_sinf below: the float rounding of a
 *     double-precision sine with a fixed reduction + polynomial (correctly rounded on every tested
 *     input; glibc's sinf agrees on ~98.7 %, CUDA's device sinf is within 2 ulp; tests/test_oracle.py);
 *   - powf(x, 5.0f) in Schlick's reflectance (raytracing.cu:436) -> (float)(x^5 in double);
 *   - acosf / atan2f in sphere_get_uv (raytracing.cu:583-590, image textures only) -> rt_acosf /
 *     rt_atan2f below (double evaluation from + - * and float seeds, identical in the kernel).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rt_render.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------- */
/* XORWOW (rocRAND flavour): state, seeding, 2^67 subsequence jumps                             */
/* ------------------------------------------------------------------------------------------- */
typedef struct { uint32_t d; uint32_t x[5]; } xw_state;

/* column-major GF(2) matrix: col[b] = M * e_b, b in [0,160) */
typedef struct { uint32_t col[160][5]; } xw_mat;

#define XW_POWERS 40
static xw_mat g_jump[XW_POWERS];   /* g_jump[k] = A^(2^67 * 2^k) */
static int g_jump_ready = 0;

static void xw_linear_step(uint32_t x[5]) {
  uint32_t t = x[0] ^ (x[0] >> 2);
  x[0] = x[1]; x[1] = x[2]; x[2] = x[3]; x[3] = x[4];
  x[4] = (x[4] ^ (x[4] << 4)) ^ (t ^ (t << 1));
}

static void xw_matvec(const xw_mat *m, uint32_t v[5]) {
  uint32_t r[5] = {0, 0, 0, 0, 0};
  for (int b = 0; b < 160; ++b) {
    if ((v[b >> 5] >> (b & 31)) & 1u) {
      for (int k = 0; k < 5; ++k) r[k] ^= m->col[b][k];
    }
  }
  memcpy(v, r, sizeof r);
}

static void xw_square(const xw_mat *m, xw_mat *out) {
  for (int b = 0; b < 160; ++b) {
    uint32_t v[5];
    memcpy(v, m->col[b], sizeof v);
    xw_matvec(m, v);
    memcpy(out->col[b], v, sizeof v);
  }
}

static void xw_build_tables(void) {
  static xw_mat a, tmp;
  for (int b = 0; b < 160; ++b) {
    uint32_t v[5] = {0, 0, 0, 0, 0};
    v[b >> 5] = 1u << (b & 31);
    xw_linear_step(v);
    memcpy(a.col[b], v, sizeof v);
  }
  for (int i = 0; i < 67; ++i) { xw_square(&a, &tmp); a = tmp; }   /* A^(2^67) */
  g_jump[0] = a;
  for (int k = 1; k < XW_POWERS; ++k) xw_square(&g_jump[k - 1], &g_jump[k]);
  g_jump_ready = 1;
}

/* rocrand_xorwow.h xorwow_engine(seed, subsequence, 0): constant salts, then subsequence jump.
 * Replaces curand_init(1234, idx, 0, &rng) (raytracing.cu:1604). */
static void xw_init(uint64_t seed, uint64_t subsequence, xw_state *s) {
  s->x[0] = 123456789u; s->x[1] = 362436069u; s->x[2] = 521288629u; s->x[3] = 88675123u;
  s->x[4] = 5783321u; s->d = 6615241u;
  uint32_t s0 = (uint32_t)seed ^ 0x2c7f967fu;
  uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xa03697cbu;
  uint32_t t0 = 1228688033u * s0;
  uint32_t t1 = 2073658381u * s1;
  s->x[0] += t0; s->x[1] ^= t0; s->x[2] += t1; s->x[3] ^= t1; s->x[4] += t0;
  s->d += t1 + t0;
  for (int k = 0; subsequence && k < XW_POWERS; ++k, subsequence >>= 1)
    if (subsequence & 1u) xw_matvec(&g_jump[k], s->x);
  /* the Weyl word d is unchanged: 2^67 steps are a multiple of 2^32 */
}

static uint32_t xw_next(xw_state *s) {
  uint32_t t = s->x[0] ^ (s->x[0] >> 2);
  s->x[0] = s->x[1]; s->x[1] = s->x[2]; s->x[2] = s->x[3]; s->x[3] = s->x[4];
  s->x[4] = (s->x[4] ^ (s->x[4] << 4)) ^ (t ^ (t << 1));
  s->d += 362437u;
  return s->d + s->x[4];
}

/* per-thread draw counter (RT_CNT_RNG_DRAWS) */
typedef struct {
  uint64_t c[RT_CNT__COUNT];
} counters;

/* rocrand_uniform: (0, 1] — stands in for curand_uniform */
static float uniform(xw_state *s, counters *cn) {
  cn->c[RT_CNT_RNG_DRAWS]++;
  const float inv = 2.3283064e-10f;
  uint32_t v = xw_next(s);
  return inv + ((float)v * inv);
}

/* ------------------------------------------------------------------------------------------- */
/* vec3 + scalar helpers (vec3.h, utility.h)                                                     */
/* ------------------------------------------------------------------------------------------- */
typedef rtr_vec3 vec3;
static inline vec3 v3(float x, float y, float z) { vec3 r = {x, y, z}; return r; }
static inline vec3 add(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }        /* :23-29 */
static inline vec3 sub(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }        /* :32-38 */
static inline vec3 scale(float s, vec3 v) { return v3(v.x * s, v.y * s, v.z * s); }           /* :41-47 */
static inline vec3 flip(vec3 v) { return v3(-v.x, -v.y, -v.z); }                              /* :50-53 */
static inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }         /* :87-89 */
static inline vec3 cross(vec3 a, vec3 b) {                                                      /* :92-98 */
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float length(vec3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }      /* :101-103 */
static inline vec3 unit(vec3 v) {                                                               /* :106-114 */
  float l = length(v);
  if (l == 0.0f) return v3(0.0f, 0.0f, 0.0f);
  return v3(v.x / l, v.y / l, v.z / l);
}
static inline vec3 comp_scale(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* :171-174 */
static inline int near_zero(vec3 v) {                                                           /* :177-180 */
  float s = 1e-8;
  return fabsf(v.x) < s && fabsf(v.y) < s && fabsf(v.z) < s;
}
static inline vec3 line_at(vec3 o, float t, vec3 d) { return add(o, scale(t, d)); }           /* :183-185 */
#define TMIN(a, b) (((a) < (b)) ? (a) : (b))   /* utility.h:6 */
#define TMAX(a, b) (((a) < (b)) ? (b) : (a))   /* utility.h:7 */

/* sinf substitute: float rounding of a double sine (Cody-Waite reduction by pi/2, Taylor kernels) */
static float rt_sinf(float xf) {
  double x = (double)xf;
  if (!(fabs(x) < 1.0e6)) return (float)sin(x);
  const double two_over_pi = 6.36619772367581382433e-01;
  const double p1 = 1.57079632673412561417e+00;   /* first 33 bits of pi/2 */
  const double p2 = 6.07710050630396597660e-11;   /* next 33 bits */
  const double p3 = 2.02226624871116645580e-21;   /* next bits */
  double k = floor(x * two_over_pi + 0.5);
  double r = ((x - k * p1) - k * p2) - k * p3;
  long q = (long)k & 3;
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
  return (float)res;
}

/* acosf / atan2f substitutes (sphere_get_uv, :583-590; only image textures read u,v): the float
 * rounding of a double evaluation built from + - * and float seeds only, so the oracle and the HIP
 * kernel (device/rt_body.h, the same operations) produce identical bits.  atan on [0,1]: anchor
 * c = k/8, r = (t - c)/(1 + t c) (|r| <= 1/16), odd Taylor series to r^15 (error < 3e-22). */
static const double RT_ATAN_K8[9] = {0.0, 0.12435499454676144, 0.24497866312686414, 0.35877067027057225,
                                     0.4636476090008061, 0.5585993153435624, 0.6435011087932844,
                                     0.7188299996216245, 0.7853981633974483};
static double rt_recip_d(double x) {            /* 1/x, x in [2^-60, 2^60]: float seed + 2 Newton steps */
  double y = (double)(1.0f / (float)x);
  y = y * (2.0 - x * y);
  y = y * (2.0 - x * y);
  return y;
}
static double rt_atan01_d(double t) {           /* t in [0, 1] */
  int k = (int)(t * 8.0 + 0.5);
  double c = (double)k * 0.125;
  double r = (t - c) * rt_recip_d(1.0 + t * c);
  double r2 = r * r;
  double p = r * (1.0 + r2 * (-1.0 / 3.0 + r2 * (1.0 / 5.0 + r2 * (-1.0 / 7.0 + r2 * (1.0 / 9.0 +
             r2 * (-1.0 / 11.0 + r2 * (1.0 / 13.0 + r2 * (-1.0 / 15.0))))))));
  return RT_ATAN_K8[k] + p;
}
static double rt_atan2_d(double y, double x) {  /* finite, not both zero */
  const double pi = 3.141592653589793, half_pi = 1.5707963267948966;
  double ax = fabs(x), ay = fabs(y);
  double m = ax > ay ? ax : ay;
  if (m < 8.673617379884035e-19) { ax *= 1.2676506002282294e30; ay *= 1.2676506002282294e30; }   /* 2^-60, 2^100 */
  else if (m > 1.152921504606847e18) { ax *= 7.888609052210118e-31; ay *= 7.888609052210118e-31; } /* 2^60, 2^-100 */
  double a;
  if (ay <= ax) a = rt_atan01_d(ay * rt_recip_d(ax));
  else a = half_pi - rt_atan01_d(ax * rt_recip_d(ay));
  if (x < 0.0 || (x == 0.0 && signbit(x))) a = pi - a;
  return signbit(y) ? -a : a;
}
static float rt_atan2f(float yf, float xf) {
  const double pi = 3.141592653589793;
  if (isnan(xf) || isnan(yf)) return xf + yf;
  double x = (double)xf, y = (double)yf, r;
  if (x == 0.0 && y == 0.0) r = signbit(x) ? pi : 0.0;
  else if (isinf(xf) && isinf(yf)) r = x > 0.0 ? 0.7853981633974483 : 2.356194490192345;
  else if (isinf(xf)) r = x > 0.0 ? 0.0 : pi;
  else if (isinf(yf)) r = 1.5707963267948966;
  else return (float)rt_atan2_d(y, x);
  return (float)(signbit(y) ? -r : r);
}
static float rt_acosf(float xf) {
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

/* powf(x, 5.0f) substitute */
static float rt_pow5f(float xf) {
  double x = (double)xf;
  double x2 = x * x;
  double x4 = x2 * x2;
  return (float)(x4 * x);
}

/* ------------------------------------------------------------------------------------------- */
/* scene access                                                                                  */
/* ------------------------------------------------------------------------------------------- */
typedef struct {
  const rt_scene *sc;
  int32_t max_bounces;
  int needs_stack_check;
} scene_ctx;

static int read_texture(const rt_scene *sc, uint64_t off, rtr_texture *t) {
  if (off + sizeof(rtr_texture) > sc->texture_bytes) return 0;
  memcpy(t, sc->textures + off, sizeof *t);
  return 1;
}

/* perlin_noise.cpp:22-46 + 1-20 (perm_x is used for all three axes, :37-39) */
static float perlin_noise_val(const rt_scene *sc, uint64_t table, vec3 p) {
  const uint8_t *base = sc->textures + table;
  float u = p.x - floorf(p.x);
  float v = p.y - floorf(p.y);
  float w = p.z - floorf(p.z);
  int32_t i = (int32_t)floorf(p.x);
  int32_t j = (int32_t)floorf(p.y);
  int32_t k = (int32_t)floorf(p.z);
  vec3 c[2][2][2];
  for (int32_t di = 0; di < 2; ++di)
    for (int32_t dj = 0; dj < 2; ++dj)
      for (int32_t dk = 0; dk < 2; ++dk) {
        int32_t pi, pj, pk;
        memcpy(&pi, base + offsetof(rtr_perlin, perm_x) + 4 * ((i + di) & 255), 4);
        memcpy(&pj, base + offsetof(rtr_perlin, perm_x) + 4 * ((j + dj) & 255), 4);
        memcpy(&pk, base + offsetof(rtr_perlin, perm_x) + 4 * ((k + dk) & 255), 4);
        int32_t g = (pi ^ pj ^ pk) & 255;
        memcpy(&c[di][dj][dk], base + offsetof(rtr_perlin, gradients) + 12 * g, 12);
      }
  float uu = u * u * (3 - 2 * u);
  float vv = v * v * (3 - 2 * v);
  float ww = w * w * (3 - 2 * w);
  float accum = 0.0f;
  for (int32_t a = 0; a < 2; a++)
    for (int32_t b = 0; b < 2; b++)
      for (int32_t d = 0; d < 2; d++) {
        vec3 wv = v3(u - (float)a, v - (float)b, w - (float)d);
        accum += (a * uu + (1 - a) * (1 - uu)) * (b * vv + (1 - b) * (1 - vv)) *
                 (d * ww + (1 - d) * (1 - ww)) * dot(c[a][b][d], wv);
      }
  return accum;
}

/* perlin_noise.cpp:72-85 */
static float perlin_turbulence(const rt_scene *sc, uint64_t table, vec3 p, int32_t depth) {
  float accum = 0.0f;
  vec3 tp = p;
  float weight = 1.0f;
  for (int32_t i = 0; i < depth; ++i) {
    accum += weight * perlin_noise_val(sc, table, tp);
    weight *= 0.5f;
    tp = v3(tp.x * 2, tp.y * 2, tp.z * 2);
  }
  return fabsf(accum);
}

/* raytracing.cu:343-354 */
static vec3 image_pixel(const rt_scene *sc, const rtr_texture *t, int32_t x, int32_t y) {
  if (t->u.image.host_pixels == 0) return v3(1, 0, 1);
  int32_t w = t->u.image.width, h = t->u.image.height;
  x = ((x) < (0) ? (0) : ((x) > (w) ? (w) : (x)));
  y = ((y) < (0) ? (0) : ((y) > (h) ? (h) : (y)));
  uint64_t off = t->u.image.pixels_offset + 12ull * ((uint64_t)y * (uint64_t)w + (uint64_t)x);
  vec3 r = v3(0, 0, 0);
  if (off + 12 <= sc->texture_bytes) memcpy(&r, sc->textures + off, 12);
  return r;
}

/* raytracing.cu:356-398 */
static vec3 texture_color(const rt_scene *sc, uint64_t off, float u, float v, vec3 p, counters *cn) {
  for (int guard = 0; guard < 64; ++guard) {
    rtr_texture t;
    if (!read_texture(sc, off, &t)) return v3(0, 0, 0);
    switch (t.kind) {
      case RTR_TEX_SOLID: return t.u.solid;
      case RTR_TEX_CHECKER: {
        int32_t x = (int32_t)floorf(t.u.checker.inv_scale * p.x);
        int32_t y = (int32_t)floorf(t.u.checker.inv_scale * p.y);
        int32_t z = (int32_t)floorf(t.u.checker.inv_scale * p.z);
        int is_even = (x + y + z) % 2 == 0;
        off = is_even ? t.u.checker.even.offset : t.u.checker.odd.offset;
        continue;
      }
      case RTR_TEX_IMAGE: {
        float cu = ((u) < (0) ? (0) : ((u) > (1) ? (1) : (u)));
        float cv = 1.0f - ((v) < (0) ? (0) : ((v) > (1) ? (1) : (v)));
        return image_pixel(sc, &t, (int32_t)(cu * t.u.image.width), (int32_t)(cv * t.u.image.height));
      }
      case RTR_TEX_NOISE: {
        cn->c[RT_CNT_PERLIN]++;
        float turb = perlin_turbulence(sc, t.u.noise.table_offset, p, 7);
        float s = 1 + rt_sinf(t.u.noise.scale * p.z + 10 * turb);
        return scale(s, v3(0.5f, 0.5f, 0.5f));
      }
      default: return v3(0, 0, 0);
    }
  }
  return v3(0, 0, 0);
}

/* ------------------------------------------------------------------------------------------- */
/* traversal (raytracing.cu:983-1251)                                                            */
/* ------------------------------------------------------------------------------------------- */
typedef struct { vec3 origin, direction; float time; } ray_t;                          /* :72-76 */
typedef struct {                                                                        /* :203-211 */
  vec3 point, normal;
  float t;
  int front;
  rtr_material mat;
  float u, v;
} hit_rec;

static void set_face_normal(hit_rec *r, const ray_t *ray, vec3 outward) {             /* :984-987 */
  r->front = dot(ray->direction, outward) < 0;
  r->normal = r->front ? outward : flip(outward);
}

static int aabb_hit(const rtr_aabb *b, const ray_t *ray, float t0, float t1) {         /* :990-1025 */
  float inv = 1.0f / ray->direction.x;
  float a = (b->x0 - ray->origin.x) * inv, c = (b->x1 - ray->origin.x) * inv;
  if (inv < 0.0f && a > c) { float s = a; a = c; c = s; }
  t0 = TMAX(t0, a); t1 = TMIN(t1, c);
  if (t1 <= t0) return 0;
  inv = 1.0f / ray->direction.y;
  a = (b->y0 - ray->origin.y) * inv; c = (b->y1 - ray->origin.y) * inv;
  if (inv < 0.0f && a > c) { float s = a; a = c; c = s; }
  t0 = TMAX(t0, a); t1 = TMIN(t1, c);
  if (t1 <= t0) return 0;
  inv = 1.0f / ray->direction.z;
  a = (b->z0 - ray->origin.z) * inv; c = (b->z1 - ray->origin.z) * inv;
  if (inv < 0.0f && a > c) { float s = a; a = c; c = s; }
  t0 = TMAX(t0, a); t1 = TMIN(t1, c);
  if (t1 <= t0) return 0;
  return 1;
}

/* :1060-1077; returns alpha/beta = +inf when the plane is missed */
static void plane_hit(const rtr_plane *g, const ray_t *ray, float tmin, float tmax,
                      float *alpha, float *beta, float *t, vec3 *p) {
  float denom = dot(g->normal, ray->direction);
  if (fabsf(denom) >= 1e-8) {
    *t = (g->d - dot(g->normal, ray->origin)) / denom;
    if (tmin <= *t && *t <= tmax) {
      *p = line_at(ray->origin, *t, ray->direction);
      vec3 q = sub(*p, g->q);
      *alpha = dot(g->w, cross(q, g->v));
      *beta = dot(g->w, cross(g->u, q));
      return;
    }
  }
  *alpha = *beta = INFINITY;
}

/* sphere_get_uv (:583-590): only image textures read u,v */
static void sphere_uv(vec3 p, float *u, float *v) {
  const float pi = 3.1415926535897932385f;
  float theta = rt_acosf(-p.y);
  float phi = rt_atan2f(-p.z, p.x) + pi;
  *u = phi / (2 * pi);
  *v = theta / pi;
}

#define STACK_CAP 4096

typedef struct {
  uint16_t data[STACK_CAP];
  int32_t count;
  int32_t max_seen;
  int overflow;
} href_stack;

static inline void push(href_stack *s, uint16_t r) {                                    /* :1037-1043 */
  if (s->count >= STACK_CAP) { s->overflow = 1; return; }
  s->data[s->count++] = r;
  if (s->count > s->max_seen) s->max_seen = s->count;
}

static int hit(const rt_scene *sc, href_stack *stack, uint16_t idx, float tmin, float tmax,
               ray_t *ray, hit_rec *rec, counters *cn) {                                 /* :1079-1251 */
  int result = 0, was_last_hit = 0;
  int32_t tcleanup = 0, ycleanup = 0;
  push(stack, idx);
  while (stack->count > 0) {
    uint16_t cur = stack->data[--stack->count];
    if (cur >= sc->hittable_count) { stack->overflow = 1; continue; }
    const rtr_hittable *h = &sc->hittables[cur];
    switch (h->kind) {
      case RTR_OBJ_SPHERE: {                                                             /* :1093-1123 */
        cn->c[RT_CNT_VISIT_SPHERE]++;
        const rtr_sphere *s = &h->u.sphere;
        vec3 center = line_at(s->center, ray->time, s->motion);
        vec3 oc = sub(center, ray->origin);
        float a = dot(ray->direction, ray->direction);
        float b = -2.0f * dot(ray->direction, oc);
        float c = dot(oc, oc) - s->radius * s->radius;
        float disc = b * b - 4 * a * c;
        if (disc >= 0) {
          float sq = sqrtf(disc);
          float root = (-b - sq) / (2.0f * a);
          if (tmin >= root || root >= tmax) root = (-b + sq) / (2.0f * a);
          if (tmin < root && root < tmax) {
            rec->t = root;
            rec->point = line_at(ray->origin, root, ray->direction);
            rec->mat = s->mat;
            vec3 outward = scale(1.0f / s->radius, sub(rec->point, center));
            sphere_uv(outward, &rec->u, &rec->v);
            set_face_normal(rec, ray, outward);
            tmax = rec->t;
            result = 1;
            if (tcleanup || ycleanup) was_last_hit = 1;
          }
        }
      } break;
      case RTR_OBJ_BVH: {                                                                /* :1124-1130 */
        cn->c[RT_CNT_VISIT_BVH]++;
        const rtr_bvh *n = &h->u.bvh;
        if (aabb_hit(&n->box, ray, tmin, tmax)) {
          if (n->right >= sc->ref_count || n->left >= sc->ref_count) { stack->overflow = 1; break; }
          push(stack, sc->refs[n->right]);
          push(stack, sc->refs[n->left]);
        }
      } break;
      case RTR_OBJ_TRIANGLE:                                                             /* :1131-1153 */
      case RTR_OBJ_QUAD: {                                                               /* :1154-1175 */
        int tri = h->kind == RTR_OBJ_TRIANGLE;
        cn->c[tri ? RT_CNT_VISIT_TRIANGLE : RT_CNT_VISIT_QUAD]++;
        const rtr_planar *q = &h->u.planar;
        float alpha = 0.0f, beta = 0.0f, t = 0.0f;
        vec3 p = v3(0, 0, 0);
        plane_hit(&q->geom, ray, tmin, tmax, &alpha, &beta, &t, &p);
        int inside = tri ? ((0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f) &&
                            (alpha + beta <= 1.0f))
                         : ((0.0f <= alpha && alpha <= 1.0f) && (0.0f <= beta && beta <= 1.0f));
        if (inside) {
          rec->u = alpha; rec->v = beta; rec->t = t; rec->point = p; rec->mat = q->mat;
          set_face_normal(rec, ray, q->geom.normal);
          tmax = rec->t;
          result = 1;
          if (tcleanup || ycleanup) was_last_hit = 1;
        }
      } break;
      case RTR_OBJ_TRANSLATE: {                                                          /* :1176-1191 */
        cn->c[RT_CNT_VISIT_TRANSLATE]++;
        const rtr_translate *tr = &h->u.translate;
        if (tcleanup == 0) {
          was_last_hit = 0;
          ray->origin = sub(ray->origin, tr->offset);
          push(stack, cur);
          push(stack, tr->child);
          tcleanup++;
        } else {
          ray->origin = add(ray->origin, tr->offset);
          tcleanup--;
          if (was_last_hit) rec->point = add(rec->point, tr->offset);
        }
      } break;
      case RTR_OBJ_YROTATE: {                                                            /* :1192-1237 */
        cn->c[RT_CNT_VISIT_YROTATE]++;
        const rtr_yrotate *y = &h->u.yrotate;
        float sn = y->sin_theta, cs = y->cos_theta;
        if (ycleanup == 0) {
          was_last_hit = 0;
          vec3 o = ray->origin, d = ray->direction;
          ray->origin = v3((cs * o.x) - (sn * o.z), o.y, (sn * o.x) + (cs * o.z));
          ray->direction = v3((cs * d.x) - (sn * d.z), d.y, (sn * d.x) + (cs * d.z));
          push(stack, cur);
          push(stack, y->child);
          ycleanup++;
        } else {
          vec3 o = ray->origin, d = ray->direction;
          ray->origin = v3((cs * o.x) + (sn * o.z), o.y, (-sn * o.x) + (cs * o.z));
          ray->direction = v3((cs * d.x) + (sn * d.z), d.y, (-sn * d.x) + (cs * d.z));
          ycleanup--;
          if (was_last_hit) {
            vec3 p = rec->point, n = rec->normal;
            rec->point = v3((cs * p.x) + (sn * p.z), p.y, (-sn * p.x) + (cs * p.z));
            rec->normal = v3((cs * n.x) + (sn * n.z), n.y, (-sn * n.x) + (cs * n.z));
          }
        }
      } break;
      case RTR_OBJ_GROUP: {                                                              /* :1238-1247 */
        cn->c[RT_CNT_VISIT_GROUP]++;
        const rtr_group *g = &h->u.group;
        for (uint16_t i = 0; i < g->count; ++i) push(stack, (uint16_t)(g->first + i));
      } break;
      default:
        break;
    }
  }
  return result;
}

/* ------------------------------------------------------------------------------------------- */
/* materials (raytracing.cu:415-502)                                                             */
/* ------------------------------------------------------------------------------------------- */
static vec3 reflect(vec3 d, vec3 n) { return sub(d, scale(2.0f * dot(d, n), n)); }      /* :425-429 */

static vec3 refract(vec3 uv, vec3 n, float e) {                                          /* :416-422 */
  float cos_theta = fminf(dot(flip(uv), n), 1.0f);
  vec3 perp = scale(e, add(uv, scale(cos_theta, n)));
  float perp_len = length(perp);
  vec3 par = scale(-sqrtf(fabsf(1.0f - perp_len * perp_len)), n);
  return add(perp, par);
}

static float reflectance(float cosine, float ri) {                                       /* :432-437 */
  float r0 = (1.0f - ri) / (1.0f + ri);
  r0 = r0 * r0;
  return r0 + (1.0f - r0) * rt_pow5f(1.0f - cosine);
}

static float bound(xw_state *rng, float lo, float hi, counters *cn) {                   /* utility.h:35-37 */
  return lo + (hi - lo) * uniform(rng, cn);
}

/* vec3.h:152-161 — Vec3(f(), f(), f()) drawn right-to-left (z, y, x) */
static vec3 random_unit_vector(xw_state *rng, counters *cn) {
  for (;;) {
    float z = bound(rng, -1.0f, 1.0f, cn);
    float y = bound(rng, -1.0f, 1.0f, cn);
    float x = bound(rng, -1.0f, 1.0f, cn);
    vec3 r = v3(x, y, z);
    float len = length(r);
    float len2 = len * len;
    if (1e-50 < len2 && len2 <= 1.0f) return scale(1.0f / len, r);
  }
}

typedef struct { int is_hit; vec3 direction, attenuation; } scatter_t;

/* cuda_material_scatter (:497-502): random_test is drawn before the unit vector (g++ order),
 * for every material including lights; material_scatter_common (:452-490). */
static scatter_t scatter(const rt_scene *sc, xw_state *rng, const hit_rec *rec, vec3 in_dir, counters *cn) {
  float random_test = uniform(rng, cn);
  vec3 ruv = random_unit_vector(rng, cn);
  scatter_t r;
  memset(&r, 0, sizeof r);
  switch (rec->mat.kind) {
    case RTR_MAT_LAMBERTIAN:
      r.is_hit = 1;
      r.direction = add(rec->normal, ruv);
      if (near_zero(r.direction)) r.direction = rec->normal;
      r.attenuation = texture_color(sc, rec->mat.u.lambert_tex.offset, rec->u, rec->v, rec->point, cn);
      break;
    case RTR_MAT_METAL: {
      vec3 refl = reflect(in_dir, rec->normal);
      r.direction = add(unit(refl), scale(rec->mat.u.metal.fuzz, ruv));
      r.attenuation = rec->mat.u.metal.albedo;
      r.is_hit = dot(r.direction, rec->normal) > 0;
    } break;
    case RTR_MAT_DIELECTRIC: {
      r.attenuation = v3(1.0f, 1.0f, 1.0f);
      float ior = rec->mat.u.dielectric.ior;
      float ri = rec->front ? (1.0f / ior) : ior;
      vec3 ud = unit(in_dir);
      float cos_theta = fminf(dot(flip(ud), rec->normal), 1.0f);
      float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
      int cannot = ri * sin_theta > 1.0f;
      if (cannot || reflectance(cos_theta, ri) > random_test) r.direction = reflect(ud, rec->normal);
      else r.direction = refract(ud, rec->normal, ri);
      r.is_hit = 1;
    } break;
    default:
      break;
  }
  return r;
}

static vec3 emitted(const rt_scene *sc, const hit_rec *rec, counters *cn) {             /* :439-450 */
  if (rec->mat.kind == RTR_MAT_DIFFUSE_LIGHT)
    return texture_color(sc, rec->mat.u.light_tex.offset, rec->u, rec->v, rec->point, cn);
  return v3(0, 0, 0);
}

/* ray_color (:1333-1371) with the colour stack of :1253-1276 */
static vec3 ray_color(const rt_scene *sc, href_stack *hs, xw_state *rng, ray_t *ray, vec3 background,
                      int32_t max_bounces, counters *cn) {
  vec3 att[256], emit[256];
  int32_t count = 0;
  int32_t bounces = max_bounces;
  vec3 result = v3(0, 0, 0);
  hit_rec rec;
  memset(&rec, 0, sizeof rec);
  uint16_t root = sc->refs[sc->root];
  while (bounces > 0) {
    if (hit(sc, hs, root, 0.001f, INFINITY, ray, &rec, cn)) {
      cn->c[RT_CNT_SHADES]++;
      vec3 e = emitted(sc, &rec, cn);
      scatter_t s = scatter(sc, rng, &rec, ray->direction, cn);
      if (s.is_hit) {
        ray->origin = rec.point;
        ray->direction = s.direction;
        att[count] = s.attenuation;
        emit[count] = e;
        count++;
        cn->c[RT_CNT_BOUNCES]++;
        bounces--;
      } else {
        result = e;
        break;
      }
    } else {
      result = background;
      break;
    }
  }
  while (count > 0) {
    count--;
    result = add(comp_scale(att[count], result), emit[count]);
  }
  return result;
}

/* ------------------------------------------------------------------------------------------- */
/* cuda_calc (:1543-1589), one pixel                                                             */
/* ------------------------------------------------------------------------------------------- */
static void render_pixel(const rt_scene *sc, const rt_camera *cam, const rt_params *p, int32_t i, int32_t j,
                         float *out, href_stack *hs, counters *cn) {
  xw_state rng;
  xw_init(p->seed, (uint64_t)i * (uint64_t)p->width + (uint64_t)j, &rng);
  int32_t max_bounces = (int32_t)(uint8_t)p->max_bounces;   /* rc_stack.max_count is u8 (:220,1596) */
  float sample_scale = 1.0f / (float)p->samples_per_pixel;  /* :1657 */
  vec3 pixel_point = add(cam->pixel00, add(scale((float)i, cam->delta_v), scale((float)j, cam->delta_u)));
  vec3 sum = v3(0, 0, 0);
  for (int32_t s = 0; s < p->samples_per_pixel; ++s) {
    ray_t ray;
    if (cam->defocus_angle <= 0) {
      ray.origin = cam->center;
    } else {                                                                         /* :1459-1476 */
      vec3 d;
      for (;;) {
        float y = bound(&rng, -1.0f, 1.0f, cn);   /* Vec3(x(), y(), 0): y drawn first */
        float x = bound(&rng, -1.0f, 1.0f, cn);
        d = v3(x, y, 0.0f);
        float l = length(d);
        if (l * l < 1.0f) break;
      }
      ray.origin = add(cam->center, add(scale(d.x, cam->defocus_u), scale(d.y, cam->defocus_v)));
    }
    float xo = uniform(&rng, cn) - 0.5f;
    float yo = uniform(&rng, cn) - 0.5f;
    ray.direction = sub(pixel_point, ray.origin);
    ray.direction = add(ray.direction, scale(xo, cam->delta_u));
    ray.direction = add(ray.direction, scale(yo, cam->delta_v));
    ray.time = uniform(&rng, cn);
    vec3 c = ray_color(sc, hs, &rng, &ray, p->background, max_bounces, cn);
    sum = add(sum, c);
    cn->c[RT_CNT_SAMPLES]++;
  }
  sum = scale(sample_scale, sum);
  out[0] = sum.x; out[1] = sum.y; out[2] = sum.z;
}

static int validate(const rt_scene *sc, const rt_camera *cam, const rt_params *p, const float *out) {
  if (!sc || !cam || !p || !out) return RT_ERR_INVALID_ARG;
  if (!sc->hittables || !sc->refs || sc->hittable_count == 0 || sc->ref_count == 0) return RT_ERR_SCENE;
  if (sc->root >= sc->ref_count || sc->refs[sc->root] >= sc->hittable_count) return RT_ERR_SCENE;
  if (p->width <= 0 || p->height <= 0 || p->samples_per_pixel <= 0) return RT_ERR_INVALID_ARG;
  if (p->row_stride <= 0 || p->row_count < 0 || p->row_offset < 0) return RT_ERR_INVALID_ARG;
  if (p->row_count > 0 && (int64_t)p->row_offset + (int64_t)(p->row_count - 1) * p->row_stride >= p->height)
    return RT_ERR_INVALID_ARG;
  return RT_OK;
}

int rt_render_cpu(const rt_scene *sc, const rt_camera *cam, const rt_params *p, float *out, rt_stats *st) {
  int v = validate(sc, cam, p, out);
  if (v != RT_OK) return v;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp critical(rt_oracle_tables)
  {
    if (!g_jump_ready) xw_build_tables();
  }
  counters total;
  memset(&total, 0, sizeof total);
  int overflow = 0;
  int32_t max_stack = 0;
  const int64_t rows = p->row_count;
#pragma omp parallel
  {
    counters cn;
    memset(&cn, 0, sizeof cn);
    href_stack *hs = (href_stack *)malloc(sizeof(href_stack));
    hs->count = 0; hs->max_seen = 0; hs->overflow = 0;
#pragma omp for schedule(dynamic, 1)
    for (int64_t r = 0; r < rows; ++r) {
      int32_t i = p->row_offset + (int32_t)r * p->row_stride;
      for (int32_t j = 0; j < p->width; ++j)
        render_pixel(sc, cam, p, i, j, out + 3 * ((size_t)r * (size_t)p->width + (size_t)j), hs, &cn);
    }
#pragma omp critical(rt_oracle_merge)
    {
      for (int k = 0; k < RT_CNT__COUNT; ++k) total.c[k] += cn.c[k];
      if (hs->overflow) overflow = 1;
      if (hs->max_seen > max_stack) max_stack = hs->max_seen;
    }
    free(hs);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (st) {
    memset(st, 0, sizeof *st);
    st->render_ms = (double)(t1.tv_sec - t0.tv_sec) * 1e3 + (double)(t1.tv_nsec - t0.tv_nsec) / 1e6;
    st->total_ms = st->render_ms;
    st->samples = (uint64_t)rows * (uint64_t)p->width * (uint64_t)p->samples_per_pixel;
    for (int k = 0; k < RT_CNT__COUNT; ++k) st->counters[k] = total.c[k];
    st->counters[RT_CNT_MAX_STACK] = (uint64_t)max_stack;
    st->counters[RT_CNT_STACK_OVERFLOW] = (uint64_t)overflow;
    st->stack_needed = max_stack;
  }
  return overflow ? RT_ERR_SCENE : RT_OK;
}

/* exported for tests: the substituted transcendental and one RNG stream */
float rt_oracle_sinf(float x) { return rt_sinf(x); }
float rt_oracle_atan2f(float y, float x) { return rt_atan2f(y, x); }
float rt_oracle_acosf(float x) { return rt_acosf(x); }
float rt_oracle_pow5f(float x) { return rt_pow5f(x); }
int rt_oracle_uniforms(uint64_t seed, uint64_t subsequence, float *out, int n) {
#pragma omp critical(rt_oracle_tables)
  {
    if (!g_jump_ready) xw_build_tables();
  }
  counters cn;
  xw_state s;
  xw_init(seed, subsequence, &s);
  for (int i = 0; i < n; ++i) out[i] = uniform(&s, &cn);
  return RT_OK;
}

/* OpenMP threads rt_render_cpu will use (bench.py reports it as cpu_baseline.cores) */
int rt_oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* bench.py's CPU baseline: the same render on n threads (1 = the single-core rate) */
int rt_oracle_set_threads(int n) {
  if (n < 1) return RT_ERR_INVALID_ARG;
#ifdef _OPENMP
  omp_set_num_threads(n);
#endif
  return RT_OK;
}
