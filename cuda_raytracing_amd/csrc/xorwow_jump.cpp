// xorwow_jump.cpp — GF(2) jump matrices for per-pixel XORWOW subsequences.
//
// The reference seeds every pixel with curand_init(1234, pixel, 0) (raytracing.cu:1604): pixel i
// starts 2^67 * i draws into one XORWOW stream.  This build uses rocRAND's XORWOW (same recurrence,
// rocrand_xorwow.h), whose state after the jump is J^i * s0 with J = A^(2^67) and A the 160x160
// transition of the five xorshift words (the Weyl word d is unchanged by multiples of 2^32 steps).
// We precompute P_k = J^(2^k) once on the host; the seeding kernel applies the P_k selected by the
// bits of i (matrix-vector products with wave-uniform matrices: scalar loads, no divergence in data).
#include "xorwow_jump.h"

#include <cstring>
#include <mutex>

namespace rt {
namespace {

// column b of the matrix = image of unit vector e_b; stored as rows[b][0..4]
struct Mat { uint32_t r[160][5]; };

void step_linear(uint32_t x[5]) {
  uint32_t t = x[0] ^ (x[0] >> 2);
  x[0] = x[1]; x[1] = x[2]; x[2] = x[3]; x[3] = x[4];
  x[4] = (x[4] ^ (x[4] << 4)) ^ (t ^ (t << 1));
}

void apply(const Mat &m, uint32_t v[5]) {
  uint32_t out[5] = {0, 0, 0, 0, 0};
  for (int b = 0; b < 160; ++b)
    if ((v[b >> 5] >> (b & 31)) & 1u)
      for (int k = 0; k < 5; ++k) out[k] ^= m.r[b][k];
  std::memcpy(v, out, sizeof out);
}

void square(const Mat &m, Mat &out) {
  for (int b = 0; b < 160; ++b) {
    uint32_t v[5];
    std::memcpy(v, m.r[b], sizeof v);
    apply(m, v);
    std::memcpy(out.r[b], v, sizeof v);
  }
}

std::once_flag g_once;
std::vector<uint32_t> g_tables;

void build() {
  Mat a, t;
  for (int b = 0; b < 160; ++b) {
    uint32_t v[5] = {0, 0, 0, 0, 0};
    v[b >> 5] = 1u << (b & 31);
    step_linear(v);
    std::memcpy(a.r[b], v, sizeof v);
  }
  for (int i = 0; i < 67; ++i) { square(a, t); a = t; }
  g_tables.resize(static_cast<size_t>(kJumpNibbleOffset) + kJumpNibbleWords);
  for (int k = 0; k < kJumpPowers; ++k) {
    std::memcpy(g_tables.data() + static_cast<size_t>(k) * kJumpMatrixWords, a.r, sizeof a.r);
    square(a, t);
    a = t;
  }
  const uint32_t *p0 = g_tables.data();   // P_0, rows [b][word]
  uint32_t *lo = g_tables.data() + kJumpNibbleOffset, *hi = lo + kJumpNibbles * 16 * 4;
  for (int c = 0; c < kJumpNibbles; ++c)
    for (int v = 0; v < 16; ++v) {
      uint32_t r[5] = {0, 0, 0, 0, 0};
      for (int i = 0; i < 4; ++i)
        if ((v >> i) & 1)
          for (int w = 0; w < 5; ++w) r[w] ^= p0[(4 * c + i) * 5 + w];
      for (int w = 0; w < 4; ++w) lo[(c * 16 + v) * 4 + w] = r[w];
      hi[c * 16 + v] = r[4];
    }
}

}  // namespace

const std::vector<uint32_t> &xorwow_jump_tables() {
  std::call_once(g_once, build);
  return g_tables;
}

void xorwow_seed_host(uint64_t seed, uint64_t subsequence, uint32_t state[6]) {
  const std::vector<uint32_t> &T = xorwow_jump_tables();
  uint32_t x[5] = {123456789u, 362436069u, 521288629u, 88675123u, 5783321u};
  uint32_t d = 6615241u;
  uint32_t s0 = static_cast<uint32_t>(seed) ^ 0x2c7f967fu;
  uint32_t s1 = static_cast<uint32_t>(seed >> 32) ^ 0xa03697cbu;
  uint32_t t0 = 1228688033u * s0, t1 = 2073658381u * s1;
  x[0] += t0; x[1] ^= t0; x[2] += t1; x[3] ^= t1; x[4] += t0;
  d += t1 + t0;
  for (int k = 0; subsequence && k < kJumpPowers; ++k, subsequence >>= 1)
    if (subsequence & 1u) apply(*reinterpret_cast<const Mat *>(T.data() + static_cast<size_t>(k) * kJumpMatrixWords), x);
  state[0] = d;
  for (int k = 0; k < 5; ++k) state[1 + k] = x[k];
}

}  // namespace rt
