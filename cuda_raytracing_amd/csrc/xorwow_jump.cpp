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
  g_tables.resize(static_cast<size_t>(kJumpNibbleOffset) + static_cast<size_t>(kJumpNibPowers) * kJumpNibbleWords);
  for (int k = 0; k < kJumpPowers; ++k) {
    std::memcpy(g_tables.data() + static_cast<size_t>(k) * kJumpMatrixWords, a.r, sizeof a.r);
    square(a, t);
    a = t;
  }
  for (int k = 0; k < kJumpNibPowers; ++k) {
    const uint32_t *pk = g_tables.data() + static_cast<size_t>(k) * kJumpMatrixWords;   // P_k, rows [b][word]
    uint32_t *lo = g_tables.data() + kJumpNibbleOffset + static_cast<size_t>(k) * kJumpNibbleWords;
    uint32_t *hi = lo + kJumpNibbles * 16 * 4;
    for (int c = 0; c < kJumpNibbles; ++c)
      for (int v = 0; v < 16; ++v) {
        uint32_t r[5] = {0, 0, 0, 0, 0};
        for (int i = 0; i < 4; ++i)
          if ((v >> i) & 1)
            for (int w = 0; w < 5; ++w) r[w] ^= pk[(4 * c + i) * 5 + w];
        for (int w = 0; w < 4; ++w) lo[(c * 16 + v) * 4 + w] = r[w];
        hi[c * 16 + v] = r[4];
      }
  }
}

// M = the 160x160 matrix of x -> J^n x (rows[b] = image of e_b), by the binary powers P_k
void power_matrix(const std::vector<uint32_t> &T, uint64_t n, Mat &m) {
  for (int b = 0; b < 160; ++b) {
    uint32_t v[5] = {0, 0, 0, 0, 0};
    v[b >> 5] = 1u << (b & 31);
    for (int k = 0; n >> k && k < kJumpPowers; ++k)
      if ((n >> k) & 1u) apply(*reinterpret_cast<const Mat *>(T.data() + static_cast<size_t>(k) * kJumpMatrixWords), v);
    std::memcpy(m.r[b], v, sizeof v);
  }
}

}  // namespace

void xorwow_jump_nib(const uint32_t *tables, int k, uint32_t x[5]) {
  xorwow_apply_nib(tables + kJumpNibbleOffset + static_cast<size_t>(k) * kJumpNibbleWords, x);
}

void xorwow_apply_nib(const uint32_t *tab, uint32_t x[5]) {
  const uint32_t *lo = tab;
  const uint32_t *hi = lo + kJumpNibbles * 16 * 4;
  uint32_t r[5] = {0, 0, 0, 0, 0};
  for (int c = 0; c < kJumpNibbles; ++c) {
    const uint32_t e = c * 16 + ((x[c >> 3] >> (4 * (c & 7))) & 15u);
    for (int w = 0; w < 4; ++w) r[w] ^= lo[e * 4 + w];
    r[4] ^= hi[e];
  }
  std::memcpy(x, r, sizeof r);
}

void xorwow_row_bases(uint64_t seed, int width, int row_offset, int row_stride, int rows, std::vector<uint32_t> *out) {
  const std::vector<uint32_t> &T = xorwow_jump_tables();
  out->assign(static_cast<size_t>(rows > 0 ? rows : 0) * 8, 0u);
  if (rows <= 0) return;
  uint32_t st[6];
  xorwow_seed_host(seed, static_cast<uint64_t>(row_offset) * static_cast<uint64_t>(width), st);
  uint32_t x[5] = {st[1], st[2], st[3], st[4], st[5]};
  Mat m;
  power_matrix(T, static_cast<uint64_t>(row_stride) * static_cast<uint64_t>(width), m);
  for (int lr = 0; lr < rows; ++lr) {
    std::memcpy(&(*out)[static_cast<size_t>(lr) * 8], x, sizeof x);
    if (lr + 1 < rows) apply(m, x);
  }
}

void xorwow_phase_bases(uint64_t seed, int width, int row_offset, int row_stride, int rows, std::vector<uint32_t> *out,
                        int phase) {
  const int pw = 1 << phase;
  std::vector<uint32_t> rb;
  xorwow_row_bases(seed, width, row_offset, row_stride, rows, &rb);
  out->assign(static_cast<size_t>(rows > 0 ? rows : 0) * pw * 8, 0u);
  const std::vector<uint32_t> &T = xorwow_jump_tables();
  for (int lr = 0; lr < rows; ++lr) {
    uint32_t x[5];
    std::memcpy(x, &rb[static_cast<size_t>(lr) * 8], sizeof x);
    for (int c = 0; c < pw; ++c) {
      std::memcpy(&(*out)[(static_cast<size_t>(lr) * pw + c) * 8], x, sizeof x);
      if (c + 1 < width) xorwow_jump_nib(T.data(), 0, x);   // the next column: subsequence + 1 = P_0
    }
  }
}

void xorwow_column_tables(int width, std::vector<uint32_t> *out, int phase) {
  const int pw = 1 << phase;
  const int groups = width > 0 ? (width + pw - 1) / pw : 0;
  const int n_hi = (groups + kColLo - 1) / kColLo;
  out->assign(static_cast<size_t>(kColLo + n_hi) * kJumpNibbleWords, 0u);
  const std::vector<uint32_t> &T = xorwow_jump_tables();
  auto emit = [&](const Mat &m, int slot) {   // the nibble table of m at table slot `slot`
    uint32_t *lo = out->data() + static_cast<size_t>(slot) * kJumpNibbleWords;
    uint32_t *hi = lo + kJumpNibbles * 16 * 4;
    for (int c = 0; c < kJumpNibbles; ++c)
      for (int v = 0; v < 16; ++v) {
        uint32_t r[5] = {0, 0, 0, 0, 0};
        for (int i = 0; i < 4; ++i)
          if ((v >> i) & 1)
            for (int w = 0; w < 5; ++w) r[w] ^= m.r[4 * c + i][w];
        for (int w = 0; w < 4; ++w) lo[(c * 16 + v) * 4 + w] = r[w];
        hi[c * 16 + v] = r[4];
      }
  };
  // low tables J^(pw b), b < kColLo: M_0 = I, M_b = P_phase M_{b-1} (column by column through P_phase's table);
  // high tables J^(kColLo pw a): M_0 = I, M_a = P_{phase + 4} M_{a-1}
  for (int level = 0; level < 2; ++level) {
    Mat m;
    for (int b = 0; b < 160; ++b) {
      std::memset(m.r[b], 0, sizeof m.r[b]);
      m.r[b][b >> 5] = 1u << (b & 31);
    }
    const int count = level == 0 ? kColLo : n_hi, k = level == 0 ? phase : phase + kColLoBits;
    for (int t = 0; t < count; ++t) {
      if (t > 0)
        for (int b = 0; b < 160; ++b) xorwow_jump_nib(T.data(), k, m.r[b]);
      emit(m, level == 0 ? t : kColLo + t);
    }
  }
}

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
