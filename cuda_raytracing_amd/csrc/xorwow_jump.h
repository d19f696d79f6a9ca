// xorwow_jump.h — host-built jump tables for rocRAND-flavoured XORWOW subsequences.
#pragma once
#include <cstdint>
#include <vector>

namespace rt {

constexpr int kJumpPowers = 40;                 // subsequences < 2^40
constexpr int kJumpMatrixWords = 160 * 5;       // rows[b][k]: image of unit vector e_b

// P_k = A^(2^67 * 2^k), k in [0, kJumpPowers), concatenated (row-major [k][b][word]), followed by
// the nibble table of P_0 (the step to the next subsequence) at kJumpNibbleOffset: for input nibble c
// (bits 4c..4c+3 of the 160-bit state) and value v, the XOR of P_0's rows for v's bits — words 0..3
// as 640 uint4 [c * 16 + v], then word 4 as 640 u32.  P_0 x = XOR over c of table[c][nibble_c(x)].
constexpr int kJumpNibbles = 40, kJumpNibbleWords = kJumpNibbles * 16 * 5;
constexpr int kJumpNibbleOffset = kJumpPowers * kJumpMatrixWords;   // 16-B aligned (128 000 B)
// Then the nibble tables of P_1 .. P_{kJumpNibPowers-1} in the same format, table k at
// kJumpNibbleOffset + k * kJumpNibbleWords: the render kernel seeds a pixel from its row's base state by the
// binary jump over its column index (columns < 2^kJumpNibPowers).
constexpr int kJumpNibPowers = 31;
const std::vector<uint32_t> &xorwow_jump_tables();

// x <- P_k x through nibble table k (host)
void xorwow_jump_nib(const uint32_t *tables, int k, uint32_t x[5]);
// Row base states of a shard (the state of the row's first pixel, subsequence = global row index * width):
// out[lr * 8 + w] = word x_w (w < 5) of global row row_offset + lr * row_stride, lr < rows.  The Weyl word d is
// the same for every subsequence (xorwow_seed_base).
void xorwow_row_bases(uint64_t seed, int width, int row_offset, int row_stride, int rows, std::vector<uint32_t> *out);
// The render kernel's seeding tables (one nibble-table jump per pixel at tile pickup), for a phase width
// pw = 1 << phase (the tile width: every lane of a tile then applies the same table):
//  * phase bases: out[(lr * pw + c) * 8 + w] = word x_w of the state of pixel (row lr, column c), c < pw — the row
//    base jumped over its first pw columns (columns past the width keep the row base: never read);
//  * column tables, two levels (so that every XCD's L2 holds the few it reads — 46 tables at 3840 px, not 480): for
//    column group t = j >> phase = kColLo a + b, the nibble tables (kJumpNibbleWords, xorwow_jump_nib's format) of
//    J^(pw b) at slot b < kColLo and of J^(kColLo pw a) at slot kColLo + a.  Pixel (lr, j) = table[kColLo + a] and
//    table[b] applied to phase base (lr, j & (pw - 1)): powers of J commute.
void xorwow_phase_bases(uint64_t seed, int width, int row_offset, int row_stride, int rows, std::vector<uint32_t> *out,
                        int phase = 3);
constexpr int kColLoBits = 4, kColLo = 1 << kColLoBits;
void xorwow_column_tables(int width, std::vector<uint32_t> *out, int phase = 3);
// x <- (the matrix of nibble table tab) x
void xorwow_apply_nib(const uint32_t *tab, uint32_t x[5]);

// Seeded state {d, x0..x4} for (seed, subsequence) — same as rocrand_init(seed, subsequence, 0).
void xorwow_seed_host(uint64_t seed, uint64_t subsequence, uint32_t state[6]);

// rocRAND's constant seeding (rocrand_xorwow.h xorwow_engine ctor), no jump
inline void xorwow_seed_base(uint64_t seed, uint32_t state[6]) {
  uint32_t x[5] = {123456789u, 362436069u, 521288629u, 88675123u, 5783321u};
  uint32_t d = 6615241u;
  uint32_t s0 = static_cast<uint32_t>(seed) ^ 0x2c7f967fu;
  uint32_t s1 = static_cast<uint32_t>(seed >> 32) ^ 0xa03697cbu;
  uint32_t t0 = 1228688033u * s0, t1 = 2073658381u * s1;
  x[0] += t0; x[1] ^= t0; x[2] += t1; x[3] ^= t1; x[4] += t0;
  d += t1 + t0;
  state[0] = d;
  for (int k = 0; k < 5; ++k) state[1 + k] = x[k];
}

}  // namespace rt
