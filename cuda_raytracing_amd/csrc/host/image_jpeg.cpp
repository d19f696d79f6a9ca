// image_jpeg.cpp — JPEG decoding for image textures, with the output of the reference's loader.
//
// make_image_texture (raytracing.cu:332-341) loads its file with stbi_loadf from the third-party
// stb_image v2.30 that the reference vendors (include/stb_image.h); the catalog's earth texture is a
// JPEG (:2043, :2180).  This decoder (ITU-T T.81: baseline and extended sequential Huffman, progressive
// with spectral selection and successive approximation, restart intervals, 1/3/4 components, any integer
// sampling factors up to 4) is derived from stb_image v2.30's JPEG decoder: the Huffman table build and
// fast-AC table (stb_image.h:2003-2073), the bit reader and block decoders (:2075-2413, incl. the
// progressive refinement loop), the zig-zag table (:2194), the resampler loop and the blinn_8x8 rounding
// (:3859) follow stb's code, so that the texels are the same bits (tests/test_image_load.py compares
// against stb_image itself, compiled from the reference tree into oracle/_ref).  Numerical choices kept:
//   - inverse DCT: the islow integer flow graph (jidctint), constants rounded to 12 fractional bits,
//     columns first with +2^9 >> 10, rows with +2^16 + 128*2^17 >> 17, clamped to 0..255, in the lane
//     widths of stb's SSE2 version (what the reference's x86-64 host runs);
//   - coefficients dequantised into 16-bit values (progressive: after the last scan);
//   - chroma upsampling: nearest for factor 1, the "fancy" triangle filters for 2x1, 1x2 and 2x2
//     ((3 near + far + 2) >> 2; 2x2: (3 (3n + f) + (3n' + f') + 8) >> 4), pixel replication otherwise;
//   - YCbCr -> RGB in 20-bit fixed point (Cb, Cr coefficients 1.402, 0.71414, 0.34414, 1.772 rounded
//     to 12 bits, the Cb term of green truncated to its upper 16 bits); Adobe RGB / CMYK / YCCK handled
//     as stb does; grey replicated to three channels;
//   - out-of-data and marker handling of the entropy decoder (zero bits after the data ends, a restart
//     marker expected every restart interval, junk after the last scan skipped).
// It returns false where stbi_loadf returns NULL (the reference's texture then has no pixels).
//
// Provenance and licence.  Parts of this file are DERIVED FROM stb_image v2.30 (Sean Barrett and contributors,
// http://nothings.org/stb), the third-party header the reference vendors as include/stb_image.h, and keep its
// structure where bit-exactness with stbi_loadf (corrupt and truncated files included) requires the same
// control flow.  stb_image is available under the MIT licence or as public domain (its ALTERNATIVE A / B);
// this derived code is used under ALTERNATIVE A, whose notice follows:
//   Copyright (c) 2017 Sean Barrett
//   Permission is hereby granted, free of charge, to any person obtaining a copy of this software and
//   associated documentation files (the "Software"), to deal in the Software without restriction, including
//   without limitation the rights to use, copy, modify, merge, publish, distribute, sublicense, and/or sell
//   copies of the Software, and to permit persons to whom the Software is furnished to do so, subject to the
//   following conditions: The above copyright notice and this permission notice shall be included in all
//   copies or substantial portions of the Software.  THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY
//   KIND, EXPRESS OR IMPLIED, INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY, FITNESS FOR A
//   PARTICULAR PURPOSE AND NONINFRINGEMENT. IN NO EVENT SHALL THE AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR
//   ANY CLAIM, DAMAGES OR OTHER LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR OTHERWISE, ARISING FROM,
//   OUT OF OR IN CONNECTION WITH THE SOFTWARE OR THE USE OR OTHER DEALINGS IN THE SOFTWARE.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "image_decoders.h"

namespace rt {
namespace jpeg {
namespace {

constexpr int kFastBits = 9;
constexpr uint8_t kNoMarker = 0xff;

// position in the 8x8 block (row-major) of the k-th coefficient of the zig-zag order; entries past 63
// keep corrupt runs inside the block
const uint8_t kZigzag[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// canonical Huffman table (T.81 Annex C) with a kFastBits-bit lookup for short codes
struct Huffman {
  uint8_t fast[1 << kFastBits];
  uint16_t code[256];
  uint8_t values[256];
  uint8_t size[257];
  uint32_t maxcode[18];
  int delta[17];
  int16_t fast_ac[1 << kFastBits];   // AC tables: (value << 8) | (run << 4) | (code + magnitude bits)

  bool build(const int counts[16]) {
    int k = 0;
    for (int len = 1; len <= 16; ++len)
      for (int j = 0; j < counts[len - 1]; ++j) {
        size[k++] = static_cast<uint8_t>(len);
        if (k >= 257) return false;
      }
    size[k] = 0;
    uint32_t c = 0;
    int s = 0;
    int len;
    for (len = 1; len <= 16; ++len) {
      delta[len] = s - static_cast<int>(c);
      if (size[s] == len) {
        while (size[s] == len) code[s++] = static_cast<uint16_t>(c++);
        if (c - 1 >= (1u << len)) return false;
      }
      maxcode[len] = c << (16 - len);
      c <<= 1;
    }
    maxcode[len] = 0xffffffffu;
    std::memset(fast, 255, sizeof fast);
    for (int i = 0; i < s; ++i)
      if (size[i] <= kFastBits) {
        const int base = code[i] << (kFastBits - size[i]), m = 1 << (kFastBits - size[i]);
        for (int j = 0; j < m; ++j) fast[base + j] = static_cast<uint8_t>(i);
      }
    return true;
  }

  // a code of at most kFastBits bits followed by all its magnitude bits, value in [-128, 127]: one lookup
  void build_fast_ac() {
    for (int i = 0; i < (1 << kFastBits); ++i) {
      fast_ac[i] = 0;
      if (fast[i] == 255) continue;
      const int rs = values[fast[i]], run = (rs >> 4) & 15, mag = rs & 15, len = size[fast[i]];
      if (mag == 0 || len + mag > kFastBits) continue;
      int v = ((i << len) & ((1 << kFastBits) - 1)) >> (kFastBits - mag);
      if (v < (1 << (mag - 1))) v += static_cast<int>(~0u << mag) + 1;   // EXTEND (F.2.2.1)
      if (v >= -128 && v <= 127) fast_ac[i] = static_cast<int16_t>(v * 256 + run * 16 + len + mag);
    }
  }
};

struct Component {
  int id = 0, h = 1, v = 1, tq = 0, hd = 0, ha = 0;
  int x = 0, y = 0;          // effective size in samples
  int w2 = 0, h2 = 0;        // sample buffer: whole MCUs
  int dc_pred = 0;
  std::vector<uint8_t> data;
  std::vector<int16_t> coeff;   // progressive: natural-order coefficients of every block
  int coeff_w = 0;
};

struct Decoder {
  const uint8_t *buf;
  size_t n, pos = 0;
  Huffman hdc[4]{}, hac[4]{};   // zeroed like stb's memset jpeg state: an undefined table reads symbol 0 from 0 bits
  uint16_t dequant[4][64];
  Component comp[4];
  int img_x = 0, img_y = 0, img_n = 0;
  int hmax = 1, vmax = 1, mcu_x = 0, mcu_y = 0;
  bool progressive = false, jfif = false;
  int adobe = -1, rgb_ids = 0;
  // scan state
  int scan_n = 0, order[4] = {0, 0, 0, 0};
  int spec_start = 0, spec_end = 0, succ_high = 0, succ_low = 0;
  int restart_interval = 0, todo = 0, eob_run = 0;
  uint32_t code_buffer = 0;
  int code_bits = 0;
  uint8_t marker = kNoMarker;
  bool nomore = false;

  Decoder(const uint8_t *b, size_t len) : buf(b), n(len) { std::memset(dequant, 0, sizeof dequant); }

  bool at_eof() const { return pos >= n; }
  uint32_t get8() { return pos < n ? buf[pos++] : 0u; }
  uint32_t get16() { const uint32_t a = get8(); return (a << 8) | get8(); }
  void skip(long k) { if (k <= 0) return; pos = (static_cast<size_t>(k) > n - pos) ? n : pos + static_cast<size_t>(k); }

  // ---- entropy-coded segment bit reader: 0xFF00 is a data byte, any other 0xFFxx ends the segment ----
  void fill() {
    do {
      uint32_t b = nomore ? 0u : get8();
      if (b == 0xff) {
        uint32_t c = get8();
        while (c == 0xff) c = get8();
        if (c != 0) { marker = static_cast<uint8_t>(c); nomore = true; return; }
      }
      code_buffer |= b << (24 - code_bits);
      code_bits += 8;
    } while (code_bits <= 24);
  }
  uint8_t next_marker() {
    if (marker != kNoMarker) { const uint8_t m = marker; marker = kNoMarker; return m; }
    uint32_t x = get8();
    if (x != 0xff) return kNoMarker;
    while (x == 0xff) x = get8();
    return static_cast<uint8_t>(x);
  }
  int decode(const Huffman &h) {
    if (code_bits < 16) fill();
    const int c = (code_buffer >> (32 - kFastBits)) & ((1 << kFastBits) - 1);
    const int f = h.fast[c];
    if (f < 255) {
      const int s = h.size[f];
      if (s > code_bits) return -1;
      code_buffer <<= s;
      code_bits -= s;
      return h.values[f];
    }
    const uint32_t top = code_buffer >> 16;
    int k;
    for (k = kFastBits + 1;; ++k) if (top < h.maxcode[k]) break;
    if (k == 17) { code_bits -= 16; return -1; }
    if (k > code_bits) return -1;
    const int sym = static_cast<int>((code_buffer >> (32 - k)) & ((1u << k) - 1)) + h.delta[k];
    if (sym < 0 || sym >= 256) return -1;
    code_bits -= k;
    code_buffer <<= k;
    return h.values[sym];
  }
  static uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> ((32 - k) & 31)); }
  int receive_extend(int k) {   // RECEIVE + EXTEND (F.2.2.1); 0 once the data has run out
    if (code_bits < k) fill();
    if (code_bits < k) return 0;
    const int neg = static_cast<int>(code_buffer >> 31) ^ 1;   // leading bit 0: a negative value
    uint32_t v = rotl(code_buffer, k);
    const uint32_t mask = (1u << k) - 1;
    code_buffer = v & ~mask;
    v &= mask;
    code_bits -= k;
    return static_cast<int>(v) - (neg ? static_cast<int>(mask) : 0);
  }
  int bits(int k) {
    if (code_bits < k) fill();
    if (code_bits < k) return 0;
    uint32_t v = rotl(code_buffer, k);
    const uint32_t mask = (1u << k) - 1;
    code_buffer = v & ~mask;
    code_bits -= k;
    return static_cast<int>(v & mask);
  }
  bool bit() {
    if (code_bits < 1) fill();
    if (code_bits < 1) return false;
    const bool b = (code_buffer & 0x80000000u) != 0;
    code_buffer <<= 1;
    --code_bits;
    return b;
  }
  void reset() {
    code_bits = 0; code_buffer = 0; nomore = false; marker = kNoMarker; eob_run = 0;
    for (Component &c : comp) c.dc_pred = 0;
    todo = restart_interval ? restart_interval : 0x7fffffff;
  }
  static bool add_ok(int a, int b) { return (b < 0) ? a >= INT32_MIN - b : a <= INT32_MAX - b; }
  static bool mul16_ok(int a, int b) {
    if (b == 0 || a == 0) return true;
    const long long p = static_cast<long long>(a) * b;
    return p >= -32768 && p <= 32767;
  }

  // ---- one block of a sequential scan (F.2.2), dequantised in natural order ----
  bool block(int16_t *d, int c) {
    Component &cp = comp[c];
    const Huffman &ha = hac[cp.ha];
    const uint16_t *q = dequant[cp.tq];
    if (code_bits < 16) fill();
    const int t = decode(hdc[cp.hd]);
    if (t < 0 || t > 15) return false;
    std::memset(d, 0, 64 * sizeof(int16_t));
    const int diff = t ? receive_extend(t) : 0;
    if (!add_ok(cp.dc_pred, diff)) return false;
    const int dc = cp.dc_pred + diff;
    cp.dc_pred = dc;
    if (!mul16_ok(dc, q[0])) return false;
    d[0] = static_cast<int16_t>(dc * q[0]);
    int k = 1;
    do {
      if (code_bits < 16) fill();
      const int fa = ha.fast_ac[(code_buffer >> (32 - kFastBits)) & ((1 << kFastBits) - 1)];
      if (fa) {
        k += (fa >> 4) & 15;
        const int s = fa & 15;
        if (s > code_bits) return false;
        code_buffer <<= s;
        code_bits -= s;
        const int z = kZigzag[k++];
        d[z] = static_cast<int16_t>((fa >> 8) * q[z]);
      } else {
        const int rs = decode(ha);
        if (rs < 0) return false;
        const int s = rs & 15, r = rs >> 4;
        if (s == 0) {
          if (rs != 0xf0) break;   // EOB
          k += 16;
        } else {
          k += r;
          const int z = kZigzag[k++];
          d[z] = static_cast<int16_t>(receive_extend(s) * q[z]);
        }
      }
    } while (k < 64);
    return true;
  }

  // ---- progressive scans (G.1.2) into the coefficient store ----
  bool block_dc(int16_t *d, int c) {
    if (spec_end != 0) return false;
    if (code_bits < 16) fill();
    if (succ_high == 0) {
      std::memset(d, 0, 64 * sizeof(int16_t));
      const int t = decode(hdc[comp[c].hd]);
      if (t < 0 || t > 15) return false;
      const int diff = t ? receive_extend(t) : 0;
      if (!add_ok(comp[c].dc_pred, diff)) return false;
      const int dc = comp[c].dc_pred + diff;
      comp[c].dc_pred = dc;
      if (!mul16_ok(dc, 1 << succ_low)) return false;
      d[0] = static_cast<int16_t>(dc * (1 << succ_low));
    } else if (bit()) {
      d[0] = static_cast<int16_t>(d[0] + (1 << succ_low));
    }
    return true;
  }
  bool block_ac(int16_t *d, int c) {
    if (spec_start == 0) return false;
    const Huffman &ha = hac[comp[c].ha];
    if (succ_high == 0) {   // first scan of the band
      if (eob_run) { --eob_run; return true; }
      int k = spec_start;
      do {
        if (code_bits < 16) fill();
        const int fa = ha.fast_ac[(code_buffer >> (32 - kFastBits)) & ((1 << kFastBits) - 1)];
        if (fa) {
          k += (fa >> 4) & 15;
          const int s = fa & 15;
          if (s > code_bits) return false;
          code_buffer <<= s;
          code_bits -= s;
          d[kZigzag[k++]] = static_cast<int16_t>((fa >> 8) * (1 << succ_low));
        } else {
          const int rs = decode(ha);
          if (rs < 0) return false;
          const int s = rs & 15, r = rs >> 4;
          if (s == 0) {
            if (r < 15) {   // EOBn
              eob_run = (1 << r);
              if (r) eob_run += bits(r);
              --eob_run;
              break;
            }
            k += 16;
          } else {
            k += r;
            d[kZigzag[k++]] = static_cast<int16_t>(receive_extend(s) * (1 << succ_low));
          }
        }
      } while (k <= spec_end);
      return true;
    }
    // refinement (G.1.2.3): one correction bit for every non-zero coefficient passed, new +-1 values
    const int16_t b = static_cast<int16_t>(1 << succ_low);
    auto refine = [&](int16_t *p) {
      if (bit() && (*p & b) == 0) *p = static_cast<int16_t>(*p > 0 ? *p + b : *p - b);
    };
    if (eob_run) {
      --eob_run;
      for (int k = spec_start; k <= spec_end; ++k) {
        int16_t *p = &d[kZigzag[k]];
        if (*p != 0) refine(p);
      }
      return true;
    }
    int k = spec_start;
    do {
      const int rs = decode(ha);
      if (rs < 0) return false;
      int s = rs & 15, r = rs >> 4;
      if (s == 0) {
        if (r < 15) {
          eob_run = (1 << r) - 1;
          if (r) eob_run += bits(r);
          r = 64;   // the rest of the band: corrections only
        }
      } else {
        if (s != 1) return false;
        s = bit() ? b : -b;
      }
      while (k <= spec_end) {
        int16_t *p = &d[kZigzag[k++]];
        if (*p != 0) {
          refine(p);
        } else {
          if (r == 0) { *p = static_cast<int16_t>(s); break; }
          --r;
        }
      }
    } while (k <= spec_end);
    return true;
  }

  bool end_of_mcu() {   // restart interval bookkeeping; false = stop the scan (not an error)
    if (--todo > 0) return true;
    if (code_bits < 24) fill();
    if (!(marker >= 0xd0 && marker <= 0xd7)) return false;
    reset();
    return true;
  }

  bool scan_data() {
    reset();
    alignas(16) int16_t d[64];
    if (scan_n == 1) {   // non-interleaved: the component's own blocks in raster order
      const int c = order[0];
      const int bw = (comp[c].x + 7) >> 3, bh = (comp[c].y + 7) >> 3;
      for (int j = 0; j < bh; ++j)
        for (int i = 0; i < bw; ++i) {
          if (!progressive) {
            if (!block(d, c)) return false;
            idct(comp[c].data.data() + comp[c].w2 * j * 8 + i * 8, comp[c].w2, d);
          } else {
            int16_t *cd = comp[c].coeff.data() + 64 * (i + j * comp[c].coeff_w);
            if (spec_start == 0 ? !block_dc(cd, c) : !block_ac(cd, c)) return false;
          }
          if (!end_of_mcu()) return true;
        }
      return true;
    }
    for (int j = 0; j < mcu_y; ++j)
      for (int i = 0; i < mcu_x; ++i) {
        for (int k = 0; k < scan_n; ++k) {
          const int c = order[k];
          for (int y = 0; y < comp[c].v; ++y)
            for (int x = 0; x < comp[c].h; ++x) {
              const int bx = i * comp[c].h + x, by = j * comp[c].v + y;
              if (!progressive) {
                if (!block(d, c)) return false;
                idct(comp[c].data.data() + comp[c].w2 * by * 8 + bx * 8, comp[c].w2, d);
              } else {
                if (!block_dc(comp[c].coeff.data() + 64 * (bx + by * comp[c].coeff_w), c)) return false;
              }
            }
        }
        if (!end_of_mcu()) return true;
      }
    return true;
  }

  // ---- islow inverse DCT (A.3.3 / jidctint), 12-bit constants ----
  // Evaluated with the integer widths of the SSE2 flow stb_image uses on x86-64 (stbi__idct_simd,
  // stb_image.h:2530): 16-bit lanes in and between the passes (sums of two inputs wrap, pass results
  // saturate), products and butterflies in 32-bit lanes.  On coefficients that stay in range this is the
  // same number as the plain 32-bit islow; on the overflowing values of a corrupt file it is stb's.
  static int32_t w32(int64_t v) { return static_cast<int32_t>(static_cast<uint32_t>(static_cast<uint64_t>(v))); }
  static int16_t w16(int v) { return static_cast<int16_t>(static_cast<uint16_t>(v)); }
  static int16_t sat16(int32_t v) { return static_cast<int16_t>(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
  // one 1-D pass over r[0..7] (one lane); constants (int)(c * 4096 + 0.5), pre-summed as stb's rotations
  static void idct_pass(int16_t r[8], int32_t bias, int shift) {
    auto rot = [](int x, int y, int cx, int cy) { return w32(static_cast<int64_t>(x) * cx + static_cast<int64_t>(y) * cy); };
    const int32_t t2e = rot(r[2], r[6], 2217, 2217 - 7567), t3e = rot(r[2], r[6], 2217 + 3135, 2217);
    const int32_t t0e = w32(static_cast<int64_t>(w16(r[0] + r[4])) * 4096), t1e = w32(static_cast<int64_t>(w16(r[0] - r[4])) * 4096);
    const int32_t x0 = w32(int64_t(t0e) + t3e), x3 = w32(int64_t(t0e) - t3e);
    const int32_t x1 = w32(int64_t(t1e) + t2e), x2 = w32(int64_t(t1e) - t2e);
    const int32_t y0 = rot(r[7], r[3], -8034 + 1223, -8034), y2 = rot(r[7], r[3], -8034, -8034 + 12586);
    const int32_t y1 = rot(r[5], r[1], -1597 + 8410, -1597), y3 = rot(r[5], r[1], -1597, -1597 + 6149);
    const int s17 = w16(r[1] + r[7]), s35 = w16(r[3] + r[5]);
    const int32_t y4 = rot(s17, s35, 4816 - 3685, 4816), y5 = rot(s17, s35, 4816, 4816 - 10497);
    const int32_t x4 = w32(int64_t(y0) + y4), x5 = w32(int64_t(y1) + y5), x6 = w32(int64_t(y2) + y5), x7 = w32(int64_t(y3) + y4);
    auto out = [&](int32_t a, int32_t b, bool sum) {
      const int32_t ab = w32(int64_t(a) + bias);
      return sat16(w32(sum ? int64_t(ab) + b : int64_t(ab) - b) >> shift);
    };
    r[0] = out(x0, x7, true); r[7] = out(x0, x7, false);
    r[1] = out(x1, x6, true); r[6] = out(x1, x6, false);
    r[2] = out(x2, x5, true); r[5] = out(x2, x5, false);
    r[3] = out(x3, x4, true); r[4] = out(x3, x4, false);
  }
  static void idct(uint8_t *out, int stride, const int16_t *d) {
    int16_t col[8][8];   // col[j] = column j of the block, top to bottom
    for (int j = 0; j < 8; ++j) {
      for (int k = 0; k < 8; ++k) col[j][k] = d[8 * k + j];
      idct_pass(col[j], 512, 10);   // columns: keep 2 extra bits
    }
    for (int i = 0; i < 8; ++i, out += stride) {   // rows: remove 2^17, re-centre on 128
      int16_t row[8];
      for (int k = 0; k < 8; ++k) row[k] = col[k][i];
      idct_pass(row, 65536 + (128 << 17), 17);
      for (int k = 0; k < 8; ++k) out[k] = static_cast<uint8_t>(row[k] < 0 ? 0 : (row[k] > 255 ? 255 : row[k]));
    }
  }

  // ---- markers ----
  bool table_or_app(uint8_t m) {
    if (m == kNoMarker) return false;
    if (m == 0xdd) {   // DRI
      if (get16() != 4) return false;
      restart_interval = static_cast<int>(get16());
      return true;
    }
    if (m == 0xdb) {   // DQT
      long L = static_cast<long>(get16()) - 2;
      while (L > 0) {
        const uint32_t q = get8();
        const int p = q >> 4, t = q & 15;
        if (p > 1 || t > 3) return false;
        for (int i = 0; i < 64; ++i) dequant[t][kZigzag[i]] = static_cast<uint16_t>(p ? get16() : get8());
        L -= p ? 129 : 65;
      }
      return L == 0;
    }
    if (m == 0xc4) {   // DHT
      long L = static_cast<long>(get16()) - 2;
      while (L > 0) {
        const uint32_t q = get8();
        const int tc = q >> 4, th = q & 15;
        if (tc > 1 || th > 3) return false;
        int counts[16], total = 0;
        for (int i = 0; i < 16; ++i) { counts[i] = static_cast<int>(get8()); total += counts[i]; }
        if (total > 256) return false;
        L -= 17;
        Huffman &h = tc ? hac[th] : hdc[th];
        if (!h.build(counts)) return false;
        for (int i = 0; i < total; ++i) h.values[i] = static_cast<uint8_t>(get8());
        if (tc) h.build_fast_ac();
        L -= total;
      }
      return L == 0;
    }
    if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {   // APPn, COM
      long L = static_cast<long>(get16());
      if (L < 2) return false;
      L -= 2;
      if (m == 0xe0 && L >= 5) {   // JFIF
        static const uint8_t tag[5] = {'J', 'F', 'I', 'F', 0};
        bool ok = true;
        for (int i = 0; i < 5; ++i) ok = (get8() == tag[i]) && ok;
        L -= 5;
        if (ok) jfif = true;
      } else if (m == 0xee && L >= 12) {   // Adobe: colour transform flag
        static const uint8_t tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
        bool ok = true;
        for (int i = 0; i < 6; ++i) ok = (get8() == tag[i]) && ok;
        L -= 6;
        if (ok) {
          get8(); get16(); get16();
          adobe = static_cast<int>(get8());
          L -= 6;
        }
      }
      skip(L);
      return true;
    }
    return false;
  }

  bool frame_header() {
    const uint32_t Lf = get16();
    if (Lf < 11) return false;
    if (get8() != 8) return false;   // 8-bit samples only
    img_y = static_cast<int>(get16());
    if (img_y == 0) return false;
    img_x = static_cast<int>(get16());
    if (img_x == 0) return false;
    if (img_x > (1 << 24) || img_y > (1 << 24)) return false;
    img_n = static_cast<int>(get8());
    if (img_n != 1 && img_n != 3 && img_n != 4) return false;
    if (Lf != static_cast<uint32_t>(8 + 3 * img_n)) return false;
    static const uint8_t rgb[3] = {'R', 'G', 'B'};
    rgb_ids = 0;
    for (int i = 0; i < img_n; ++i) {
      comp[i].id = static_cast<int>(get8());
      if (img_n == 3 && comp[i].id == rgb[i]) ++rgb_ids;
      const uint32_t q = get8();
      comp[i].h = static_cast<int>(q >> 4);
      comp[i].v = static_cast<int>(q & 15);
      if (comp[i].h < 1 || comp[i].h > 4 || comp[i].v < 1 || comp[i].v > 4) return false;
      comp[i].tq = static_cast<int>(get8());
      if (comp[i].tq > 3) return false;
    }
    // stb's size guard: img_x * img_y * img_n must stay below 2^31
    if (static_cast<long long>(img_x) * img_y * img_n >= (1ll << 31)) return false;
    for (int i = 0; i < img_n; ++i) { hmax = std::max(hmax, comp[i].h); vmax = std::max(vmax, comp[i].v); }
    for (int i = 0; i < img_n; ++i)
      if (hmax % comp[i].h || vmax % comp[i].v) return false;
    mcu_x = (img_x + hmax * 8 - 1) / (hmax * 8);
    mcu_y = (img_y + vmax * 8 - 1) / (vmax * 8);
    for (int i = 0; i < img_n; ++i) {
      Component &c = comp[i];
      c.x = (img_x * c.h + hmax - 1) / hmax;
      c.y = (img_y * c.v + vmax - 1) / vmax;
      c.w2 = mcu_x * c.h * 8;
      c.h2 = mcu_y * c.v * 8;
      c.data.assign(static_cast<size_t>(c.w2) * c.h2, 0);
      if (progressive) {
        c.coeff_w = c.w2 / 8;
        c.coeff.assign(static_cast<size_t>(c.w2) * c.h2, 0);
      }
    }
    return true;
  }

  bool scan_header() {
    const uint32_t Ls = get16();
    scan_n = static_cast<int>(get8());
    if (scan_n < 1 || scan_n > 4 || scan_n > img_n) return false;
    if (Ls != static_cast<uint32_t>(6 + 2 * scan_n)) return false;
    for (int i = 0; i < scan_n; ++i) {
      const int id = static_cast<int>(get8());
      const uint32_t q = get8();
      int which = 0;
      while (which < img_n && comp[which].id != id) ++which;
      if (which == img_n) return false;
      comp[which].hd = static_cast<int>(q >> 4);
      comp[which].ha = static_cast<int>(q & 15);
      if (comp[which].hd > 3 || comp[which].ha > 3) return false;
      order[i] = which;
    }
    spec_start = static_cast<int>(get8());
    spec_end = static_cast<int>(get8());
    const uint32_t aa = get8();
    succ_high = static_cast<int>(aa >> 4);
    succ_low = static_cast<int>(aa & 15);
    if (progressive) {
      if (spec_start > 63 || spec_end > 63 || spec_start > spec_end || succ_high > 13 || succ_low > 13) return false;
    } else {
      if (spec_start != 0 || succ_high != 0 || succ_low != 0) return false;
      spec_end = 63;
    }
    return true;
  }

  uint8_t skip_junk() {   // after a scan: bytes up to the next marker
    while (!at_eof()) {
      uint32_t x = get8();
      while (x == 0xff) {
        if (at_eof()) return kNoMarker;
        x = get8();
        if (x != 0x00 && x != 0xff) return static_cast<uint8_t>(x);
      }
    }
    return kNoMarker;
  }

  bool decode_image() {
    marker = kNoMarker;
    if (next_marker() != 0xd8) return false;   // SOI
    uint8_t m = next_marker();
    while (!(m == 0xc0 || m == 0xc1 || m == 0xc2)) {
      if (!table_or_app(m)) return false;
      m = next_marker();
      while (m == kNoMarker) {
        if (at_eof()) return false;
        m = next_marker();
      }
    }
    progressive = m == 0xc2;
    if (!frame_header()) return false;
    m = next_marker();
    while (m != 0xd9) {   // EOI
      if (m == 0xda) {   // SOS
        if (!scan_header()) return false;
        if (!scan_data()) return false;
        if (marker == kNoMarker) marker = skip_junk();
        m = next_marker();
        if (m >= 0xd0 && m <= 0xd7) m = next_marker();
      } else if (m == 0xdc) {   // DNL
        const uint32_t Ld = get16(), NL = get16();
        if (Ld != 4 || NL != static_cast<uint32_t>(img_y)) return false;
        m = next_marker();
      } else {
        // an unknown or missing marker ends the image as decoded so far: stb returns success without
        // the progressive finishing pass, so such an image's planes stay as allocated (zeros here)
        if (!table_or_app(m)) return true;
        m = next_marker();
      }
    }
    if (progressive)
      for (int c = 0; c < img_n; ++c) {
        const int bw = (comp[c].x + 7) >> 3, bh = (comp[c].y + 7) >> 3;
        for (int j = 0; j < bh; ++j)
          for (int i = 0; i < bw; ++i) {
            int16_t *d = comp[c].coeff.data() + 64 * (i + j * comp[c].coeff_w);
            for (int k = 0; k < 64; ++k) d[k] = static_cast<int16_t>(d[k] * dequant[comp[c].tq][k]);
            idct(comp[c].data.data() + comp[c].w2 * j * 8 + i * 8, comp[c].w2, d);
          }
      }
    return true;
  }
};

// ---- upsampling of one output row of a component (its "near" and "far" input rows) ----
void upsample(uint8_t *out, const uint8_t *near, const uint8_t *far, int w, int hs, int vs, const uint8_t **res) {
  if (hs == 1 && vs == 1) { *res = near; return; }
  *res = out;
  if (hs == 1 && vs == 2) {
    for (int i = 0; i < w; ++i) out[i] = static_cast<uint8_t>((3 * near[i] + far[i] + 2) >> 2);
  } else if (hs == 2 && vs == 1) {
    if (w == 1) { out[0] = out[1] = near[0]; return; }
    out[0] = near[0];
    out[1] = static_cast<uint8_t>((near[0] * 3 + near[1] + 2) >> 2);
    int i;
    for (i = 1; i < w - 1; ++i) {
      const int c = 3 * near[i] + 2;
      out[2 * i] = static_cast<uint8_t>((c + near[i - 1]) >> 2);
      out[2 * i + 1] = static_cast<uint8_t>((c + near[i + 1]) >> 2);
    }
    out[2 * i] = static_cast<uint8_t>((near[w - 2] * 3 + near[w - 1] + 2) >> 2);
    out[2 * i + 1] = near[w - 1];
  } else if (hs == 2 && vs == 2) {
    if (w == 1) { out[0] = out[1] = static_cast<uint8_t>((3 * near[0] + far[0] + 2) >> 2); return; }
    int t1 = 3 * near[0] + far[0];
    out[0] = static_cast<uint8_t>((t1 + 2) >> 2);
    for (int i = 1; i < w; ++i) {
      const int t0 = t1;
      t1 = 3 * near[i] + far[i];
      out[2 * i - 1] = static_cast<uint8_t>((3 * t0 + t1 + 8) >> 4);
      out[2 * i] = static_cast<uint8_t>((3 * t1 + t0 + 8) >> 4);
    }
    out[2 * w - 1] = static_cast<uint8_t>((t1 + 2) >> 2);
  } else {
    for (int i = 0; i < w; ++i)
      for (int j = 0; j < hs; ++j) out[i * hs + j] = near[i];
  }
}

inline uint8_t blinn(uint8_t x, uint8_t y) {   // x * y / 255, rounded
  const unsigned t = static_cast<unsigned>(x) * y + 128u;
  return static_cast<uint8_t>((t + (t >> 8)) >> 8);
}

void ycbcr_row(uint8_t *out, const uint8_t *y, const uint8_t *cb, const uint8_t *cr, int count) {
  // 1.40200, 0.71414, 0.34414, 1.77200 as (int)(c * 4096 + 0.5) << 8
  constexpr int kCr = 5743 << 8, kCrG = 2925 << 8, kCbG = 1410 << 8, kCb = 7258 << 8;
  for (int i = 0; i < count; ++i, out += 3) {
    const int yf = (y[i] << 20) + (1 << 19);
    const int vr = cr[i] - 128, vb = cb[i] - 128;
    int r = yf + vr * kCr;
    int g = yf + vr * -kCrG + static_cast<int>(static_cast<unsigned>(vb * -kCbG) & 0xffff0000u);
    int b = yf + vb * kCb;
    r >>= 20; g >>= 20; b >>= 20;
    out[0] = static_cast<uint8_t>(r < 0 ? 0 : (r > 255 ? 255 : r));
    out[1] = static_cast<uint8_t>(g < 0 ? 0 : (g > 255 ? 255 : g));
    out[2] = static_cast<uint8_t>(b < 0 ? 0 : (b > 255 ? 255 : b));
  }
}

}  // namespace

bool is_jpeg(const uint8_t *b, size_t n) {
  // stb's test: the SOI marker (with any 0xFF fill before it)
  size_t p = 0;
  if (p >= n || b[p] != 0xff) return false;
  while (p < n && b[p] == 0xff) ++p;
  return p < n && b[p] == 0xd8;
}

// 8-bit RGB texels, rows top first; false where stbi_loadf fails
bool decode(const uint8_t *b, size_t n, std::vector<uint8_t> *rgb, int *w, int *h) {
  Decoder z(b, n);
  if (!z.decode_image()) return false;
  const int W = z.img_x, H = z.img_y;
  const bool is_rgb = z.img_n == 3 && (z.rgb_ids == 3 || (z.adobe == 0 && !z.jfif));
  struct Res { int hs, vs, ystep, w_lores, ypos; const uint8_t *line0, *line1; std::vector<uint8_t> buf; };
  Res res[4];
  for (int k = 0; k < z.img_n; ++k) {
    Res &r = res[k];
    r.hs = z.hmax / z.comp[k].h;
    r.vs = z.vmax / z.comp[k].v;
    r.ystep = r.vs >> 1;
    r.w_lores = (W + r.hs - 1) / r.hs;
    r.ypos = 0;
    r.line0 = r.line1 = z.comp[k].data.data();
    r.buf.assign(static_cast<size_t>(W) + 3, 0);
  }
  rgb->assign(static_cast<size_t>(W) * H * 3, 0);
  const uint8_t *co[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int j = 0; j < H; ++j) {
    uint8_t *out = rgb->data() + static_cast<size_t>(W) * 3 * j;
    for (int k = 0; k < z.img_n; ++k) {
      Res &r = res[k];
      const bool bot = r.ystep >= (r.vs >> 1);
      upsample(r.buf.data(), bot ? r.line1 : r.line0, bot ? r.line0 : r.line1, r.w_lores, r.hs, r.vs, &co[k]);
      if (++r.ystep >= r.vs) {
        r.ystep = 0;
        r.line0 = r.line1;
        if (++r.ypos < z.comp[k].y) r.line1 += z.comp[k].w2;
      }
    }
    if (z.img_n == 3) {
      if (is_rgb) {
        for (int i = 0; i < W; ++i) { out[3 * i] = co[0][i]; out[3 * i + 1] = co[1][i]; out[3 * i + 2] = co[2][i]; }
      } else {
        ycbcr_row(out, co[0], co[1], co[2], W);
      }
    } else if (z.img_n == 4) {
      if (z.adobe == 0) {   // CMYK
        for (int i = 0; i < W; ++i) {
          const uint8_t m = co[3][i];
          out[3 * i] = blinn(co[0][i], m); out[3 * i + 1] = blinn(co[1][i], m); out[3 * i + 2] = blinn(co[2][i], m);
        }
      } else if (z.adobe == 2) {   // YCCK
        ycbcr_row(out, co[0], co[1], co[2], W);
        for (int i = 0; i < W; ++i) {
          const uint8_t m = co[3][i];
          for (int c = 0; c < 3; ++c) out[3 * i + c] = blinn(static_cast<uint8_t>(255 - out[3 * i + c]), m);
        }
      } else {   // YCbCr + a fourth channel that is ignored
        ycbcr_row(out, co[0], co[1], co[2], W);
      }
    } else {
      for (int i = 0; i < W; ++i) out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = co[0][i];
    }
  }
  *w = W;
  *h = H;
  return true;
}

}  // namespace jpeg
}  // namespace rt
