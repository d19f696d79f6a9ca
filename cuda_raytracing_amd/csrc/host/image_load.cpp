// image_load.cpp — image files for image textures (make_image_texture, raytracing.cu:332-341).
//
// The reference loads texels with stbi_loadf(file, &w, &h, &n, 3) from stb_image v2.30 (the third-party
// header it vendors as include/stb_image.h): three float channels per texel, row 0 = the top row of the
// picture; Radiance HDR texels as stored, every 8-bit format converted by pow(c / 255, 2.2) * 1 (stb's
// default LDR->float gamma and scale).  This file restates that loader for this project:
//   - the order in which it tries the formats (stbi__loadf_main, stb_image.h:1460; stbi__load_main :1137):
//     HDR, then PNG, BMP, GIF, PSD, PIC, JPEG, binary PNM and TGA last (TGA has no magic number);
//   - its FILE reader (stbi__start_file :877 and the context functions :1597-1689): a 128-byte buffer
//     refilled by fread, zeros once the file is exhausted, "rewind" back to the first buffer after each
//     format test, skips by fseek — so truncated and odd files read the same bytes as they do there;
//   - the BMP (:5346-5732), TGA (:5739-6074), PSD (:6081-6325), Softimage PIC (:6336-6546), GIF (:6553-7081,
//     the first image), PNM (:7494-7629) and HDR (:7087-7287) decoders; JPEG and PNG are image_jpeg.cpp and
//     image_png.cpp.
// A file that does not exist, is of no known type or fails to decode is the reference's failed load,
// RT_IMAGE_MISSING: no pixels, the texture renders magenta (:346-347).  Two deliberate differences: where stb
// "succeeds" with a zero-area image (a BMP, HDR, GIF, PSD or PIC header saying width 0), the reference's texel
// lookup would index outside the buffer; and where a corrupt PIC file of non-zero area fails stb's core loop, stb
// converts the NULL it got back and faults.  Both are RT_IMAGE_MISSING here.
// The BMP helpers high_bit / bitcount / shiftsigned are stb's (:5370-5413) with the same tables.
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
#include <array>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "image_decoders.h"
#include "rt_host.h"

namespace {

constexpr uint32_t kMaxDim = 1u << 24;   // STBI_MAX_DIMENSIONS

// stbi__ldr_to_hdr: (float) pow(c / 255.0f, stbi__l2h_gamma = 2.2f) * stbi__l2h_scale = 1.0f, in float
// (the float overload of pow in a C++ translation unit)
// (a function-local static initialised once, thread-safely: worlds may be built concurrently)
const float *ldr_table() {
  static const std::array<float, 256> t = [] {
    std::array<float, 256> v{};
    for (int c = 0; c < 256; ++c) v[c] = std::pow(static_cast<float>(c) / 255.0f, 2.2f) * 1.0f;
    return v;
  }();
  return t.data();
}

// stbi__mul2sizes_valid / stbi__addsizes_valid / stbi__mad3sizes_valid / stbi__mad4sizes_valid (:1002-1043)
bool mul2_ok(int a, int b) { return a >= 0 && b >= 0 && (b == 0 || a <= INT_MAX / b); }
bool add_ok(int a, int b) { return b >= 0 && a <= INT_MAX - b; }
bool mad3_ok(int a, int b, int c, int add) { return mul2_ok(a, b) && mul2_ok(a * b, c) && add_ok(a * b * c, add); }
bool mad4_ok(int a, int b, int c, int d, int add) {
  return mul2_ok(a, b) && mul2_ok(a * b, c) && mul2_ok(a * b * c, d) && add_ok(a * b * c * d, add);
}

// stb's context over a FILE opened by stbi_loadf, with the file held in memory: fpos_ is the FILE's
// position, eof_ its end-of-file flag, buf_ the context's 128-byte buffer_start.
class StbFile {
 public:
  explicit StbFile(const std::vector<uint8_t> &f) : f_(f) {   // stbi__start_callbacks
    refill();
    orig_end_ = end_;
  }
  uint32_t get8() {
    if (cur_ < end_) return buf_[cur_++];
    if (from_file_) {
      refill();
      return buf_[cur_++];
    }
    return 0;
  }
  int get16le() { const int z = static_cast<int>(get8()); return z + (static_cast<int>(get8()) << 8); }
  uint32_t get32le() { const uint32_t z = static_cast<uint32_t>(get16le()); return z + (static_cast<uint32_t>(get16le()) << 16); }
  int get16be() { const int z = static_cast<int>(get8()); return (z << 8) + static_cast<int>(get8()); }
  uint32_t get32be() { const uint32_t z = static_cast<uint32_t>(get16be()); return (z << 16) + static_cast<uint32_t>(get16be()); }
  void skip(int n) {
    if (n == 0) return;
    if (n < 0) { cur_ = end_; return; }
    const int blen = end_ - cur_;
    if (blen < n) {   // stbi__stdio_skip: fseek (clears EOF), then fgetc / ungetc (sets it at the end)
      cur_ = end_;
      fpos_ += static_cast<size_t>(n - blen);
      eof_ = fpos_ >= f_.size();
      return;
    }
    cur_ += n;
  }
  bool getn(uint8_t *out, int n) {
    const int blen = end_ - cur_;
    if (blen < n) {
      std::memcpy(out, buf_ + cur_, static_cast<size_t>(blen));
      const size_t want = static_cast<size_t>(n - blen);
      const size_t got = fread(out + blen, want);
      cur_ = end_;
      return got == want;
    }
    std::memcpy(out, buf_ + cur_, static_cast<size_t>(n));
    cur_ += n;
    return true;
  }
  bool at_eof() const {
    if (!eof_) return false;
    if (!from_file_) return true;
    return cur_ >= end_;
  }
  void rewind() { cur_ = 0; end_ = orig_end_; }
  int bytes_read() const { return already_read_ + cur_; }   // callback_already_read + (img_buffer - original)

 private:
  size_t fread(uint8_t *dst, size_t n) {
    const size_t avail = fpos_ < f_.size() ? f_.size() - fpos_ : 0, k = std::min(n, avail);
    if (k) std::memcpy(dst, f_.data() + fpos_, k);
    fpos_ += k;
    if (k < n) eof_ = true;
    return k;
  }
  void refill() {   // stbi__refill_buffer
    const size_t n = fread(buf_, sizeof buf_);
    already_read_ += cur_;
    cur_ = 0;
    if (n == 0) {
      from_file_ = false;
      end_ = 1;
      buf_[0] = 0;
    } else {
      end_ = static_cast<int>(n);
    }
  }

  const std::vector<uint8_t> &f_;
  size_t fpos_ = 0;
  bool eof_ = false, from_file_ = true;
  uint8_t buf_[128] = {0};
  int cur_ = 0, end_ = 0, orig_end_ = 0, already_read_ = 0;
};

// ---- format tests (each leaves the context rewound, except a PNM match) ----

bool png_test(StbFile &s) {   // stbi__check_png_header
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  bool r = true;
  for (int i = 0; i < 8 && r; ++i) r = s.get8() == sig[i];
  s.rewind();
  return r;
}

bool bmp_test(StbFile &s) {
  bool r = s.get8() == 'B' && s.get8() == 'M';
  if (r) {
    s.get32le(); s.get16le(); s.get16le(); s.get32le();
    const uint32_t sz = s.get32le();
    r = sz == 12 || sz == 40 || sz == 56 || sz == 108 || sz == 124;
  }
  s.rewind();
  return r;
}

bool gif_test(StbFile &s) {
  bool r = s.get8() == 'G' && s.get8() == 'I' && s.get8() == 'F' && s.get8() == '8';
  if (r) {
    const uint32_t sz = s.get8();
    r = (sz == '9' || sz == '7') && s.get8() == 'a';
  }
  s.rewind();
  return r;
}

bool psd_test(StbFile &s) {
  const bool r = s.get32be() == 0x38425053u;
  s.rewind();
  return r;
}

bool pic_is4(StbFile &s, const char *str) {
  for (int i = 0; i < 4; ++i)
    if (s.get8() != static_cast<uint8_t>(str[i])) return false;
  return true;
}

bool pic_test(StbFile &s) {
  bool r = pic_is4(s, "\x53\x80\xF6\x34");
  if (r) {
    for (int i = 0; i < 84; ++i) s.get8();
    r = pic_is4(s, "PICT");
  }
  s.rewind();
  return r;
}

bool jpeg_test(StbFile &s) {   // stbi__decode_jpeg_header(SCAN_type): stbi__get_marker() == SOI
  uint32_t x = s.get8();
  bool r = false;
  if (x == 0xff) {
    while (x == 0xff) x = s.get8();
    r = x == 0xd8;
  }
  s.rewind();
  return r;
}

bool pnm_test(StbFile &s) {
  const char p = static_cast<char>(s.get8()), t = static_cast<char>(s.get8());
  if (p != 'P' || (t != '5' && t != '6')) {
    s.rewind();
    return false;
  }
  return true;
}

bool hdr_test_core(StbFile &s, const char *signature) {
  for (int i = 0; signature[i]; ++i)
    if (s.get8() != static_cast<uint8_t>(signature[i])) return false;
  s.rewind();
  return true;
}

bool hdr_test(StbFile &s) {
  bool r = hdr_test_core(s, "#?RADIANCE\n");
  s.rewind();
  if (!r) {
    r = hdr_test_core(s, "#?RGBE\n");
    s.rewind();
  }
  return r;
}

int tga_get_comp(int bits_per_pixel, bool is_grey, int *is_rgb16) {
  if (is_rgb16) *is_rgb16 = 0;
  switch (bits_per_pixel) {
    case 8: return 1;
    case 16:
      if (is_grey) return 2;
      [[fallthrough]];
    case 15:
      if (is_rgb16) *is_rgb16 = 1;
      return 3;
    case 24:
    case 32: return bits_per_pixel / 8;
    default: return 0;
  }
}

bool tga_test(StbFile &s) {
  bool r = false;
  do {
    s.get8();   // offset
    const uint32_t color_type = s.get8();
    if (color_type > 1) break;
    uint32_t sz = s.get8();   // image type
    if (color_type == 1) {
      if (sz != 1 && sz != 9) break;
      s.skip(4);
      sz = s.get8();   // palette entry bits
      if (sz != 8 && sz != 15 && sz != 16 && sz != 24 && sz != 32) break;
      s.skip(4);
    } else {
      if (sz != 2 && sz != 3 && sz != 10 && sz != 11) break;
      s.skip(9);
    }
    if (s.get16le() < 1) break;
    if (s.get16le() < 1) break;
    sz = s.get8();   // bits per pixel
    if (color_type == 1 && sz != 8 && sz != 16) break;
    if (sz != 8 && sz != 15 && sz != 16 && sz != 24 && sz != 32) break;
    r = true;
  } while (false);
  s.rewind();
  return r;
}

// ---- decoders: 8-bit texels with `comp` channels, rows top first ----

struct Pixels {
  std::vector<uint8_t> px;
  int w = 0, h = 0, comp = 3;
};

void bmp_mask_defaults(int bpp, int compress, uint32_t *mr, uint32_t *mg, uint32_t *mb, uint32_t *ma) {
  if (compress != 0) return;   // BI_BITFIELDS keeps its masks; other values leave them as read
  if (bpp == 16) {
    *mr = 31u << 10; *mg = 31u << 5; *mb = 31u;
  } else if (bpp == 32) {
    *mr = 0xffu << 16; *mg = 0xffu << 8; *mb = 0xffu; *ma = 0xffu << 24;
  } else {
    *mr = *mg = *mb = *ma = 0;
  }
}

int high_bit(uint32_t z) {
  if (z == 0) return -1;
  int n = 0;
  if (z >= 0x10000) { n += 16; z >>= 16; }
  if (z >= 0x00100) { n += 8; z >>= 8; }
  if (z >= 0x00010) { n += 4; z >>= 4; }
  if (z >= 0x00004) { n += 2; z >>= 2; }
  if (z >= 0x00002) n += 1;
  return n;
}

int bitcount(uint32_t a) {
  a = (a & 0x55555555u) + ((a >> 1) & 0x55555555u);
  a = (a & 0x33333333u) + ((a >> 2) & 0x33333333u);
  a = (a + (a >> 4)) & 0x0f0f0f0fu;
  a = a + (a >> 8);
  a = a + (a >> 16);
  return static_cast<int>(a & 0xff);
}

// an arbitrarily aligned field of `bits` bits, widened to 8 bits by repeating its bit pattern
int shiftsigned(uint32_t v, int shift, int bits) {
  static const uint32_t mul[9] = {0, 0xff, 0x55, 0x49, 0x11, 0x21, 0x41, 0x81, 0x01};
  static const int rsh[9] = {0, 0, 0, 1, 0, 2, 4, 6, 0};
  if (shift < 0) v <<= -shift;
  else v >>= shift;
  v >>= (8 - bits);
  return static_cast<int>(v * mul[bits]) >> rsh[bits];
}

bool bmp_load(StbFile &s, Pixels *o) {
  // stbi__bmp_parse_header
  if (s.get8() != 'B' || s.get8() != 'M') return false;
  s.get32le(); s.get16le(); s.get16le();
  const int offset = static_cast<int>(s.get32le());
  const int hsz = static_cast<int>(s.get32le());
  uint32_t mr = 0, mg = 0, mb = 0, ma = 0;
  int extra_read = 14;
  if (offset < 0) return false;
  if (hsz != 12 && hsz != 40 && hsz != 56 && hsz != 108 && hsz != 124) return false;
  uint32_t img_x, img_y;
  if (hsz == 12) {
    img_x = static_cast<uint32_t>(s.get16le());
    img_y = static_cast<uint32_t>(s.get16le());
  } else {
    img_x = s.get32le();
    img_y = s.get32le();
  }
  if (s.get16le() != 1) return false;
  const int bpp = s.get16le();
  if (hsz != 12) {
    const int compress = static_cast<int>(s.get32le());
    if (compress == 1 || compress == 2) return false;   // RLE
    if (compress >= 4) return false;                    // JPEG / PNG payloads
    if (compress == 3 && bpp != 16 && bpp != 32) return false;
    for (int i = 0; i < 5; ++i) s.get32le();   // size, resolutions, colours used / important
    if (hsz == 40 || hsz == 56) {
      if (hsz == 56)
        for (int i = 0; i < 4; ++i) s.get32le();
      if (bpp == 16 || bpp == 32) {
        if (compress == 0) {
          bmp_mask_defaults(bpp, compress, &mr, &mg, &mb, &ma);
        } else if (compress == 3) {
          mr = s.get32le(); mg = s.get32le(); mb = s.get32le();
          extra_read += 12;
          if (mr == mg && mg == mb) return false;
        } else {
          return false;
        }
      }
    } else {   // V4 / V5 header
      mr = s.get32le(); mg = s.get32le(); mb = s.get32le(); ma = s.get32le();
      if (compress != 3) bmp_mask_defaults(bpp, compress, &mr, &mg, &mb, &ma);
      for (int i = 0; i < 13; ++i) s.get32le();   // colour space and its parameters
      if (hsz == 124)
        for (int i = 0; i < 4; ++i) s.get32le();
    }
  }

  // stbi__bmp_load
  const bool flip = static_cast<int32_t>(img_y) > 0;
  if (static_cast<int32_t>(img_y) != INT_MIN) img_y = static_cast<uint32_t>(std::abs(static_cast<int32_t>(img_y)));
  if (img_y > kMaxDim || img_x > kMaxDim) return false;
  const int W = static_cast<int>(img_x), H = static_cast<int>(img_y);
  int psize = 0;
  if (hsz == 12) {
    if (bpp < 24) psize = (offset - extra_read - 24) / 3;
  } else {
    if (bpp < 16) psize = (offset - extra_read - hsz) >> 2;
  }
  if (psize == 0) {
    const int so_far = s.bytes_read();
    if (so_far <= 0 || so_far > 1024) return false;
    if (offset < so_far || offset - so_far > 256 * 4) return false;
    s.skip(offset - so_far);
  }
  const int target = 3;   // req_comp
  if (!mad3_ok(target, W, H, 0)) return false;
  o->px.assign(static_cast<size_t>(W) * H * target, 0);
  o->w = W;
  o->h = H;
  o->comp = target;
  uint8_t *out = o->px.data();
  size_t z = 0;
  if (bpp < 16) {
    if (psize == 0 || psize > 256) return false;
    uint8_t pal[256][4] = {};   // (entries past psize: stb's are uninitialised; zeros here)
    for (int i = 0; i < psize; ++i) {
      pal[i][2] = static_cast<uint8_t>(s.get8());
      pal[i][1] = static_cast<uint8_t>(s.get8());
      pal[i][0] = static_cast<uint8_t>(s.get8());
      if (hsz != 12) s.get8();
      pal[i][3] = 255;
    }
    s.skip(offset - extra_read - hsz - psize * (hsz == 12 ? 3 : 4));
    int width;
    if (bpp == 1) width = (W + 7) >> 3;
    else if (bpp == 4) width = (W + 1) >> 1;
    else if (bpp == 8) width = W;
    else return false;
    const int pad = (-width) & 3;
    if (bpp == 1) {
      for (int j = 0; j < H; ++j) {
        int bit_offset = 7, v = static_cast<int>(s.get8());
        for (int i = 0; i < W; ++i) {
          const int color = (v >> bit_offset) & 1;
          out[z++] = pal[color][0]; out[z++] = pal[color][1]; out[z++] = pal[color][2];
          if (i + 1 == W) break;
          if (--bit_offset < 0) {
            bit_offset = 7;
            v = static_cast<int>(s.get8());
          }
        }
        s.skip(pad);
      }
    } else {
      for (int j = 0; j < H; ++j) {
        for (int i = 0; i < W; i += 2) {
          int v = static_cast<int>(s.get8()), v2 = 0;
          if (bpp == 4) {
            v2 = v & 15;
            v >>= 4;
          }
          out[z++] = pal[v][0]; out[z++] = pal[v][1]; out[z++] = pal[v][2];
          if (i + 1 == W) break;
          v = bpp == 8 ? static_cast<int>(s.get8()) : v2;
          out[z++] = pal[v][0]; out[z++] = pal[v][1]; out[z++] = pal[v][2];
        }
        s.skip(pad);
      }
    }
  } else {
    int rshift = 0, gshift = 0, bshift = 0, rcount = 0, gcount = 0, bcount = 0, acount = 0;
    s.skip(offset - extra_read - hsz);
    const int width = bpp == 24 ? 3 * W : bpp == 16 ? 2 * W : 0;
    const int pad = (-width) & 3;
    int easy = 0;
    if (bpp == 24) easy = 1;
    else if (bpp == 32 && mb == 0xffu && mg == 0xff00u && mr == 0x00ff0000u && ma == 0xff000000u) easy = 2;
    if (!easy) {
      if (!mr || !mg || !mb) return false;
      rshift = high_bit(mr) - 7; rcount = bitcount(mr);
      gshift = high_bit(mg) - 7; gcount = bitcount(mg);
      bshift = high_bit(mb) - 7; bcount = bitcount(mb);
      acount = bitcount(ma);
      if (rcount > 8 || gcount > 8 || bcount > 8 || acount > 8) return false;
    }
    for (int j = 0; j < H; ++j) {
      if (easy) {
        for (int i = 0; i < W; ++i) {
          out[z + 2] = static_cast<uint8_t>(s.get8());
          out[z + 1] = static_cast<uint8_t>(s.get8());
          out[z + 0] = static_cast<uint8_t>(s.get8());
          z += 3;
          if (easy == 2) s.get8();   // alpha: dropped by the 3 requested channels
        }
      } else {
        for (int i = 0; i < W; ++i) {
          const uint32_t v = bpp == 16 ? static_cast<uint32_t>(s.get16le()) : s.get32le();
          out[z++] = static_cast<uint8_t>(shiftsigned(v & mr, rshift, rcount) & 255);
          out[z++] = static_cast<uint8_t>(shiftsigned(v & mg, gshift, gcount) & 255);
          out[z++] = static_cast<uint8_t>(shiftsigned(v & mb, bshift, bcount) & 255);
        }
      }
      s.skip(pad);
    }
  }
  if (flip) {
    const size_t row = static_cast<size_t>(W) * target;
    for (int j = 0; j < (H >> 1); ++j)
      std::swap_ranges(out + j * row, out + (j + 1) * row, out + static_cast<size_t>(H - 1 - j) * row);
  }
  return true;
}

void tga_read_rgb16(StbFile &s, uint8_t *out) {
  const uint32_t px = static_cast<uint16_t>(s.get16le());
  const int r = (px >> 10) & 31, g = (px >> 5) & 31, b = px & 31;
  out[0] = static_cast<uint8_t>((r * 255) / 31);
  out[1] = static_cast<uint8_t>((g * 255) / 31);
  out[2] = static_cast<uint8_t>((b * 255) / 31);
}

bool tga_load(StbFile &s, Pixels *o) {
  const int offset = static_cast<int>(s.get8());
  const int indexed = static_cast<int>(s.get8());
  int image_type = static_cast<int>(s.get8());
  const int pal_start = s.get16le(), pal_len = s.get16le(), pal_bits = static_cast<int>(s.get8());
  s.get16le(); s.get16le();   // x / y origin (unused by stb)
  const int W = s.get16le(), H = s.get16le(), bpp = static_cast<int>(s.get8());
  int inverted = static_cast<int>(s.get8());
  bool rle = false;
  if (image_type >= 8) {
    image_type -= 8;
    rle = true;
  }
  inverted = 1 - ((inverted >> 5) & 1);   // bottom-up unless the descriptor's bit 5 says top-down
  int rgb16 = 0;
  const int comp = indexed ? tga_get_comp(pal_bits, false, &rgb16) : tga_get_comp(bpp, image_type == 3, &rgb16);
  if (!comp) return false;
  if (!mad3_ok(W, H, comp, 0)) return false;
  std::vector<uint8_t> data(static_cast<size_t>(W) * H * comp, 0);
  s.skip(offset);
  if (!indexed && !rle && !rgb16) {
    for (int i = 0; i < H; ++i) {
      const int row = inverted ? H - i - 1 : i;
      s.getn(data.data() + static_cast<size_t>(row) * W * comp, W * comp);
    }
  } else {
    std::vector<uint8_t> pal;
    if (indexed) {
      if (pal_len == 0) return false;
      s.skip(pal_start);
      pal.assign(static_cast<size_t>(pal_len) * comp, 0);
      if (rgb16) {
        for (int i = 0; i < pal_len; ++i) tga_read_rgb16(s, &pal[static_cast<size_t>(i) * comp]);
      } else if (!s.getn(pal.data(), pal_len * comp)) {
        return false;
      }
    }
    uint8_t raw[4] = {0, 0, 0, 0};
    int rle_count = 0;
    bool rle_repeating = false, read_next = true;
    const size_t n = static_cast<size_t>(W) * H;
    for (size_t i = 0; i < n; ++i) {
      if (rle) {
        if (rle_count == 0) {
          const int cmd = static_cast<int>(s.get8());
          rle_count = 1 + (cmd & 127);
          rle_repeating = (cmd >> 7) != 0;
          read_next = true;
        } else if (!rle_repeating) {
          read_next = true;
        }
      } else {
        read_next = true;
      }
      if (read_next) {
        if (indexed) {
          int idx = bpp == 8 ? static_cast<int>(s.get8()) : s.get16le();
          if (idx >= pal_len) idx = 0;
          for (int j = 0; j < comp; ++j) raw[j] = pal[static_cast<size_t>(idx) * comp + j];
        } else if (rgb16) {
          tga_read_rgb16(s, raw);
        } else {
          for (int j = 0; j < comp; ++j) raw[j] = static_cast<uint8_t>(s.get8());
        }
        read_next = false;
      }
      for (int j = 0; j < comp; ++j) data[i * comp + j] = raw[j];
      --rle_count;
    }
    if (inverted) {
      const size_t row = static_cast<size_t>(W) * comp;
      for (int j = 0; j * 2 < H; ++j)
        std::swap_ranges(data.begin() + j * row, data.begin() + (j + 1) * row, data.begin() + (H - 1 - j) * row);
    }
  }
  if (comp >= 3 && !rgb16)   // stored B G R (A)
    for (size_t i = 0; i < data.size(); i += comp) std::swap(data[i], data[i + 2]);
  o->px = std::move(data);
  o->w = W;
  o->h = H;
  o->comp = comp;
  return true;
}

bool pnm_isspace(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }

void pnm_skip_whitespace(StbFile &s, char *c) {
  for (;;) {
    while (!s.at_eof() && pnm_isspace(*c)) *c = static_cast<char>(s.get8());
    if (s.at_eof() || *c != '#') break;
    while (!s.at_eof() && *c != '\n' && *c != '\r') *c = static_cast<char>(s.get8());
  }
}

int pnm_getinteger(StbFile &s, char *c) {
  int value = 0;
  while (!s.at_eof() && *c >= '0' && *c <= '9') {
    value = value * 10 + (*c - '0');
    *c = static_cast<char>(s.get8());
    if (value > 214748364 || (value == 214748364 && *c > '7')) return 0;   // overflow: stbi__err
  }
  return value;
}

bool pnm_load(StbFile &s, Pixels *o) {
  // stbi__pnm_info
  s.rewind();
  const char p = static_cast<char>(s.get8()), t = static_cast<char>(s.get8());
  if (p != 'P' || (t != '5' && t != '6')) return false;
  const int comp = t == '6' ? 3 : 1;
  char c = static_cast<char>(s.get8());
  pnm_skip_whitespace(s, &c);
  const int x = pnm_getinteger(s, &c);
  if (x == 0) return false;
  pnm_skip_whitespace(s, &c);
  const int y = pnm_getinteger(s, &c);
  if (y == 0) return false;
  pnm_skip_whitespace(s, &c);
  const int maxv = pnm_getinteger(s, &c);
  if (maxv > 65535) return false;
  const int bytes = maxv > 255 ? 2 : 1;
  // stbi__pnm_load
  if (static_cast<uint32_t>(y) > kMaxDim || static_cast<uint32_t>(x) > kMaxDim) return false;
  if (!mad4_ok(comp, x, y, bytes, 0)) return false;
  std::vector<uint8_t> raw(static_cast<size_t>(comp) * x * y * bytes, 0);
  if (!s.getn(raw.data(), static_cast<int>(raw.size()))) return false;
  // 16-bit samples are read into native (little-endian) words and reduced with >> 8
  // (stbi__convert_16_to_8): the sample's second byte
  o->px.resize(static_cast<size_t>(comp) * x * y);
  for (size_t i = 0; i < o->px.size(); ++i) o->px[i] = raw[i * bytes + bytes - 1];
  o->w = x;
  o->h = y;
  o->comp = comp;
  return true;
}

// stbi__hdr_gettoken (:7109)
const char *hdr_gettoken(StbFile &s, char *buffer) {
  constexpr int kBufLen = 1024;
  int len = 0;
  char c = static_cast<char>(s.get8());
  while (!s.at_eof() && c != '\n') {
    buffer[len++] = c;
    if (len == kBufLen - 1) {
      while (!s.at_eof() && s.get8() != '\n') {
      }
      break;
    }
    c = static_cast<char>(s.get8());
  }
  buffer[len] = 0;
  return buffer;
}

// stbi__hdr_convert for 3 channels: RGBE -> float, exponent bias 128 + 8
void hdr_convert(float *out, const uint8_t *in) {
  if (in[3] != 0) {
    const float f1 = static_cast<float>(std::ldexp(1.0f, in[3] - static_cast<int>(128 + 8)));
    out[0] = in[0] * f1;
    out[1] = in[1] * f1;
    out[2] = in[2] * f1;
  } else {
    out[0] = out[1] = out[2] = 0;
  }
}

bool hdr_load(StbFile &s, std::vector<float> *data, int *pw, int *ph) {
  char buffer[1024];
  const char *tok = hdr_gettoken(s, buffer);
  if (std::strcmp(tok, "#?RADIANCE") != 0 && std::strcmp(tok, "#?RGBE") != 0) return false;
  bool valid = false;
  for (;;) {
    tok = hdr_gettoken(s, buffer);
    if (tok[0] == 0) break;
    if (std::strcmp(tok, "FORMAT=32-bit_rle_rgbe") == 0) valid = true;
  }
  if (!valid) return false;
  char *t = const_cast<char *>(hdr_gettoken(s, buffer));
  if (std::strncmp(t, "-Y ", 3)) return false;
  t += 3;
  const int height = static_cast<int>(std::strtol(t, &t, 10));
  while (*t == ' ') ++t;
  if (std::strncmp(t, "+X ", 3)) return false;
  t += 3;
  const int width = static_cast<int>(std::strtol(t, nullptr, 10));
  if (height > static_cast<int>(kMaxDim) || width > static_cast<int>(kMaxDim)) return false;
  if (!mad4_ok(width, height, 3, static_cast<int>(sizeof(float)), 0)) return false;
  data->assign(static_cast<size_t>(width) * height * 3, 0.0f);
  *pw = width;
  *ph = height;
  float *out = data->data();
  int j0 = 0, i0 = 0;   // where flat reading starts
  bool flat = width < 8 || width >= 32768;
  if (!flat) {
    std::vector<uint8_t> scanline(static_cast<size_t>(width) * 4, 0);
    for (int j = 0; j < height; ++j) {
      const int c1 = static_cast<int>(s.get8()), c2 = static_cast<int>(s.get8());
      int len = static_cast<int>(s.get8());
      if (c1 != 2 || c2 != 2 || (len & 0x80)) {
        // not run-length encoded: this is a flat file after all (stb's goto main_decode_loop), whose
        // first texel these four bytes are; the rest of the image is read flat from texel 1 of row 0
        const uint8_t rgbe[4] = {static_cast<uint8_t>(c1), static_cast<uint8_t>(c2), static_cast<uint8_t>(len),
                                 static_cast<uint8_t>(s.get8())};
        hdr_convert(out, rgbe);
        flat = true;
        j0 = 0;
        i0 = 1;
        break;
      }
      len = (len << 8) | static_cast<int>(s.get8());
      if (len != width) return false;
      for (int k = 0; k < 4; ++k) {
        int i = 0, nleft;
        while ((nleft = width - i) > 0) {
          int count = static_cast<int>(s.get8());
          if (count > 128) {
            const uint8_t value = static_cast<uint8_t>(s.get8());
            count -= 128;
            if (count == 0 || count > nleft) return false;
            for (int z = 0; z < count; ++z) scanline[static_cast<size_t>(i++) * 4 + k] = value;
          } else {
            if (count == 0 || count > nleft) return false;
            for (int z = 0; z < count; ++z) scanline[static_cast<size_t>(i++) * 4 + k] = static_cast<uint8_t>(s.get8());
          }
        }
      }
      for (int i = 0; i < width; ++i) hdr_convert(out + (static_cast<size_t>(j) * width + i) * 3, &scanline[static_cast<size_t>(i) * 4]);
    }
  }
  if (flat) {
    for (int j = j0; j < height; ++j)
      for (int i = (j == j0 ? i0 : 0); i < width; ++i) {
        uint8_t rgbe[4] = {0, 0, 0, 0};
        s.getn(rgbe, 4);
        hdr_convert(out + (static_cast<size_t>(j) * width + i) * 3, rgbe);
      }
  }
  return true;
}

// ---- Photoshop PSD (:6126-6325, as stbi_loadf runs it: 8-bit output) ----
// RGB colour mode only; 8- or 16-bit channels (a 16-bit raw sample keeps its high byte; RLE data is read as bytes
// whatever the depth); channels past the file's are 0, alpha 255; a pixel with partial alpha loses the white matte.

// PackBits into every 4th byte: n < 128 copies n + 1 bytes, n > 128 repeats the next byte 257 - n times, 128 is a
// no-op; a run past the channel's end is corrupt (:6088-6124)
bool psd_rle_channel(StbFile &s, uint8_t *p, int count) {
  int done = 0;
  while (count - done > 0) {
    const int left = count - done;
    int n = static_cast<int>(s.get8());
    if (n == 128) continue;
    if (n < 128) {
      n += 1;
      if (n > left) return false;
      for (int i = 0; i < n; ++i, p += 4) *p = static_cast<uint8_t>(s.get8());
    } else {
      n = 257 - n;
      if (n > left) return false;
      const uint8_t v = static_cast<uint8_t>(s.get8());
      for (int i = 0; i < n; ++i, p += 4) *p = v;
    }
    done += n;
  }
  return true;
}

bool psd_load(StbFile &s, Pixels *o) {
  if (s.get32be() != 0x38425053u) return false;   // "8BPS"
  if (s.get16be() != 1) return false;             // version
  s.skip(6);
  const int channels = s.get16be();
  if (channels > 16) return false;
  const int h = static_cast<int>(s.get32be()), w = static_cast<int>(s.get32be());   // as stb's int conversions
  if (h > static_cast<int>(kMaxDim) || w > static_cast<int>(kMaxDim)) return false;
  const int depth = s.get16be();
  if (depth != 8 && depth != 16) return false;
  if (s.get16be() != 3) return false;             // colour mode: RGB
  for (int k = 0; k < 3; ++k) s.skip(static_cast<int>(s.get32be()));   // mode data, image resources, reserved
  const int compression = s.get16be();
  if (compression > 1) return false;
  if (!mad3_ok(4, w, h, 0)) return false;
  const int n = w * h;
  o->px.assign(static_cast<size_t>(n) * 4, 0);
  o->w = w;
  o->h = h;
  o->comp = 4;
  uint8_t *out = o->px.data();
  if (compression) s.skip(h * channels * 2);      // the per-row byte counts
  for (int ch = 0; ch < 4; ++ch) {
    uint8_t *p = out + ch;
    if (ch >= channels) {
      const uint8_t v = ch == 3 ? 255 : 0;
      for (int i = 0; i < n; ++i) p[4 * i] = v;
    } else if (compression) {
      if (!psd_rle_channel(s, p, n)) return false;
    } else if (depth == 16) {
      for (int i = 0; i < n; ++i) p[4 * i] = static_cast<uint8_t>(s.get16be() >> 8);
    } else {
      for (int i = 0; i < n; ++i) p[4 * i] = static_cast<uint8_t>(s.get8());
    }
  }
  if (channels >= 4) {   // un-premultiply against white: c / a + 255 (1 - 1 / a), in float, truncated to a byte
    for (int i = 0; i < n; ++i) {
      uint8_t *px = out + 4 * i;
      if (px[3] == 0 || px[3] == 255) continue;
      const float a = static_cast<float>(px[3]) / 255.0f;
      const float ra = 1.0f / a;
      const float inv_a = 255.0f * (1.0f - ra);
      for (int c = 0; c < 3; ++c) {
        const float v = static_cast<float>(px[c]) * ra + inv_a;
        // (the C conversion of an out-of-range float to unsigned char, as the x86-64 build of stb executes it: to a
        // 32-bit int, then its low byte; |v| < 2^17 here)
        px[c] = static_cast<uint8_t>(static_cast<uint32_t>(static_cast<int32_t>(v)));
      }
    }
  }
  return true;
}

// ---- Softimage PIC (:6346-6539) ----
// A 104-byte header (the 92 skipped bytes, width, height, ratio, fields, pad), a chain of at most 10 channel packets
// (8 bits each; mask 0x80 R, 0x40 G, 0x20 B, 0x10 A), then per row, per packet: raw, pure-RLE or mixed-RLE runs of the
// packet's channels.  Texels start at 255 in every channel.  (Where the data is corrupt and the picture has area, stb
// converts the NULL it gets back from its core loop and faults; here that is a failed load.)
struct PicPacket { uint8_t size, type, channel; };

bool pic_value(StbFile &s, int channel, uint8_t *dest) {   // stbi__readval: an early end fails the read
  for (int i = 0, mask = 0x80; i < 4; ++i, mask >>= 1) {
    if (channel & mask) {
      if (s.at_eof()) return false;
      dest[i] = static_cast<uint8_t>(s.get8());
    }
  }
  return true;
}

void pic_copy(int channel, uint8_t *dest, const uint8_t *src) {
  for (int i = 0, mask = 0x80; i < 4; ++i, mask >>= 1)
    if (channel & mask) dest[i] = src[i];
}

bool pic_load(StbFile &s, Pixels *o) {
  for (int i = 0; i < 92; ++i) s.get8();
  const int w = s.get16be(), h = s.get16be();
  if (s.at_eof()) return false;
  if (!mad3_ok(w, h, 4, 0)) return false;
  s.get32be();   // ratio
  s.get16be();   // fields
  s.get16be();   // pad
  o->px.assign(static_cast<size_t>(w) * h * 4, 0xff);
  o->w = w;
  o->h = h;
  o->comp = 4;
  PicPacket packets[10];
  int count = 0;
  uint32_t chained = 0;
  do {
    if (count == 10) return false;   // too many packets
    PicPacket &p = packets[count++];
    chained = s.get8();
    p.size = static_cast<uint8_t>(s.get8());
    p.type = static_cast<uint8_t>(s.get8());
    p.channel = static_cast<uint8_t>(s.get8());
    if (s.at_eof()) return false;
    if (p.size != 8) return false;
  } while (chained);
  for (int y = 0; y < h; ++y) {
    for (int k = 0; k < count; ++k) {
      const PicPacket &p = packets[k];
      uint8_t *dest = o->px.data() + static_cast<size_t>(y) * w * 4;
      if (p.type == 0) {            // uncompressed
        for (int x = 0; x < w; ++x, dest += 4)
          if (!pic_value(s, p.channel, dest)) return false;
      } else if (p.type == 1) {     // pure RLE: (count, value) pairs, a count past the row clamped to it
        int left = w;
        while (left > 0) {
          int n = static_cast<int>(s.get8());
          if (s.at_eof()) return false;
          if (n > left) n = left;
          uint8_t v[4];
          if (!pic_value(s, p.channel, v)) return false;
          for (int i = 0; i < n; ++i, dest += 4) pic_copy(p.channel, dest, v);
          left -= n;
        }
      } else if (p.type == 2) {     // mixed RLE: >= 128 a repeat (128: 16-bit count follows), else count + 1 raw
        int left = w;
        while (left > 0) {
          int n = static_cast<int>(s.get8());
          if (s.at_eof()) return false;
          if (n >= 128) {
            n = n == 128 ? s.get16be() : n - 127;
            if (n > left) return false;
            uint8_t v[4];
            if (!pic_value(s, p.channel, v)) return false;
            for (int i = 0; i < n; ++i, dest += 4) pic_copy(p.channel, dest, v);
          } else {
            n += 1;
            if (n > left) return false;
            for (int i = 0; i < n; ++i, dest += 4)
              if (!pic_value(s, p.channel, dest)) return false;
          }
          left -= n;
        }
      } else {
        return false;               // unknown packet type
      }
    }
  }
  return true;
}

// ---- GIF (:6597-6950, 7048-7075): the first image of the file ----
// The LZW raster (codes up to 12 bits, a clear code first), interlaced rows, global / local colour tables, the
// graphic-control extension's transparent index (transparent texels are not written), and the first frame's
// background: texels the image did not reach take the background entry of the global table when its index is not 0
// — copied in the table's stored order (blue, green, red), as stb does.
struct Gif {
  int w = 0, h = 0, flags = 0, bgindex = 0, transparent = -1, eflags = 0, lflags = 0;
  uint8_t pal[256][4] = {}, lpal[256][4] = {};
  struct Code { int16_t prefix; uint8_t first, suffix; };
  Code codes[8192] = {};
  const uint8_t *table = nullptr;
  int parse = 0, step = 0, start_x = 0, start_y = 0, max_x = 0, max_y = 0, cur_x = 0, cur_y = 0, line = 0;
  std::vector<uint8_t> out, history;
  std::vector<uint8_t> chain;   // a code's string, last texel first
};

void gif_table(StbFile &s, uint8_t pal[256][4], int n, int transp) {   // stored as blue, green, red, alpha
  for (int i = 0; i < n; ++i) {
    pal[i][2] = static_cast<uint8_t>(s.get8());
    pal[i][1] = static_cast<uint8_t>(s.get8());
    pal[i][0] = static_cast<uint8_t>(s.get8());
    pal[i][3] = transp == i ? 0 : 255;
  }
}

// the texels of one code, first to last (stbi__out_gif_code's recursion over the prefixes, unrolled): each one
// written unless transparent, then the cursor moves on (interlace passes 8, 8 from 4, 4 from 2, 2 from 1)
void gif_emit(Gif &g, int code) {
  g.chain.clear();
  for (int c = code; c >= 0; c = g.codes[c].prefix) g.chain.push_back(g.codes[c].suffix);
  for (size_t k = g.chain.size(); k-- > 0;) {
    if (g.cur_y >= g.max_y) continue;
    const int idx = g.cur_x + g.cur_y;
    uint8_t *p = &g.out[static_cast<size_t>(idx)];
    g.history[static_cast<size_t>(idx / 4)] = 1;
    const uint8_t *c = g.table + g.chain[k] * 4;
    if (c[3] > 128) {
      p[0] = c[2];
      p[1] = c[1];
      p[2] = c[0];
      p[3] = c[3];
    }
    g.cur_x += 4;
    if (g.cur_x >= g.max_x) {
      g.cur_x = g.start_x;
      g.cur_y += g.step;
      while (g.cur_y >= g.max_y && g.parse > 0) {
        g.step = (1 << g.parse) * g.line;
        g.cur_y = g.start_y + (g.step >> 1);
        --g.parse;
      }
    }
  }
}

bool gif_raster(StbFile &s, Gif &g) {
  const int lzw_cs = static_cast<int>(s.get8());
  if (lzw_cs > 12) return false;
  const int clear = 1 << lzw_cs;
  bool first = true;   // a stream must open with a clear code
  int codesize = lzw_cs + 1, codemask = (1 << codesize) - 1, bits = 0, valid_bits = 0;
  for (int c = 0; c < clear; ++c) g.codes[c] = {-1, static_cast<uint8_t>(c), static_cast<uint8_t>(c)};
  int avail = clear + 2, oldcode = -1, len = 0;
  for (;;) {
    if (valid_bits < codesize) {
      if (len == 0) {
        len = static_cast<int>(s.get8());   // the next data sub-block; an empty one ends the raster
        if (len == 0) return true;
      }
      --len;
      bits |= static_cast<int>(s.get8()) << valid_bits;
      valid_bits += 8;
      continue;
    }
    const int code = bits & codemask;
    bits >>= codesize;
    valid_bits -= codesize;
    if (code == clear) {
      codesize = lzw_cs + 1;
      codemask = (1 << codesize) - 1;
      avail = clear + 2;
      oldcode = -1;
      first = false;
    } else if (code == clear + 1) {   // end of information: skip the rest of the sub-blocks
      s.skip(len);
      while ((len = static_cast<int>(s.get8())) > 0) s.skip(len);
      return true;
    } else if (code <= avail) {
      if (first) return false;
      if (oldcode >= 0) {
        Gif::Code &p = g.codes[avail++];
        if (avail > 8192) return false;
        p.prefix = static_cast<int16_t>(oldcode);
        p.first = g.codes[oldcode].first;
        p.suffix = code == avail ? p.first : g.codes[code].first;
      } else if (code == avail) {
        return false;
      }
      gif_emit(g, code);
      if ((avail & codemask) == 0 && avail <= 0x0fff) {
        ++codesize;
        codemask = (1 << codesize) - 1;
      }
      oldcode = code;
    } else {
      return false;
    }
  }
}

bool gif_load(StbFile &s, Pixels *o) {
  std::unique_ptr<Gif> gp(new Gif());
  Gif &g = *gp;
  if (s.get8() != 'G' || s.get8() != 'I' || s.get8() != 'F' || s.get8() != '8') return false;
  const uint32_t version = s.get8();
  if (version != '7' && version != '9') return false;
  if (s.get8() != 'a') return false;
  g.w = s.get16le();
  g.h = s.get16le();
  g.flags = static_cast<int>(s.get8());
  g.bgindex = static_cast<int>(s.get8());
  s.get8();   // aspect ratio
  if (g.flags & 0x80) gif_table(s, g.pal, 2 << (g.flags & 7), -1);
  if (!mad3_ok(4, g.w, g.h, 0)) return false;
  const size_t n = static_cast<size_t>(g.w) * g.h;
  g.out.assign(4 * n, 0);
  g.history.assign(n, 0);
  for (;;) {
    const uint32_t tag = s.get8();
    if (tag == 0x2c) {   // image descriptor
      const int x = s.get16le(), y = s.get16le(), w = s.get16le(), h = s.get16le();
      if (x + w > g.w || y + h > g.h) return false;
      g.line = g.w * 4;
      g.start_x = x * 4;
      g.start_y = y * g.line;
      g.max_x = g.start_x + w * 4;
      g.max_y = g.start_y + h * g.line;
      g.cur_x = g.start_x;
      g.cur_y = w == 0 ? g.max_y : g.start_y;
      g.lflags = static_cast<int>(s.get8());
      if (g.lflags & 0x40) {
        g.step = 8 * g.line;
        g.parse = 3;
      } else {
        g.step = g.line;
        g.parse = 0;
      }
      if (g.lflags & 0x80) {
        gif_table(s, g.lpal, 2 << (g.lflags & 7), (g.eflags & 0x01) ? g.transparent : -1);
        g.table = &g.lpal[0][0];
      } else if (g.flags & 0x80) {
        g.table = &g.pal[0][0];
      } else {
        return false;   // no colour table
      }
      if (!gif_raster(s, g)) return false;
      if (g.bgindex > 0) {
        for (size_t i = 0; i < n; ++i) {
          if (g.history[i] == 0) {
            g.pal[g.bgindex][3] = 255;
            std::memcpy(&g.out[4 * i], g.pal[g.bgindex], 4);
          }
        }
      }
      o->px.swap(g.out);
      o->w = g.w;
      o->h = g.h;
      o->comp = 4;
      return true;
    }
    if (tag == 0x21) {   // extension
      int len;
      if (s.get8() == 0xf9) {   // graphic control
        len = static_cast<int>(s.get8());
        if (len != 4) {
          s.skip(len);
          continue;
        }
        g.eflags = static_cast<int>(s.get8());
        s.get16le();   // delay
        if (g.transparent >= 0) g.pal[g.transparent][3] = 255;
        if (g.eflags & 0x01) {
          g.transparent = static_cast<int>(s.get8());
          g.pal[g.transparent][3] = 0;
        } else {
          s.skip(1);
          g.transparent = -1;
        }
      }
      while ((len = static_cast<int>(s.get8())) != 0) s.skip(len);
      continue;
    }
    return false;   // the trailer before any image, or an unknown block
  }
}

bool read_file(const char *path, std::vector<uint8_t> *out) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out->insert(out->end(), buf, buf + n);
  std::fclose(f);
  return true;
}

// 8-bit texels -> float RGB: stbi__convert_format to 3 channels (grey replicated, alpha dropped), then
// stbi__ldr_to_hdr (whose own allocation check, x * y * 3 * sizeof(float), bounds the texel count)
float *to_float_rgb(const Pixels &p) {
  if (!mad4_ok(p.w, p.h, 3, static_cast<int>(sizeof(float)), 0)) return nullptr;
  const float *L = ldr_table();
  const size_t n = static_cast<size_t>(p.w) * static_cast<size_t>(p.h);
  float *out = static_cast<float *>(std::malloc(n * 3 * sizeof(float)));
  if (!out) return nullptr;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t *s = &p.px[i * p.comp];
    const bool grey = p.comp < 3;
    for (int k = 0; k < 3; ++k) out[i * 3 + k] = L[grey ? s[0] : s[k]];
  }
  return out;
}

// stbi__loadf_main / stbi__load_main over the file's bytes
int load(const std::vector<uint8_t> &bytes, float **rgb, int32_t *width, int32_t *height) {
  StbFile s(bytes);
  if (hdr_test(s)) {
    std::vector<float> f;
    int w = 0, h = 0;
    if (!hdr_load(s, &f, &w, &h) || w <= 0 || h <= 0) return RT_IMAGE_MISSING;
    *rgb = static_cast<float *>(std::malloc(f.size() * sizeof(float)));
    if (!*rgb) return RT_IMAGE_MISSING;
    std::memcpy(*rgb, f.data(), f.size() * sizeof(float));
    *width = w;
    *height = h;
    return RT_OK;
  }
  Pixels p;
  bool ok = false;
  if (png_test(s)) {
    ok = rt::png::decode(bytes.data(), bytes.size(), &p.px, &p.w, &p.h);
  } else if (bmp_test(s)) {
    ok = bmp_load(s, &p);
  } else if (gif_test(s)) {
    ok = gif_load(s, &p);
  } else if (psd_test(s)) {
    ok = psd_load(s, &p);
  } else if (pic_test(s)) {
    ok = pic_load(s, &p);
  } else if (jpeg_test(s)) {
    ok = rt::jpeg::decode(bytes.data(), bytes.size(), &p.px, &p.w, &p.h);
  } else if (pnm_test(s)) {
    ok = pnm_load(s, &p);
  } else if (tga_test(s)) {
    // (stb tests HDR again before TGA: that test already failed above and reads the same bytes)
    ok = tga_load(s, &p);
  }
  if (!ok || p.w <= 0 || p.h <= 0) return RT_IMAGE_MISSING;
  *rgb = to_float_rgb(p);
  if (!*rgb) return RT_IMAGE_MISSING;
  *width = p.w;
  *height = p.h;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_image_load(const char *path, float **rgb, int32_t *width, int32_t *height) {
  if (!path || !rgb || !width || !height) return RT_ERR_INVALID_ARG;
  *rgb = nullptr;
  *width = 0;
  *height = 0;
  std::vector<uint8_t> bytes;
  if (!read_file(path, &bytes)) return RT_IMAGE_MISSING;
  const int st = load(bytes, rgb, width, height);
  if (st != RT_OK) {
    std::free(*rgb);
    *rgb = nullptr;
    *width = 0;
    *height = 0;
  }
  return st;
}

void rt_image_free(float *rgb) { std::free(rgb); }

}  // extern "C"
