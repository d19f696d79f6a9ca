// image_load.cpp — image files for image textures (make_image_texture, raytracing.cu:332-341).
//
// The reference loads texels with stb_image's stbi_loadf(file, &w, &h, &n, 3): three float channels per
// texel, row 0 = the top row of the picture, 8-bit formats converted by pow(c / 255, 2.2) * 1 (stb_image's
// default LDR->float gamma and scale).  stb_image itself is a third-party header that is not part of this
// build; this file decodes the uncompressed formats it reads — binary PNM (P5 grey, P6 RGB; 8 and 16 bit),
// BMP (BI_RGB, 24 and 32 bit) and TGA (uncompressed true-colour and grey, 8/24/32 bit) — with the same
// output convention.  A file that exists in another format (JPEG, PNG, ...) is RT_ERR_UNSUPPORTED; a file
// that does not exist is the reference's failed load (no pixels: the texture renders magenta, :346-347).
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_host.h"

namespace {

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

struct Reader {
  std::vector<uint8_t> b;
  size_t p = 0;
  bool ok(size_t n) const { return p + n <= b.size(); }
  uint32_t u8() { return ok(1) ? b[p++] : 0u; }
  uint32_t le16() { uint32_t a = u8(); return a | (u8() << 8); }
  uint32_t le32() { uint32_t a = le16(); return a | (le16() << 16); }
};

bool read_file(const char *path, std::vector<uint8_t> *out) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out->insert(out->end(), buf, buf + n);
  std::fclose(f);
  return true;
}

// 8-bit texels (comp channels, rows top first) -> float RGB (grey replicated, alpha dropped:
// stbi__convert_format to 3 channels, then stbi__ldr_to_hdr)
float *to_float_rgb(const std::vector<uint8_t> &px, int w, int h, int comp) {
  const float *L = ldr_table();
  const size_t n = static_cast<size_t>(w) * static_cast<size_t>(h);
  float *out = static_cast<float *>(std::malloc(n * 3 * sizeof(float)));
  if (!out) return nullptr;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t *s = &px[i * comp];
    const bool grey = comp < 3;
    for (int k = 0; k < 3; ++k) out[i * 3 + k] = L[grey ? s[0] : s[k]];
  }
  return out;
}

bool dims_ok(uint64_t w, uint64_t h) { return w > 0 && h > 0 && w <= (1u << 24) && h <= (1u << 24) && w * h <= (1ull << 28); }

// binary PNM: P5 / P6 (stbi__pnm_info / stbi__pnm_load).  Samples are taken as stored, not rescaled by
// maxval; maxval > 255 means two bytes per sample, which stb_image reads into native (little-endian) 16-bit
// words and reduces with >> 8 (stbi__convert_16_to_8): the sample's second byte.
int load_pnm(Reader &r, float **rgb, int32_t *w, int32_t *h) {
  if (!r.ok(2) || r.b[0] != 'P' || (r.b[1] != '5' && r.b[1] != '6')) return RT_ERR_UNSUPPORTED;
  const int comp = r.b[1] == '6' ? 3 : 1;
  r.p = 2;
  uint64_t v[3];
  for (int k = 0; k < 3; ++k) {
    for (;;) {   // whitespace and comments
      while (r.ok(1) && std::strchr(" \t\n\v\f\r", r.b[r.p])) r.p++;
      if (r.ok(1) && r.b[r.p] == '#') { while (r.ok(1) && r.b[r.p] != '\n' && r.b[r.p] != '\r') r.p++; continue; }
      break;
    }
    if (!r.ok(1) || r.b[r.p] < '0' || r.b[r.p] > '9') return RT_ERR_UNSUPPORTED;
    v[k] = 0;
    while (r.ok(1) && r.b[r.p] >= '0' && r.b[r.p] <= '9' && v[k] < (1ull << 32)) v[k] = v[k] * 10 + (r.b[r.p++] - '0');
  }
  if (!r.ok(1)) return RT_ERR_UNSUPPORTED;
  r.p++;   // the single whitespace after maxval
  if (!dims_ok(v[0], v[1]) || v[2] > 65535) return RT_ERR_UNSUPPORTED;
  const size_t bps = v[2] > 255 ? 2 : 1, n = v[0] * v[1] * comp;
  if (!r.ok(n * bps)) return RT_ERR_UNSUPPORTED;
  std::vector<uint8_t> px(n);
  for (size_t i = 0; i < n; ++i) px[i] = r.b[r.p + i * bps + bps - 1];
  *w = static_cast<int32_t>(v[0]);
  *h = static_cast<int32_t>(v[1]);
  *rgb = to_float_rgb(px, *w, *h, comp);
  return *rgb ? RT_OK : RT_ERR_INVALID_ARG;
}

// BMP: BITMAPINFOHEADER or later, BI_RGB (or BI_BITFIELDS with the default 32-bit masks), 24 / 32 bit
int load_bmp(Reader &r, float **rgb, int32_t *w, int32_t *h) {
  if (!r.ok(54) || r.b[0] != 'B' || r.b[1] != 'M') return RT_ERR_UNSUPPORTED;
  r.p = 10;
  const uint32_t data = r.le32();
  const uint32_t hsz = r.le32();
  if (hsz < 40) return RT_ERR_UNSUPPORTED;
  const int32_t bw = static_cast<int32_t>(r.le32()), bh = static_cast<int32_t>(r.le32());
  const uint32_t planes = r.le16(), bpp = r.le16(), compr = r.le32();
  if (planes != 1 || (bpp != 24 && bpp != 32) || !(compr == 0 || (compr == 3 && bpp == 32))) return RT_ERR_UNSUPPORTED;
  if (compr == 3) {   // only the default masks (B G R A in byte order)
    r.p = 14 + 40;
    if (hsz == 40 && !r.ok(12)) return RT_ERR_UNSUPPORTED;
    const uint32_t mr = r.le32(), mg = r.le32(), mb = r.le32();
    if (mr != 0x00ff0000u || mg != 0x0000ff00u || mb != 0x000000ffu) return RT_ERR_UNSUPPORTED;
  }
  const bool flip = bh > 0;   // bottom-up rows (stb returns the top row first)
  const uint64_t W = static_cast<uint64_t>(bw < 0 ? -static_cast<int64_t>(bw) : bw);
  const uint64_t H = static_cast<uint64_t>(bh < 0 ? -static_cast<int64_t>(bh) : bh);
  if (bw <= 0 || !dims_ok(W, H)) return RT_ERR_UNSUPPORTED;
  const size_t bypp = bpp / 8, stride = (W * bypp + 3) & ~static_cast<size_t>(3);
  if (data + stride * (H - 1) + W * bypp > r.b.size()) return RT_ERR_UNSUPPORTED;
  std::vector<uint8_t> px(W * H * 3);
  for (uint64_t y = 0; y < H; ++y) {
    const uint8_t *row = &r.b[data + stride * (flip ? H - 1 - y : y)];
    for (uint64_t x = 0; x < W; ++x) {
      const uint8_t *s = row + x * bypp;
      uint8_t *d = &px[(y * W + x) * 3];
      d[0] = s[2]; d[1] = s[1]; d[2] = s[0];   // BGR(A) -> RGB
    }
  }
  *w = static_cast<int32_t>(W);
  *h = static_cast<int32_t>(H);
  *rgb = to_float_rgb(px, *w, *h, 3);
  return *rgb ? RT_OK : RT_ERR_INVALID_ARG;
}

// TGA: uncompressed true-colour (type 2: 24 / 32 bit) and grey (type 3: 8 bit), no colour map
int load_tga(Reader &r, float **rgb, int32_t *w, int32_t *h) {
  if (!r.ok(18)) return RT_ERR_UNSUPPORTED;
  const uint32_t idlen = r.b[0], cmap = r.b[1], type = r.b[2];
  r.p = 12;
  const uint32_t W = r.le16(), H = r.le16(), bpp = r.u8(), desc = r.u8();
  if (cmap != 0 || !((type == 2 && (bpp == 24 || bpp == 32)) || (type == 3 && bpp == 8)) || !dims_ok(W, H))
    return RT_ERR_UNSUPPORTED;
  const size_t bypp = bpp / 8, off = 18 + idlen;
  if (off + static_cast<size_t>(W) * H * bypp > r.b.size()) return RT_ERR_UNSUPPORTED;
  const bool top_first = (desc & 0x20) != 0, right_to_left = (desc & 0x10) != 0;
  if (right_to_left) return RT_ERR_UNSUPPORTED;
  const int comp = type == 3 ? 1 : 3;
  std::vector<uint8_t> px(static_cast<size_t>(W) * H * comp);
  for (uint32_t y = 0; y < H; ++y) {
    const uint8_t *row = &r.b[off + static_cast<size_t>(top_first ? y : H - 1 - y) * W * bypp];
    for (uint32_t x = 0; x < W; ++x) {
      const uint8_t *s = row + x * bypp;
      uint8_t *d = &px[(static_cast<size_t>(y) * W + x) * comp];
      if (comp == 1) d[0] = s[0];
      else { d[0] = s[2]; d[1] = s[1]; d[2] = s[0]; }
    }
  }
  *w = static_cast<int32_t>(W);
  *h = static_cast<int32_t>(H);
  *rgb = to_float_rgb(px, *w, *h, comp);
  return *rgb ? RT_OK : RT_ERR_INVALID_ARG;
}

}  // namespace

extern "C" {

int rt_image_load(const char *path, float **rgb, int32_t *width, int32_t *height) {
  if (!path || !rgb || !width || !height) return RT_ERR_INVALID_ARG;
  *rgb = nullptr;
  *width = 0;
  *height = 0;
  Reader r;
  if (!read_file(path, &r.b)) return RT_IMAGE_MISSING;
  int st = load_pnm(r, rgb, width, height);
  if (st == RT_ERR_UNSUPPORTED) { r.p = 0; st = load_bmp(r, rgb, width, height); }
  if (st == RT_ERR_UNSUPPORTED) {
    // TGA has no magic number: only when the name says so
    const size_t n = std::strlen(path);
    if (n >= 4 && (std::strcmp(path + n - 4, ".tga") == 0 || std::strcmp(path + n - 4, ".TGA") == 0)) {
      r.p = 0;
      st = load_tga(r, rgb, width, height);
    }
  }
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
