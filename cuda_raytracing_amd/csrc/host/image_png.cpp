// image_png.cpp — PNG (and its DEFLATE stream) for image textures, with the reference loader's output.
//
// stbi_loadf (make_image_texture, raytracing.cu:332-341; stb_image v2.30, vendored by the reference)
// reads PNG files too.  This decoder is written for this project from the PNG specification (ISO/IEC
// 15948: chunks, the five filters, Adam7 interlacing, bit depths 1-16, every colour type, palettes) and
// RFC 1950/1951 (zlib framing, stored / fixed / dynamic Huffman blocks), and returns the texels
// stbi_loadf returns for 3 requested channels:
//   - grey below 8 bits scaled to 0..255 (x 0xff, 0x55, 0x11); palette indices looked up; grey replicated;
//     alpha (including tRNS) dropped; 16-bit samples reduced to their high byte;
//   - CRCs and the Adler-32 trailer are not checked; an unknown critical chunk, a bad IHDR, a zlib
//     stream that is malformed or runs past its end, or too few pixel bytes fail the load (the reference
//     then renders the texture magenta); Apple's CgBI variant is read with a headerless DEFLATE stream
//     and its channels left as stored.
#include <cstdint>
#include <cstring>
#include <vector>

#include "image_decoders.h"

namespace rt {
namespace png {
namespace {

// ---- DEFLATE (RFC 1951) ----
struct Huff {   // canonical code: counts per length, symbols in code order
  uint16_t count[16];
  uint16_t symbol[320];
  bool build(const uint8_t *len, int n) {
    std::memset(count, 0, sizeof count);
    for (int i = 0; i < n; ++i) count[len[i]]++;
    count[0] = 0;
    int code = 0;
    for (int l = 1; l < 16; ++l) {   // over-subscribed sets fail (incomplete ones are allowed)
      if (count[l] > (1 << l)) return false;
      code += count[l];
      if (count[l] && code - 1 >= (1 << l)) return false;
      code <<= 1;
    }
    uint16_t offs[16];
    offs[1] = 0;
    for (int l = 1; l < 15; ++l) offs[l + 1] = static_cast<uint16_t>(offs[l] + count[l]);
    for (int i = 0; i < n; ++i)
      if (len[i]) symbol[offs[len[i]]++] = static_cast<uint16_t>(i);
    return true;
  }
};

// The bit reader keeps stb_image's accounting (stbi__zbuf, stb_image.h:4177-4330): bits are taken LSB
// first from a 32-bit buffer; refills past the end of the data read zero bytes; a Huffman decode that
// finds fewer than 16 bits at the end adds 16 zero bits once (a second time fails), and an end-of-block
// code that consumed any of those added bits fails the stream as cut short.
struct Inflate {
  const uint8_t *p = nullptr, *end = nullptr;
  uint32_t code_buffer = 0;
  int num_bits = 0;
  bool hit_zeof_once = false;
  std::vector<uint8_t> out;

  bool zeof() const { return p >= end; }
  uint32_t zget8() { return zeof() ? 0u : *p++; }
  void fill_bits() {
    do {
      if (num_bits < 0 || num_bits >= 32 || code_buffer >= (1u << num_bits)) {   // stray bits: treat as the end
        p = end;
        return;
      }
      code_buffer |= zget8() << num_bits;
      num_bits += 8;
    } while (num_bits <= 24);
  }
  uint32_t receive(int n) {
    if (num_bits < n) fill_bits();
    const uint32_t k = code_buffer & ((1u << n) - 1);
    code_buffer >>= n;
    num_bits -= n;
    return k;
  }
  int decode(const Huff &h) {   // canonical code, its bits MSB-first within the LSB-first stream
    if (num_bits < 16) {
      if (zeof()) {
        if (hit_zeof_once) return -1;
        hit_zeof_once = true;
        num_bits += 16;   // implicit zero bits
      } else {
        fill_bits();
      }
    }
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; ++l) {
      code |= static_cast<int>((code_buffer >> (l - 1)) & 1u);
      const int c = h.count[l];
      if (code - c < first) {
        code_buffer >>= l;
        num_bits -= l;
        return h.symbol[index + (code - first)];
      }
      index += c;
      first = (first + c) << 1;
      code <<= 1;
    }
    return -1;
  }
  bool stored() {
    if (num_bits & 7) receive(num_bits & 7);   // to a byte boundary
    uint8_t hdr[4] = {0, 0, 0, 0};
    int k = 0;
    while (num_bits > 0) {   // the bytes already in the bit buffer first
      if (k >= 4) return false;
      hdr[k++] = static_cast<uint8_t>(code_buffer & 255);
      code_buffer >>= 8;
      num_bits -= 8;
    }
    if (num_bits < 0) return false;
    while (k < 4) hdr[k++] = static_cast<uint8_t>(zget8());
    const uint32_t len = hdr[0] | (hdr[1] << 8), nlen = hdr[2] | (hdr[3] << 8);
    if (nlen != (len ^ 0xffffu)) return false;
    if (static_cast<size_t>(end - p) < len) return false;
    out.insert(out.end(), p, p + len);
    p += len;
    return true;
  }
  bool codes(const Huff &lit, const Huff &dst) {
    static const uint16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99,
                                       115, 131, 163, 195, 227, 258};
    static const uint8_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static const uint16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
    static const uint8_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    for (;;) {
      const int s = decode(lit);
      if (s < 0) return false;
      if (s < 256) { out.push_back(static_cast<uint8_t>(s)); continue; }
      if (s == 256) return !(hit_zeof_once && num_bits < 16);   // consumed added bits: cut short
      if (s >= 286) return false;
      size_t len = lbase[s - 257];
      if (lext[s - 257]) len += receive(lext[s - 257]);
      const int d = decode(dst);
      if (d < 0 || d >= 30) return false;
      size_t dist = dbase[d];
      if (dext[d]) dist += receive(dext[d]);
      if (dist > out.size()) return false;
      for (size_t i = 0; i < len; ++i) out.push_back(out[out.size() - dist]);
    }
  }
  bool dynamic(Huff *lit, Huff *dst) {
    static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    const uint32_t hlit = receive(5) + 257, hdist = receive(5) + 1, hclen = receive(4) + 4;
    uint8_t cl[19] = {0};
    for (uint32_t i = 0; i < hclen; ++i) cl[order[i]] = static_cast<uint8_t>(receive(3));
    Huff clh;
    if (!clh.build(cl, 19)) return false;
    uint8_t lens[286 + 32 + 140];
    const uint32_t ntot = hlit + hdist;
    uint32_t n = 0;
    while (n < ntot) {
      const int c = decode(clh);
      if (c < 0 || c >= 19) return false;
      if (c < 16) { lens[n++] = static_cast<uint8_t>(c); continue; }
      uint32_t rep;
      uint8_t fill = 0;
      if (c == 16) {
        rep = receive(2) + 3;
        if (n == 0) return false;
        fill = lens[n - 1];
      } else if (c == 17) {
        rep = receive(3) + 3;
      } else {
        rep = receive(7) + 11;
      }
      if (ntot - n < rep) return false;
      std::memset(lens + n, fill, rep);
      n += rep;
    }
    return lit->build(lens, static_cast<int>(hlit)) && dst->build(lens + hlit, static_cast<int>(hdist));
  }
  bool run(bool zlib_header) {
    if (zlib_header) {   // stbi__parse_zlib_header
      const int cmf = static_cast<int>(zget8()), flg = static_cast<int>(zget8());
      if (zeof()) return false;
      if ((cmf * 256 + flg) % 31 != 0 || (flg & 32) || (cmf & 15) != 8) return false;
    }
    uint32_t final = 0;
    do {
      final = receive(1);
      const uint32_t type = receive(2);
      if (type == 0) {
        if (!stored()) return false;
      } else if (type == 1) {
        uint8_t l[288], d[32];
        for (int i = 0; i < 288; ++i) l[i] = i < 144 ? 8 : (i < 256 ? 9 : (i < 280 ? 7 : 8));
        for (int i = 0; i < 32; ++i) d[i] = 5;
        Huff lit, dst;
        if (!lit.build(l, 288) || !dst.build(d, 32) || !codes(lit, dst)) return false;
      } else if (type == 2) {
        Huff lit, dst;
        if (!dynamic(&lit, &dst) || !codes(lit, dst)) return false;
      } else {
        return false;
      }
    } while (!final);
    return true;
  }
};

uint32_t be32(const uint8_t *b) { return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | b[3]; }

inline int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// unfilter one (sub)image of x * y pixels of n channels at `depth` bits from raw, into samples (8-bit, or
// 16-bit values) of n channels per pixel; raw advances past it
bool unfilter(const uint8_t *&raw, size_t &raw_len, uint32_t x, uint32_t y, int n, int depth, int color,
              std::vector<uint16_t> *samples) {
  const uint64_t row_bytes = (static_cast<uint64_t>(n) * x * depth + 7) >> 3;
  const uint64_t need = (row_bytes + 1) * y;
  if (need > raw_len) return false;
  const int bpp = depth < 8 ? 1 : n * depth / 8;   // filter distance in bytes
  std::vector<uint8_t> prior(row_bytes, 0), cur(row_bytes, 0);
  static const uint8_t scale_table[9] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 0x01};
  const int scale = (color == 0 && depth < 8) ? scale_table[depth] : 1;
  samples->assign(static_cast<size_t>(x) * y * n, 0);
  for (uint32_t j = 0; j < y; ++j) {
    int f = *raw++;
    if (f > 4) return false;
    const uint8_t *r = raw;
    for (uint64_t k = 0; k < row_bytes; ++k) {
      const int a = k >= static_cast<uint64_t>(bpp) ? cur[k - bpp] : 0;
      const int b = prior[k], c = k >= static_cast<uint64_t>(bpp) ? prior[k - bpp] : 0;
      int pred = 0;
      switch (f) {
        case 1: pred = a; break;
        case 2: pred = b; break;
        case 3: pred = (a + b) >> 1; break;
        case 4: pred = paeth(a, b, c); break;
        default: break;
      }
      cur[k] = static_cast<uint8_t>(r[k] + pred);
    }
    raw += row_bytes;
    uint16_t *dst = samples->data() + static_cast<size_t>(j) * x * n;
    const uint64_t nsmp = static_cast<uint64_t>(x) * n;
    if (depth == 8) {
      for (uint64_t i = 0; i < nsmp; ++i) dst[i] = cur[i];
    } else if (depth == 16) {
      for (uint64_t i = 0; i < nsmp; ++i) dst[i] = static_cast<uint16_t>((cur[2 * i] << 8) | cur[2 * i + 1]);
    } else {
      const int per = 8 / depth, mask = (1 << depth) - 1;
      for (uint64_t i = 0; i < nsmp; ++i) {
        const int byte = cur[i / per], sh = 8 - depth * (static_cast<int>(i % per) + 1);
        dst[i] = static_cast<uint16_t>(scale * ((byte >> sh) & mask));
      }
    }
    std::swap(prior, cur);
  }
  raw_len -= need;
  return true;
}

}  // namespace

bool is_png(const uint8_t *b, size_t n) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  return n >= 8 && std::memcmp(b, sig, 8) == 0;
}

// 8-bit RGB texels, rows top first; false where stbi_loadf fails
bool decode(const uint8_t *b, size_t n, std::vector<uint8_t> *rgb, int *w, int *h) {
  if (!is_png(b, n)) return false;
  size_t pos = 8;
  bool first = true, iphone = false;
  uint32_t W = 0, H = 0;
  int depth = 0, color = 0, interlace = 0, img_n = 0;
  bool palette_img = false;
  uint8_t palette[256 * 3] = {0};
  uint32_t pal_len = 0;
  std::vector<uint8_t> idat;
  for (;;) {
    if (n - pos < 8) return false;   // out of data (stb reads zeros: a critical type 0 chunk, a failure)
    const uint32_t len = be32(b + pos), type = be32(b + pos + 4);
    pos += 8;
    const size_t avail = n - pos;
    auto chunk_type = [](const char *t) { return be32(reinterpret_cast<const uint8_t *>(t)); };
    if (type == chunk_type("CgBI")) {
      iphone = true;
    } else if (type == chunk_type("IHDR")) {
      if (!first || len != 13 || avail < 13) return false;
      first = false;
      W = be32(b + pos);
      H = be32(b + pos + 4);
      if (W > (1u << 24) || H > (1u << 24)) return false;
      depth = b[pos + 8];
      color = b[pos + 9];
      if (depth != 1 && depth != 2 && depth != 4 && depth != 8 && depth != 16) return false;
      if (color > 6 || (color == 3 && depth == 16)) return false;
      if (color == 3) palette_img = true;
      else if (color & 1) return false;
      if (b[pos + 10] || b[pos + 11] || b[pos + 12] > 1) return false;   // compression, filter, interlace
      interlace = b[pos + 12];
      if (!W || !H) return false;
      if (!palette_img) {
        img_n = (color & 2 ? 3 : 1) + (color & 4 ? 1 : 0);
        if ((1u << 30) / W / static_cast<uint32_t>(img_n) < H) return false;
      } else {
        img_n = 1;
        if ((1u << 30) / W / 4 < H) return false;
      }
    } else if (type == chunk_type("PLTE")) {
      if (first || len > 256 * 3 || len % 3 != 0 || avail < len) return false;
      pal_len = len / 3;
      std::memcpy(palette, b + pos, len);
    } else if (type == chunk_type("tRNS")) {
      if (first || !idat.empty()) return false;
      if (palette_img) {
        if (pal_len == 0 || len > pal_len) return false;
      } else {
        if (!(img_n & 1) || len != static_cast<uint32_t>(img_n) * 2) return false;
      }
      // transparency only fills the alpha channel, which three requested channels drop
    } else if (type == chunk_type("IDAT")) {
      if (first || (palette_img && !pal_len)) return false;
      if (len > (1u << 30) || avail < len) return false;
      idat.insert(idat.end(), b + pos, b + pos + len);
    } else if (type == chunk_type("IEND")) {
      if (first || idat.empty()) return false;
      Inflate z;
      z.p = idat.data();
      z.end = idat.data() + idat.size();
      if (!z.run(!iphone)) return false;
      const uint8_t *raw = z.out.data();
      size_t raw_len = z.out.size();
      std::vector<uint16_t> smp;
      std::vector<uint16_t> full;
      if (!interlace) {
        if (!unfilter(raw, raw_len, W, H, img_n, depth, color, &full)) return false;
      } else {   // Adam7: seven reduced images, scattered into the full one
        static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
        static const int xs[7] = {8, 8, 4, 4, 2, 2, 1}, ys[7] = {8, 8, 8, 4, 4, 2, 2};
        full.assign(static_cast<size_t>(W) * H * img_n, 0);
        for (int pz = 0; pz < 7; ++pz) {
          const uint32_t x = (W - xo[pz] + xs[pz] - 1) / xs[pz], y = (H - yo[pz] + ys[pz] - 1) / ys[pz];
          if (W <= static_cast<uint32_t>(xo[pz]) || H <= static_cast<uint32_t>(yo[pz]) || !x || !y) continue;
          if (!unfilter(raw, raw_len, x, y, img_n, depth, color, &smp)) return false;
          for (uint32_t j = 0; j < y; ++j)
            for (uint32_t i = 0; i < x; ++i)
              for (int c = 0; c < img_n; ++c)
                full[(static_cast<size_t>(j * ys[pz] + yo[pz]) * W + i * xs[pz] + xo[pz]) * img_n + c] =
                    smp[(static_cast<size_t>(j) * x + i) * img_n + c];
        }
      }
      rgb->assign(static_cast<size_t>(W) * H * 3, 0);
      const size_t np = static_cast<size_t>(W) * H;
      for (size_t i = 0; i < np; ++i) {
        uint8_t *o = rgb->data() + 3 * i;
        const uint16_t *s = full.data() + i * img_n;
        auto to8 = [&](uint16_t v) { return static_cast<uint8_t>(depth == 16 ? v >> 8 : v); };
        if (palette_img) {
          const uint32_t k = s[0];   // (an index past the palette: stb reads unset entries; zeros here)
          for (int c = 0; c < 3; ++c) o[c] = palette[3 * (k & 255) + c];
        } else if (img_n >= 3) {
          o[0] = to8(s[0]); o[1] = to8(s[1]); o[2] = to8(s[2]);
        } else {
          o[0] = o[1] = o[2] = to8(s[0]);
        }
      }
      *w = static_cast<int>(W);
      *h = static_cast<int>(H);
      return true;
    } else {
      if (first) return false;
      if ((type & (1u << 29)) == 0) return false;   // unknown critical chunk
    }
    if (avail < static_cast<size_t>(len) + 4) {
      if (type == chunk_type("IDAT")) return false;
      pos = n;   // ran out inside a skipped chunk: the next header reads as zeros
    } else {
      pos += static_cast<size_t>(len) + 4;   // data + CRC (not checked)
    }
  }
}

}  // namespace png
}  // namespace rt
