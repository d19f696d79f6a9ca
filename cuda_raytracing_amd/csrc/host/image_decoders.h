// image_decoders.h — the compressed-format decoders behind rt_image_load (image_load.cpp).
// Each decodes a whole file held in memory into 8-bit RGB texels, rows top first, and returns false
// where the reference's stbi_loadf returns NULL (its texture then renders magenta).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rt {
namespace jpeg {
bool is_jpeg(const uint8_t *b, size_t n);   // stbi__jpeg_test: an SOI marker
bool decode(const uint8_t *b, size_t n, std::vector<uint8_t> *rgb, int *w, int *h);
}  // namespace jpeg
namespace png {
bool is_png(const uint8_t *b, size_t n);    // stbi__png_test: the 8-byte signature
bool decode(const uint8_t *b, size_t n, std::vector<uint8_t> *rgb, int *w, int *h);
}  // namespace png
}  // namespace rt
