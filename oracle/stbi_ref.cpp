// oracle/stbi_ref.cpp — test infrastructure only: the reference's own image loader (stb_image v2.30, the
// third-party header vendored at /root/reference/include/stb_image.h, used by make_image_texture,
// raytracing.cu:332-341) compiled where it lies into oracle/_ref/libstbi_ref.so (Makefile target `ref`).
// Compiled as C++ like the reference's main.cu, so pow(float, float) resolves as it does there.
// tests/test_image_load.py decodes the same files with it and with rt_image_load and compares the texels
// bit for bit.  Nothing in the product links or loads it.
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"

extern "C" float *rt_ref_stbi_loadf(const char *file, int *w, int *h) {
  int n = 0;
  return stbi_loadf(file, w, h, &n, 3);   // make_image_texture's call: 3 channels
}
extern "C" void rt_ref_stbi_free(void *p) { stbi_image_free(p); }
