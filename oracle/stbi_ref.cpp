// oracle/stbi_ref.cpp — test infrastructure only: the reference's own image loader (stb_image v2.30, the
// third-party header vendored at /root/reference/include/stb_image.h, used by make_image_texture,
// raytracing.cu:332-341) compiled where it lies into oracle/_ref/libstbi_ref*.so (Makefile target `ref`).
// Compiled as C++ like the reference's main.cu, so pow(float, float) resolves as it does there.
// tests/test_image_load.py decodes the same files with it and with rt_image_load and compares the texels
// bit for bit.  Nothing in the product links or loads it.
//
// Built three ways: as-is (libstbi_ref.so: the reference's loader), and twice with its uninitialised
// memory made explicit — heap blocks filled through stb's own STBI_MALLOC hook (RT_STBI_FILL), stack
// variables through clang's -ftrivial-auto-var-init, and the stack below the call scrubbed with the same
// byte first (for the variable a goto jumps past: stbi__hdr_load's main_decode_loop) — once with zeros
// (libstbi_ref_zero.so) and once with a pattern (libstbi_ref_pattern.so).  Where a corrupt file makes stb
// read memory it never wrote, the two differ; rt_image_load reads zeros there, so it is compared with the
// zero build.
#ifdef RT_STBI_FILL
#include <cstdlib>
#include <cstring>
static void *rt_stbi_fill_malloc(size_t n) {
  void *p = std::malloc(n);
  if (p) std::memset(p, RT_STBI_FILL, n);
  return p;
}
__attribute__((noinline)) static void rt_stbi_scrub_stack() {
  volatile unsigned char buf[1 << 18];
  for (size_t i = 0; i < sizeof buf; ++i) buf[i] = RT_STBI_FILL;
}
#define STBI_MALLOC(sz) rt_stbi_fill_malloc(sz)
#define STBI_REALLOC(p, newsz) std::realloc(p, newsz)
#define STBI_FREE(p) std::free(p)
#endif
#define STB_IMAGE_IMPLEMENTATION
#include "stb_image.h"

#include <csetjmp>
#include <csignal>

// A corrupt Softimage PIC file of non-zero area makes stb convert the NULL its core loop returned (stbi__pic_load,
// stb_image.h:6529-6536) and fault reading it.  The checker turns that fault into a reported crash
// (rt_ref_stbi_crashed) instead of ending the test process: a segmentation fault inside the call jumps back here.
static sigjmp_buf rt_stbi_jmp;
static volatile sig_atomic_t rt_stbi_in_call = 0, rt_stbi_faulted = 0;
static void rt_stbi_on_segv(int sig) {
  if (rt_stbi_in_call) siglongjmp(rt_stbi_jmp, 1);
  std::signal(sig, SIG_DFL);
  std::raise(sig);
}

extern "C" float *rt_ref_stbi_loadf(const char *file, int *w, int *h) {
  int n = 0;
#ifdef RT_STBI_FILL
  rt_stbi_scrub_stack();
#endif
  struct sigaction sa = {}, old_segv = {}, old_bus = {};
  sa.sa_handler = rt_stbi_on_segv;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &old_segv);
  sigaction(SIGBUS, &sa, &old_bus);
  float *r = nullptr;
  rt_stbi_faulted = 0;
  if (sigsetjmp(rt_stbi_jmp, 1) == 0) {
    rt_stbi_in_call = 1;
    r = stbi_loadf(file, w, h, &n, 3);   // make_image_texture's call: 3 channels
  } else {
    rt_stbi_faulted = 1;
    r = nullptr;
  }
  rt_stbi_in_call = 0;
  sigaction(SIGSEGV, &old_segv, nullptr);
  sigaction(SIGBUS, &old_bus, nullptr);
  return r;
}
extern "C" int rt_ref_stbi_crashed() { return rt_stbi_faulted; }
extern "C" void rt_ref_stbi_free(void *p) { stbi_image_free(p); }
