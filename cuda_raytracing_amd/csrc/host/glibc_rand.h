// glibc_rand.h — the reference's host RNG: glibc rand() (TYPE_3 additive feedback, degree 31,
// separation 3), seeded with 1 because the reference never calls srand (utility.h:26-41).
// Re-implemented so scene bytes do not depend on the process's libc state; tests pin it
// against the libc rand() of this image.
#pragma once
#include <cstdint>

namespace rt {

class GlibcRand {
 public:
  explicit GlibcRand(uint32_t seed = 1) { reseed(seed); }

  void reseed(uint32_t seed) {
    if (seed == 0) seed = 1;
    int32_t r[34];
    r[0] = static_cast<int32_t>(seed);
    for (int i = 1; i < 31; ++i) {
      // 16807 * r mod (2^31 - 1), Schrage-free with 64-bit arithmetic (glibc random_r.c semantics)
      int64_t v = (16807LL * r[i - 1]) % 2147483647LL;
      if (v < 0) v += 2147483647LL;
      r[i] = static_cast<int32_t>(v);
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 0; i < 34; ++i) ring_[i] = static_cast<uint32_t>(r[i]);
    pos_ = 34;
    for (int i = 34; i < 344; ++i) step();   // glibc discards the first 310 outputs
  }

  // one rand() value in [0, RAND_MAX]
  int32_t next() { return static_cast<int32_t>(step() >> 1); }

 private:
  uint32_t step() {
    uint32_t v = ring_[(pos_ - 31) & 63] + ring_[(pos_ - 3) & 63];
    ring_[pos_ & 63] = v;
    ++pos_;
    return v;
  }
  uint32_t ring_[64] = {};
  uint64_t pos_ = 0;
};

}  // namespace rt
