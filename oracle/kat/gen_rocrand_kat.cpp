// gen_rocrand_kat.cpp — known-answer vectors for the device RNG, taken from rocRAND itself.
//
// The reference draws from cuRAND XORWOW (curand_init(1234, pixel, 0), raytracing.cu:1604;
// curand_uniform at :1573-1578, utility.h:35-37, vec3.h:141-160).  cuRAND is not in this image;
// this build substitutes rocRAND's XORWOW (ROCm 7.2 rocrand_xorwow.h: same recurrence, Weyl step
// 362437, 2^67-long subsequences; different seed salting and uniform mapping).
// This program is run by oracle/Makefile (target `kat`) and writes tests/golden/rng_kat.json,
// which pins both the oracle's and the HIP kernel's independent XORWOW restatements.
#include <cstdio>
#include <rocrand/rocrand_xorwow.h>
#include <rocrand/rocrand_uniform.h>
#include <cstdio>
#include <cstring>

int main() {
  const unsigned long long seeds[] = {1234ull, 0ull, 0x123456789abcdefull};
  const unsigned long long subs[] = {0ull, 1ull, 2ull, 3ull, 63ull, 64ull, 1000ull, 36863ull,
                                     1000000ull, 2073599ull, 8294399ull, 16777215ull, 123456789ull};
  std::printf("{\n  \"generator\": \"rocrand_state_xorwow (ROCm 7.2 headers), rocrand_uniform\",\n");
  std::printf("  \"draws\": 8,\n  \"cases\": [\n");
  bool first = true;
  for (unsigned long long seed : seeds) {
    for (unsigned long long sub : subs) {
      if (seed != 1234ull && sub > 1000000ull) continue;
      rocrand_state_xorwow st;
      rocrand_init(seed, sub, 0, &st);
      std::printf("%s    {\"seed\": %llu, \"subsequence\": %llu, \"uniform_bits\": [", first ? "" : ",\n",
                  seed, sub);
      first = false;
      for (int i = 0; i < 8; ++i) {
        float u = rocrand_uniform(&st);
        unsigned int bits;
        std::memcpy(&bits, &u, 4);
        std::printf("%s%u", i ? ", " : "", bits);
      }
      std::printf("]}");
    }
  }
  std::printf("\n  ]\n}\n");
  return 0;
}
