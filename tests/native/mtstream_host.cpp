// Host build of the device MT stream (spl_rng.h) for a CPU unit test against the oracle's
// full-state MT19937.  Compiled by tests/test_device_rng_host.py; test code only.
#define SPL_HOST_UNIT_TEST 1
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <initializer_list>
#define __device__
#define __host__
#define __constant__ static constexpr
#define __forceinline__ inline
struct uint2 { uint32_t x, y; };
struct uint4 { uint32_t x, y, z, w; };
static inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return {a, b, c, d}; }
static inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
static inline int __clz(int x) { return x ? __builtin_clz((unsigned)x) : 32; }
#include "../../splendor-gym_amd/csrc/spl_rng.h"
extern "C" {
struct orc_mt_t { uint32_t mt[624]; int index; };
void orc_mt_seed(orc_mt_t*, uint64_t);
uint32_t orc_mt_next(orc_mt_t*);
}
int main(int argc, char** argv) {
  int nseeds = argc > 1 ? atoi(argv[1]) : 200;
  uint64_t x = 88172645463325252ull; int bad = 0;
  for (int s = 0; s < nseeds; ++s) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    uint64_t seed = (s % 3 == 0) ? (x & 0x7fffffffu) : (s % 3 == 1 ? (x & 0xfffffffffull) : x);
    if (s < 4) seed = (uint64_t[]){0, 1, 0xffffffffull, 0x100000000ull}[s];
    orc_mt_t ref; orc_mt_seed(&ref, seed);
    spl::MTStream ms; ms.init(seed);
    for (int j = 0; j < spl::MTStream::kMaxOut; ++j) {
      uint32_t a = ms.next(j), b = orc_mt_next(&ref);
      if (a != b) { printf("seed %llu out %d: %u != %u\n", (unsigned long long)seed, j, a, b); bad++; break; }
    }
    // the full-state continuation (LaneMT) picks up at output kMaxOut and runs through later twists
    static uint32_t region[624];
    spl::LaneMT lm{region, 0};
    lm.init(seed);
    lm.start_at(spl::MTStream::kMaxOut);
    for (int j = spl::MTStream::kMaxOut; j < 2600; ++j) {
      uint32_t a = lm.next(), b = orc_mt_next(&ref);
      if (a != b) { printf("LaneMT seed %llu out %d: %u != %u\n", (unsigned long long)seed, j, a, b); bad++; break; }
    }
    for (int start : {1, 3, 40, 227, 300}) {  // the test hook's lower limits: continue at any output
      orc_mt_t r2; orc_mt_seed(&r2, seed);
      for (int j = 0; j < start; ++j) orc_mt_next(&r2);
      spl::LaneMT l2{region, 0};
      l2.init(seed);
      l2.start_at(start);
      for (int j = start; j < 1300; ++j) {
        uint32_t a = l2.next(), b = orc_mt_next(&r2);
        if (a != b) { printf("LaneMT start %d seed %llu out %d\n", start, (unsigned long long)seed, j); bad++; break; }
      }
    }
  }
  printf(bad ? "FAIL %d\n" : "OK\n", bad);
  return bad != 0;
}
