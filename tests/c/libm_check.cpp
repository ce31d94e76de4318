// Checks the restated glibc sinf/cosf/powf(x, 2) of csrc/libm_glibc.h (the
// functions the batch path's rotation select evaluates on the device) against
// this host's glibc, bit for bit.
//
//   libm_check stride K   every K-th float (both signs): sinf/cosf for |x| < 120,
//                         powf(x, 2) for 2^-60 <= |x| < 2^61
//   libm_check full       every float of those ranges (8 threads, ~1 min)
//
// Prints one line per function with the number of inputs and mismatches; exit
// status 1 on any mismatch.  Test infrastructure (tests/test_libm_glibc.py).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

#include "libm_glibc.h"

static float (*volatile g_sinf)(float) = sinf;
static float (*volatile g_cosf)(float) = cosf;
static float (*volatile g_powf)(float, float) = powf;

static float as_float(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static bool same(float a, float b) { return memcmp(&a, &b, 4) == 0; }

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: libm_check stride K | full\n");
    return 2;
  }
  const bool full = !strcmp(argv[1], "full");
  const uint32_t stride = full ? 1 : (uint32_t)strtoul(argv[2], nullptr, 0);
  std::vector<uint32_t> table;
  uph::glibc::build_pow2_table(g_powf, table);
  for (uint32_t v : table)
    if (v == 0xffffffffu) {
      printf("powf(x, 2) differs from x*x by more than one ulp: not reproducible\n");
      return 1;
    }
  const int nt = full ? 8 : 1;
  const uint32_t trig_hi = 0x42F00000u;  // 120.0f
  const uint32_t pow_lo = (127u - 60) << 23, pow_hi = (127u + 61) << 23;
  std::atomic<long> n_trig{0}, bad_sin{0}, bad_cos{0}, n_pow{0}, bad_pow{0};
  auto work = [&](int t) {
    long nt_ = 0, bs = 0, bc = 0, np = 0, bp = 0;
    for (uint64_t u = (uint64_t)t * stride; u < trig_hi; u += (uint64_t)stride * nt)
      for (uint32_t sg = 0; sg < 2; sg++) {
        const float x = as_float((uint32_t)u | (sg << 31));
        nt_++;
        if (!same(uph::glibc::sinf(x), g_sinf(x))) {
          if (bs++ < 3) printf("sinf(%a): %a vs glibc %a\n", x, uph::glibc::sinf(x), g_sinf(x));
        }
        if (!same(uph::glibc::cosf(x), g_cosf(x))) {
          if (bc++ < 3) printf("cosf(%a): %a vs glibc %a\n", x, uph::glibc::cosf(x), g_cosf(x));
        }
      }
    for (uint64_t u = pow_lo + (uint64_t)t * stride; u < pow_hi; u += (uint64_t)stride * nt)
      for (uint32_t sg = 0; sg < 2; sg++) {
        const float x = as_float((uint32_t)u | (sg << 31));
        np++;
        const float a = uph::glibc::pow2(x, table.data(), (int)table.size());
        if (!same(a, g_powf(x, 2.0f))) {
          if (bp++ < 3) printf("powf(%a, 2): %a vs glibc %a\n", x, a, g_powf(x, 2.0f));
        }
      }
    n_trig += nt_;
    bad_sin += bs;
    bad_cos += bc;
    n_pow += np;
    bad_pow += bp;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  printf("pow2 table: %zu exception mantissas\n", table.size());
  printf("sinf: %ld inputs, %ld mismatches\n", n_trig.load(), bad_sin.load());
  printf("cosf: %ld inputs, %ld mismatches\n", n_trig.load(), bad_cos.load());
  printf("powf2: %ld inputs, %ld mismatches\n", n_pow.load(), bad_pow.load());
  return bad_sin || bad_cos || bad_pow ? 1 : 0;
}
