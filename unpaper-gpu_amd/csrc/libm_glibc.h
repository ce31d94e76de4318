// glibc's single-precision sinf, cosf and powf(x, 2), evaluated identically on
// the host and the device.
//
// The reference computes the deskew rotation's sin/cos with the host libm
// (deskew.c:260-261) and the edge deviation with powf(d, 2) (deskew.c:226; the
// reference's meson default build is -O0, so powf is really called).  The
// batch path decides rotations on the device (k_rot_select), so for more than
// two deskew edges -- where the combinations are too many for a host table --
// it needs these functions bit-identical to glibc.
//
// Third-party algorithm restated: glibc >= 2.28 sysdeps/ieee754/flt-32
// (s_sinf.c, s_cosf.c, sincosf.h, s_sincosf_data.c; the image's glibc is
// 2.35).  |x| < pi/4: a double polynomial in x^2; |x| < 120: one
// multiply-subtract range reduction by pi/2 and the polynomial of the
// quadrant.  On x86-64 glibc selects the FMA build of these files (ifunc,
// sysdeps/x86_64/fpu/multiarch/s_sinf-fma.c), whose compiler contracts every
// a*b + c of the polynomials: the fused form below.  Checked against the
// host's glibc for EVERY float with |x| < 120 (tests/c/libm_check.cpp, the
// exhaustive mode: 0 mismatches for sinf and cosf); the non-FMA build agrees
// with it for |x| < 17, far beyond any deskew angle.  |x| >= 120 (glibc's
// large-argument reduction) is not reproduced: the deskew angle is at most the
// scan range, a few degrees.
//
// powf(x, 2): glibc's powf is not correctly rounded.  For normal results it
// differs from the correctly rounded x*x by exactly +-1 ulp on a fixed set of
// mantissas (6,061 of 2^23 with the image's glibc), the same set in every
// binade 2^-60 .. 2^7 (checked exhaustively).  The host finds that set once
// with its own powf (glibc_pow2_table) and the device corrects x*x by it.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define UPH_LIBM_FN __host__ __device__ inline
#else
#define UPH_LIBM_FN inline
#endif

namespace uph {
namespace glibc {

// s_sincosf_data.c __sincosf_table[0]; entry [1] (quadrants 2 and 3) only
// negates c0..c4, which negates the cosine polynomial exactly (every rounding
// is sign-symmetric), so it is applied to the result below.
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;  // 2/pi * 2^24: quadrant in bits 24..31
constexpr double kHpi = 0x1.921FB54442D18p0;
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                 kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7,
                 kS3 = -0x1.994eb3774cf24p-13;

UPH_LIBM_FN double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

UPH_LIBM_FN uint32_t abstop12(float x) {
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  return (u >> 20) & 0x7ff;
}

// sincosf.h sinf_poly: n even -> sine polynomial of x, odd -> cosine (of
// table entry [neg])
UPH_LIBM_FN float poly(double x, double x2, int n, bool neg) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = fma_(x2, kS3, kS2);
    const double x7 = x3 * x2;
    const double s = fma_(x3, kS1, x);
    return (float)fma_(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = fma_(x2, kC4, kC3);
  const double c1 = fma_(x2, kC1, kC0);
  const double x6 = x4 * x2;
  const double c = fma_(x4, kC2, c1);
  const float r = (float)fma_(x6, c2, c);
  return neg ? -r : r;
}

// sincosf.h reduce_fast (the integer-rounding variant): x mod pi/2 and quadrant
UPH_LIBM_FN double reduce_fast(double x, int* np) {
  const double r = x * kHpiInv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fma_(-(double)n, kHpi, x);
}

constexpr float kPio4 = 0x1.921FB6p-1f;

UPH_LIBM_FN float sinf(float y) {
  double x = y;
  if (abstop12(y) < abstop12(kPio4)) {
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return poly(x, x * x, 0, false);
  }
  int n;
  x = reduce_fast(x, &n);
  const double s = ((n + 1) & 2) ? -1.0 : 1.0;  // sign[n & 3] = {1, -1, -1, 1}
  return poly(x * s, x * x, n, (n & 2) != 0);
}

UPH_LIBM_FN float cosf(float y) {
  double x = y;
  if (abstop12(y) < abstop12(kPio4)) {
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return poly(x, x * x, 1, false);
  }
  int n;
  x = reduce_fast(x, &n);
  const double s = ((n + 2) & 2) ? -1.0 : 1.0;  // sign[(n + 1) & 3]
  return poly(x * s, x * x, n ^ 1, ((n + 1) & 2) != 0);
}

// powf(x, 2) from the correctly rounded x*x and the sorted exception table:
// entry = mantissa (23 bits) | 1 << 31 when glibc's result is one ulp above
// (else one below).  Results below the normal range (|x| < 2^-63) are x*x.
UPH_LIBM_FN float pow2(float x, const uint32_t* table, int n) {
  const float r = x * x;
  uint32_t u;
  __builtin_memcpy(&u, &x, 4);
  const uint32_t e = (u >> 23) & 0xff;
  if (e < 127 - 60 || e > 127 + 60) return r;  // squares outside 2^-120 .. 2^122
  const uint32_t m = u & 0x7fffff;
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((table[mid] & 0x7fffff) < m)
      lo = mid + 1;
    else
      hi = mid;
  }
  if (lo >= n || (table[lo] & 0x7fffff) != m) return r;
  uint32_t ur;
  __builtin_memcpy(&ur, &r, 4);
  ur += (table[lo] >> 31) ? 1u : 0xffffffffu;
  float out;
  __builtin_memcpy(&out, &ur, 4);
  return out;
}

// Host only: the exception table of powf(x, 2) over the binade [1, 2), found
// with the given powf (the process's glibc).  8.4 M evaluations, ~0.15 s.
template <class Vec>
inline void build_pow2_table(float (*powf_fn)(float, float), Vec& out) {
  out.clear();
  for (uint32_t m = 0; m < (1u << 23); m++) {
    const uint32_t v = 0x3f800000u | m;
    float x, a;
    __builtin_memcpy(&x, &v, 4);
    const float b = x * x;
    a = powf_fn(x, 2.0f);
    uint32_t ua, ub;
    __builtin_memcpy(&ua, &a, 4);
    __builtin_memcpy(&ub, &b, 4);
    if (ua == ub + 1)
      out.push_back(m | 0x80000000u);
    else if (ua + 1 == ub)
      out.push_back(m);
    else if (ua != ub)
      out.push_back(0xffffffffu);  // not a +-1 ulp difference: flagged for the caller
  }
}

}  // namespace glibc

// Host: glibc's table for this process, built once (thread-safe).  Returns
// null if this libm's powf(x, 2) differs from x*x by more than one ulp
// somewhere in [1, 2) (then the device cannot reproduce it).
const uint32_t* glibc_pow2_table(int* n);

}  // namespace uph
