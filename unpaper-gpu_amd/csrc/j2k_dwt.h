// j2k_dwt.h — the JPEG 2000 wavelet lifting on one line of samples (host and
// device; ISO/IEC 15444-1 Annex F): the reversible 5/3 integer filter
// (F.3.8.1 / F.4.8.1, OpenJPEG dwt.c's rounding) and the irreversible 9/7
// (F.3.8.2), with whole-sample symmetric extension at both ends.  A line is
// held interleaved: sample i sits at absolute position i0 + i, low-pass
// coefficients at even absolute positions (cas = i0 & 1), elements `s` apart.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define J2K_HD __host__ __device__

namespace uph {
namespace j2k {

J2K_HD inline int mirror(int i, int n) { return i < 0 ? -i : i >= n ? 2 * (n - 1) - i : i; }

// Inverse 5/3: lows x -= (l + r + 2) >> 2, then highs x += (l + r) >> 1.
J2K_HD inline void idwt53_line(int32_t* x, int n, int cas, int64_t s) {
  if (n == 1) {
    if (cas) x[0] /= 2;  // a single high-pass sample (OpenJPEG dwt.c)
    return;
  }
  for (int i = cas; i < n; i += 2)
    x[i * s] -= (x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s] + 2) >> 2;
  for (int i = 1 - cas; i < n; i += 2)
    x[i * s] += (x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s]) >> 1;
}

// Forward 5/3 (the exact inverse of the above): highs, then lows.
J2K_HD inline void fdwt53_line(int32_t* x, int n, int cas, int64_t s) {
  if (n == 1) {
    if (cas) x[0] *= 2;
    return;
  }
  for (int i = 1 - cas; i < n; i += 2)
    x[i * s] -= (x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s]) >> 1;
  for (int i = cas; i < n; i += 2)
    x[i * s] += (x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s] + 2) >> 2;
}

// Inverse 9/7 (F.3.8.2): lows x K, highs x 1/K, then the four lifting steps
// undone (delta, gamma, beta, alpha), each as x - c * (l + r) in float.
// OpenJPEG (dwt.c opj_v8dwt_decode) scales the highs by 13318 / 8192, a
// fixed-point 2/K, against band steps without the band gain; 13318 / 16384
// against steps with the gain (as here) gives its values exactly (the factors
// of two cancel), where the true 1/K would differ by up to 0.005 a sample.
J2K_HD inline void idwt97_line(float* x, int n, int cas, int64_t s) {
  const float kA = -1.586134342059924f, kB = -0.052980118572961f;
  const float kG = 0.882911075530934f, kD = 0.443506852043971f;
  const float kK = 1.230174104914001f, kInvK = 13318.0f / 16384.0f;
  if (n == 1) {
    if (cas) x[0] *= 0.5f;
    return;
  }
  for (int i = cas; i < n; i += 2) x[i * s] = x[i * s] * kK;
  for (int i = 1 - cas; i < n; i += 2) x[i * s] = x[i * s] * kInvK;
  for (int i = cas; i < n; i += 2) {
    const float t = x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s];
    x[i * s] = x[i * s] - kD * t;
  }
  for (int i = 1 - cas; i < n; i += 2) {
    const float t = x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s];
    x[i * s] = x[i * s] - kG * t;
  }
  for (int i = cas; i < n; i += 2) {
    const float t = x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s];
    x[i * s] = x[i * s] - kB * t;
  }
  for (int i = 1 - cas; i < n; i += 2) {
    const float t = x[mirror(i - 1, n) * s] + x[mirror(i + 1, n) * s];
    x[i * s] = x[i * s] - kA * t;
  }
}

// A line of the Mallat layout (low part first, then high; elements s apart)
// into its interleaved natural order (elements ts apart), and back.
template <class T>
J2K_HD inline void interleave(const T* src, int64_t s, int n, int cas, T* dst, int64_t ts) {
  const int sn = (n + 1 - cas) / 2;  // low-pass samples
  for (int i = 0; i < n; i++) {
    const bool low = ((i + cas) & 1) == 0;
    const int k = low ? (i - cas) / 2 : sn + (i - (1 - cas)) / 2;
    dst[i * ts] = src[k * s];
  }
}
template <class T>
J2K_HD inline void deinterleave(const T* src, int64_t ts, int n, int cas, T* dst, int64_t s) {
  const int sn = (n + 1 - cas) / 2;
  for (int i = 0; i < n; i++) {
    const bool low = ((i + cas) & 1) == 0;
    const int k = low ? (i - cas) / 2 : sn + (i - (1 - cas)) / 2;
    dst[k * s] = src[i * ts];
  }
}

// The inverse component transforms and the DC level shift of one pixel
// (G.2: RCT for reversible, ICT for irreversible data; 8-bit output)
J2K_HD inline uint8_t clamp8(int32_t v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }
J2K_HD inline void rct_inverse(int32_t y0, int32_t y1, int32_t y2, uint8_t* r, uint8_t* g,
                               uint8_t* b) {
  const int32_t G = y0 - ((y1 + y2) >> 2);
  *g = clamp8(G + 128);
  *r = clamp8(y2 + G + 128);
  *b = clamp8(y1 + G + 128);
}
J2K_HD inline int32_t round_half_even(float f) {
  const float r = __builtin_rintf(f);
  return (int32_t)r;
}
J2K_HD inline void ict_inverse(float y, float u, float v, uint8_t* r, uint8_t* g, uint8_t* b) {
  const float R = y + (v * 1.402f);
  const float G = y - (u * 0.34413f) - (v * 0.71414f);
  const float B = y + (u * 1.772f);
  *r = clamp8(round_half_even(R) + 128);
  *g = clamp8(round_half_even(G) + 128);
  *b = clamp8(round_half_even(B) + 128);
}

}  // namespace j2k
}  // namespace uph
