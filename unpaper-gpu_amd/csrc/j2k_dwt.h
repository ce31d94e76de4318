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

// ---------------------------------------------------------------------------
// The same transforms one output pair at a time, for a thread per pair: the
// lifting steps recomputed over a window of the line's whole-sample
// symmetric (periodic) extension, which equals the in-place sequential
// lifting above value for value (each lifted value of the extension is the
// value at its mirrored position; the float steps keep the operands and
// their order).  Line i of n samples: the Mallat layout (lows [0, sn),
// highs [sn, n); elements s apart) on the inverse's input and the forward's
// output, natural order (elements ds apart) on the other side.

J2K_HD inline int mirror_ext(int i, int n) {  // n >= 2
  const int P = 2 * (n - 1);
  i %= P;
  if (i < 0) i += P;
  return i >= n ? P - i : i;
}
// natural position i (0 <= i < n) of a Mallat line
J2K_HD inline int mallat_index(int i, int n, int cas) {
  const int sn = (n + 1 - cas) / 2;
  return ((i + cas) & 1) == 0 ? (i - cas) / 2 : sn + (i - (1 - cas)) / 2;
}

// Inverse: natural-order samples 2t and 2t + 1 (when < n) of a Mallat line.
template <class T, int CAS>
J2K_HD inline void idwt_pair(const T* src, int64_t s, int n, int t, T* o0, T* o1) {
  const int b = 2 * t;
  constexpr bool kInt = T(1) / T(2) == T(0);  // 5/3 (int32) or 9/7 (float)
  if (n == 1) {  // a single sample: a high one is halved (OpenJPEG dwt.c)
    const T x = src[0];
    if constexpr (kInt) *o0 = CAS ? x / 2 : x;
    else *o0 = CAS ? x * 0.5f : x;
    return;
  }
  auto ld = [&](int j) -> T { return src[(int64_t)mallat_index(mirror_ext(b + j, n), n, CAS) * s]; };
  // low positions: ((j + CAS) & 1) == 0
  if constexpr (kInt) {  // 5/3: window b-2 .. b+3
    T w[6];
#pragma unroll
    for (int j = 0; j < 6; j++) w[j] = ld(j - 2);
    T s1[6];
#pragma unroll
    for (int j = 1; j < 5; j++)
      s1[j] = ((j - 2 + CAS) & 1) == 0 ? w[j] - ((w[j - 1] + w[j + 1] + 2) >> 2) : w[j];
    T out[2];
#pragma unroll
    for (int j = 2; j < 4; j++)
      out[j - 2] = ((j - 2 + CAS) & 1) == 0 ? s1[j] : w[j] + ((s1[j - 1] + s1[j + 1]) >> 1);
    *o0 = out[0];
    if (b + 1 < n) *o1 = out[1];
  } else {  // 9/7 float: window b-4 .. b+5
    const float kA = -1.586134342059924f, kB = -0.052980118572961f;
    const float kG = 0.882911075530934f, kD = 0.443506852043971f;
    const float kK = 1.230174104914001f, kInvK = 13318.0f / 16384.0f;
    float a[10];
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const float x = ld(j - 4);
      a[j] = ((j - 4 + CAS) & 1) == 0 ? x * kK : x * kInvK;
    }
    float c[10];
#pragma unroll
    for (int j = 1; j < 9; j++)  // delta on the lows
      c[j] = ((j - 4 + CAS) & 1) == 0 ? a[j] - kD * (a[j - 1] + a[j + 1]) : a[j];
#pragma unroll
    for (int j = 2; j < 8; j++)  // gamma on the highs
      a[j] = ((j - 4 + CAS) & 1) != 0 ? c[j] - kG * (c[j - 1] + c[j + 1]) : c[j];
#pragma unroll
    for (int j = 3; j < 7; j++)  // beta on the lows
      c[j] = ((j - 4 + CAS) & 1) == 0 ? a[j] - kB * (a[j - 1] + a[j + 1]) : a[j];
#pragma unroll
    for (int j = 4; j < 6; j++)  // alpha on the highs
      a[j] = ((j - 4 + CAS) & 1) != 0 ? c[j] - kA * (c[j - 1] + c[j + 1]) : c[j];
    *o0 = (T)a[4];
    if (b + 1 < n) *o1 = (T)a[5];
  }
}

// Forward 5/3: natural-order samples 2t and 2t + 1 (when < n) lifted, for
// their Mallat positions.
template <int CAS>
J2K_HD inline void fdwt53_pair(const int32_t* src, int64_t ds, int n, int t, int32_t* o0,
                               int32_t* o1) {
  const int b = 2 * t;
  if (n == 1) {
    *o0 = CAS ? src[0] * 2 : src[0];
    return;
  }
  int32_t w[6];
#pragma unroll
  for (int j = 0; j < 6; j++) w[j] = src[(int64_t)mirror_ext(b + j - 2, n) * ds];
  int32_t h1[6];
#pragma unroll
  for (int j = 1; j < 5; j++)  // highs: predict
    h1[j] = ((j - 2 + CAS) & 1) != 0 ? w[j] - ((w[j - 1] + w[j + 1]) >> 1) : w[j];
  int32_t out[2];
#pragma unroll
  for (int j = 2; j < 4; j++)  // lows: update
    out[j - 2] = ((j - 2 + CAS) & 1) == 0 ? h1[j] + ((h1[j - 1] + h1[j + 1] + 2) >> 2) : h1[j];
  *o0 = out[0];
  if (b + 1 < n) *o1 = out[1];
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
