// common.h — shared device/host definitions of the HIP backend (gfx950).
//
// Data model: a batch of S sheets lives in HBM as two
// ping-pong plane arrays; sheet s, plane k starts at base[k] + s*stride, rows
// are `pitch` bytes apart (pitch is a multiple of 256 so every row starts on
// its own cache line).  Each sheet has a device-resident SheetCtl: which plane
// is current, its masks/rotations/borders, and status bits — written by the
// small per-sheet control kernels and read by the data-parallel kernels, so a
// whole pipeline runs without a host round trip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <mutex>
#include <set>
#include <utility>

#include "unpaper_hip.h"

#define UPH_HD __host__ __device__ __forceinline__

namespace uph {

// Dynamic LDS above 64 KiB needs the kernel's attribute raised, once per
// device and kernel (the whole CU's 160 KiB, so any size up to it launches).
inline void allow_dynamic_lds(const void* kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return;
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  if (done.insert({dev, kernel}).second)
    (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}


// Pixel layouts the kernels address directly.  MONO* are only handled by the
// conversion / copy / fill / geometry kernels (see kernels_blit.hip).
enum Fmt : int32_t {
  F_GRAY8 = UPHIP_FMT_GRAY8,
  F_Y400A = UPHIP_FMT_Y400A,
  F_RGB24 = UPHIP_FMT_RGB24,
  F_MONOWHITE = UPHIP_FMT_MONOWHITE,
  F_MONOBLACK = UPHIP_FMT_MONOBLACK,
};

UPH_HD int bytes_per_pixel(int fmt) {
  return fmt == F_GRAY8 ? 1 : fmt == F_Y400A ? 2 : fmt == F_RGB24 ? 3 : 0;
}
UPH_HD bool is_mono(int fmt) { return fmt == F_MONOWHITE || fmt == F_MONOBLACK; }
UPH_HD int64_t row_bytes(int32_t w, int fmt) {
  return is_mono(fmt) ? ((int64_t)w + 7) / 8 : (int64_t)w * bytes_per_pixel(fmt);
}
UPH_HD int64_t round_pitch(int64_t bytes) { return (bytes + 255) & ~(int64_t)255; }

// ---------------------------------------------------------------------------
// Geometry helpers (primitives.c semantics)
// ---------------------------------------------------------------------------
struct Rect {
  int32_t x0, y0, x1, y1;  // inclusive corners as stored (may be inverted)
};

UPH_HD Rect to_rect(UphipRectangle r) {
  return Rect{r.vertex[0].x, r.vertex[0].y, r.vertex[1].x, r.vertex[1].y};
}
UPH_HD UphipRectangle from_rect(Rect r) {
  UphipRectangle o;
  o.vertex[0].x = r.x0;
  o.vertex[0].y = r.y0;
  o.vertex[1].x = r.x1;
  o.vertex[1].y = r.y1;
  return o;
}
UPH_HD int32_t imin(int32_t a, int32_t b) { return a < b ? a : b; }
UPH_HD int32_t imax(int32_t a, int32_t b) { return a > b ? a : b; }
UPH_HD int32_t iabs(int32_t a) { return a < 0 ? -a : a; }
UPH_HD Rect normalize(Rect r) {  // normalize_rectangle, primitives.c:46-61
  return Rect{imin(r.x0, r.x1), imin(r.y0, r.y1), imax(r.x0, r.x1), imax(r.y0, r.y1)};
}
UPH_HD Rect clip(Rect r, int32_t W, int32_t H) {  // clip_rectangle, image.c:72-88
  Rect n = normalize(r);
  return Rect{imax(n.x0, 0), imax(n.y0, 0), imin(n.x1, W - 1), imin(n.y1, H - 1)};
}
// count_pixels (primitives.c:88-92): |dx|+1 times |dy|+1, never zero even for
// an inverted (fully outside) clip.
UPH_HD uint64_t count_pixels(Rect r) {
  return (uint64_t)(uint32_t)((iabs(r.x0 - r.x1) + 1) * (iabs(r.y0 - r.y1) + 1));
}
UPH_HD bool point_in(int32_t x, int32_t y, Rect in) {  // point_in_rectangle
  Rect a = normalize(in);
  return x >= a.x0 && x <= a.x1 && y >= a.y0 && y <= a.y1;
}
UPH_HD Rect rect_from_size(int32_t x, int32_t y, int32_t w, int32_t h) {
  return Rect{x, y, x + w - 1, y + h - 1};
}
UPH_HD bool rects_overlap(Rect a_in, Rect b_in) {  // primitives.c:117-123
  Rect a = normalize(a_in), b = normalize(b_in);
  return point_in(a.x0, a.y0, b) || point_in(a.x1, a.y1, b);
}

// ---------------------------------------------------------------------------
// Pixel model (pixel.c): reads outside the image are WHITE.
// ---------------------------------------------------------------------------
struct Px {
  uint8_t r, g, b;
};
UPH_HD uint8_t gray_of(Px p) { return (uint8_t)(((int)p.r + p.g + p.b) / 3); }
UPH_HD uint8_t light_of(Px p) {
  uint8_t m = p.r < p.g ? p.r : p.g;
  return m < p.b ? m : p.b;
}
UPH_HD uint8_t dark_of(Px p) {
  uint8_t m = p.r > p.g ? p.r : p.g;
  return m > p.b ? m : p.b;
}

// Load one pixel of a byte format (GRAY8 / Y400A / RGB24) from a row.
template <int FMT>
__device__ __forceinline__ Px load_px_row(const uint8_t* row, int32_t x) {
  if (FMT == F_GRAY8) {
    uint8_t v = row[x];
    return Px{v, v, v};
  } else if (FMT == F_Y400A) {
    uint8_t v = row[2 * x];
    return Px{v, v, v};
  } else {
    const uint8_t* q = row + 3 * x;
    return Px{q[0], q[1], q[2]};
  }
}

template <int FMT>
__device__ __forceinline__ void store_px_row(uint8_t* row, int32_t x, Px p) {
  if (FMT == F_GRAY8) {
    row[x] = gray_of(p);
  } else if (FMT == F_Y400A) {
    row[2 * x] = gray_of(p);
    row[2 * x + 1] = 0xFF;
  } else {
    uint8_t* q = row + 3 * x;
    q[0] = p.r;
    q[1] = p.g;
    q[2] = p.b;
  }
}

// Generic runtime-format read (any of the five formats), WHITE outside.
__device__ __forceinline__ Px load_px_any(const uint8_t* base, int64_t pitch, int fmt,
                                          int32_t W, int32_t H, int32_t x, int32_t y) {
  if (x < 0 || y < 0 || x >= W || y >= H) return Px{255, 255, 255};
  const uint8_t* row = base + (int64_t)y * pitch;
  switch (fmt) {
    case F_GRAY8: return load_px_row<F_GRAY8>(row, x);
    case F_Y400A: return load_px_row<F_Y400A>(row, x);
    case F_RGB24: return load_px_row<F_RGB24>(row, x);
    case F_MONOWHITE: return (row[x >> 3] & (128 >> (x & 7))) ? Px{0, 0, 0} : Px{255, 255, 255};
    default: return (row[x >> 3] & (128 >> (x & 7))) ? Px{255, 255, 255} : Px{0, 0, 0};
  }
}

// XCD-aware block order: workgroups are dispatched round-robin over the 8
// XCDs (each with its own L2), so consecutive block ids sit on different L2s.
// This bijection of the linear block id gives each XCD one contiguous run of
// (x, y, z) tiles, so data shared by neighbouring tiles is fetched into one L2.
__device__ __forceinline__ void xcd_block(int* bx, int* by, int* bz) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int nblk = gx * gy * gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int q = nblk >> 3, rr = nblk & 7, xcd = lin & 7;
  const int t = xcd * q + (xcd < rr ? xcd : rr) + (lin >> 3);
  *bz = t / (gx * gy);
  const int rem = t - *bz * gx * gy;
  *by = rem / gx;
  *bx = rem - *by * gx;
}

// xcd_block with its two divisions by host-computed reciprocals
// m = floor((2^32 - 1) / d) + 1 (exact for n * d < 2^32; m = 0 marks d = 1).
inline uint32_t div_magic(uint32_t d) { return d > 1 ? (uint32_t)(0xFFFFFFFFull / d + 1) : 0u; }
__device__ __forceinline__ int div_by_magic(int n, uint32_t m) {
  return m ? (int)__umulhi((uint32_t)n, m) : n;
}
__device__ __forceinline__ void xcd_block_m(uint32_t m_gxy, uint32_t m_gx, int* bx, int* by,
                                            int* bz) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int nblk = gx * gy * gridDim.z;
  const int lin = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int q = nblk >> 3, rr = nblk & 7, xcd = lin & 7;
  const int t = xcd * q + (xcd < rr ? xcd : rr) + (lin >> 3);
  *bz = div_by_magic(t, m_gxy);
  const int rem = t - *bz * gx * gy;
  *by = div_by_magic(rem, m_gx);
  *bx = rem - *by * gx;
}

// ---------------------------------------------------------------------------
// A batch of frames of identical geometry and format.  Frame s of plane k is
// base[k] + s*stride.  For single-image ops stride = 0 and count = 1.
// ---------------------------------------------------------------------------
struct Planes {
  uint8_t* base[2];
  int64_t pitch;
  int64_t stride;
  int32_t W, H;
  int32_t fmt;
  int32_t count;
};

// Per-sheet control block (device memory).  `cur` selects the current plane.
struct SheetCtl {
  int32_t cur;
  int32_t status;              // bit flags (STATUS_*)
  int32_t point_count;
  int32_t mask_count;
  UphipPoint points[UPHIP_MAX_POINTS];
  UphipRectangle masks[UPHIP_MAX_POINTS];
  UphipRectangle border_masks[UPHIP_MAX_PAGES];
  float rotation[UPHIP_MAX_PAGES];
  int32_t rot_index[UPHIP_MAX_PAGES][4];
  // generic per-op argument scratch written by control kernels
  int32_t op_active;           // non-zero: the pending op applies to this sheet
  int32_t op_i[8];
  float op_f[4];
  UphipRectangle op_rect[4];
};

enum : int32_t {
  STATUS_FLOOD_OVERFLOW = 1 << 0,
  STATUS_NOISE_OVERFLOW = 1 << 1,
  STATUS_EDGE_GUARD = 1 << 2,     // detect_edge left the image (reference would not stop)
  STATUS_SORT_OVERFLOW = 1 << 3,
};

__device__ __forceinline__ uint8_t* sheet_plane(const Planes& P, int s, int k) {
  return P.base[k] + (int64_t)s * P.stride;
}

// Timing diagnostics, compiled only into a tuning build (make lib
// DIAG=1 -> -DUPHIP_DIAG).  The product library has none of them: there the
// helpers are the constant 0 and every launch below is a single launch.
//   UPHIP_DIAG_SKIP   bit mask of sequential kernels not launched
//                     (1 black, 2 noise resolve, 4 gray decide, 8 blur resolve)
//   UPHIP_DIAG_DOUBLE bit mask of idempotent full-chip kernels launched twice,
//                     so that the throughput drop under the multi-stream load
//                     measures each kernel's marginal cost (1 rotation band,
//                     2 rotate, 4 mask move, 8 decode copy, 16 rotation points,
//                     32 gray cells, 64 blur counts, 128 rotation final + line
//                     walk; 256/512/1024/2048 rotate variants)
//   UPHIP_DIAG_NOISE  noise classify early exit (1, 2, 3)
// Any of these gives wrong pages by design.
#ifdef UPHIP_DIAG
inline int diag_env(const char* name) {
  const char* v = getenv(name);
  return v ? atoi(v) : 0;
}
inline int diag_skip() {
  static const int v = diag_env("UPHIP_DIAG_SKIP");
  return v;
}
inline int diag_double() {
  static const int v = diag_env("UPHIP_DIAG_DOUBLE");
  return v;
}
inline int diag_noise() {
  static const int v = diag_env("UPHIP_DIAG_NOISE");
  return v;
}
#define UPH_DIAG_BITS(d, m) ((d) & (m))
#define UPH_LAUNCH_DIAG(bit, ...)                              \
  do {                                                         \
    hipLaunchKernelGGL(__VA_ARGS__);                           \
    if (::uph::diag_double() & (bit)) hipLaunchKernelGGL(__VA_ARGS__); \
  } while (0)
#else
constexpr int diag_skip() { return 0; }
constexpr int diag_double() { return 0; }
constexpr int diag_noise() { return 0; }
#define UPH_DIAG_BITS(d, m) 0
#define UPH_LAUNCH_DIAG(bit, ...) hipLaunchKernelGGL(__VA_ARGS__)
#endif

}  // namespace uph
