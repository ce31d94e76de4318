// kernels_black.hip — blackfilter (filters.c:49-127) with the reference's
// recursive flood fill (fill.c:16-107) replayed exactly on the GPU.
//
// Bars: darkness of every bar of the (only) scanned stripe per direction comes
// from one column-sum (row-sum) pass of max(r,g,b).  Fills only lighten, so a
// bar that is not dark enough on the original image never triggers later;
// candidates are re-measured on the current image once a fill has painted.
//
// Flood fill: the reference recursion (paint, four fill_lines, then for each
// line position its two perpendicular neighbours, depth first) is order-
// dependent (lines stop on painted pixels, and paint up to intensity-1
// non-matching pixels), so it is replayed in order by one wave per sheet,
// with an explicit stack of frames.  The replay never reads the image: the
// only question the fill asks of a pixel is "gray <= mask_max" (fill.c:29,
// :85) and the only change it makes is painting white, so it runs on bit
// planes M (the pixel matched before the fill) and P (painted): a pixel
// matches now iff M and not P (for mask_max < 255; white still matches
// otherwise).  Both are kept twice, row-major and column-major (one u64 per
// 64 pixels of a row / of a column), so that a lane reads 64 positions of a
// line in either direction with two words, and a round trip of one wave
// reads 16 windows (1024 positions) of each of a frame's four lines, or 8
// windows of each neighbour side: a line's stop, or its first matching
// neighbour, is a few 64-bit operations per lane.  The image is painted from
// P afterwards.
#include <climits>

#include "filters.h"

namespace uph {

bool black_geometry(int32_t W, int32_t H, const UphipBlackfilterParameters& p, uint8_t mask_max,
                    BlackGeom* g, BlackBar* bars, int max_bars) {
  g->W = W;
  g->H = H;
  g->abs_threshold = p.abs_threshold;
  g->mask_max = mask_max;
  g->intensity = (uint64_t)(int64_t)p.intensity;
  g->nbars = 0;
  g->nbars_h = 0;
  g->diag = 0;
  g->hregion = Rect{0, 0, -1, -1};
  g->vregion = Rect{0, 0, -1, -1};
  int64_t cap = (int64_t)W * H;
  if (cap > (1 << 20)) cap = 1 << 20;
  g->stack_capacity = (int32_t)(cap < 1024 ? 1024 : cap);
  const Rect img{0, 0, W - 1, H - 1};
  for (int dir = 0; dir < 2; dir++) {
    const bool on = dir == 0 ? p.scan_direction.horizontal : p.scan_direction.vertical;
    if (!on) continue;
    // blackfilter_cpu, filters.c:111-127
    const int32_t sx = dir == 0 ? p.scan_step.horizontal : 0;
    const int32_t sy = dir == 0 ? 0 : p.scan_step.vertical;
    const int32_t w = dir == 0 ? p.scan_size.width : (int32_t)p.scan_depth.horizontal;
    const int32_t h = dir == 0 ? (int32_t)p.scan_depth.vertical : p.scan_size.height;
    const int32_t shx = dir == 0 ? 0 : (int32_t)p.scan_depth.horizontal;
    const int32_t shy = dir == 0 ? (int32_t)p.scan_depth.vertical : 0;
    if (sx + sy <= 0) return false;  // the reference would not terminate
    // blackfilter_scan, filters.c:49-104
    Rect a = rect_from_size(0, 0, w, h);
    int stripes = 0;
    while (point_in(a.x0, a.y0, img)) {
      if (!point_in(a.x1, a.y1, img)) {
        const int32_t dx = img.x1 - a.x1, dy = img.y1 - a.y1;
        a = Rect{a.x0 + dx, a.y0 + dy, a.x1 + dx, a.y1 + dy};
      }
      if (stripes++ > 0) return false;  // unreachable for positive steps; keep one stripe
      const Rect region = dir == 0 ? clip(Rect{0, a.y0, W - 1, a.y1}, W, H)
                                   : clip(Rect{a.x0, 0, a.x1, H - 1}, W, H);
      if (dir == 0) g->hregion = region; else g->vregion = region;
      do {
        if (g->nbars >= max_bars) return false;
        BlackBar& b = bars[g->nbars++];
        b.r = a;
        b.dir = dir;
        b.excluded = 0;
        for (size_t n = 0; n < p.exclusions_count && n < UPHIP_MAX_MASKS; n++)
          if (rects_overlap(a, to_rect(p.exclusions[n]))) b.excluded = 1;
        a = Rect{a.x0 + sx, a.y0 + sy, a.x1 + sx, a.y1 + sy};
      } while (point_in(a.x0, a.y0, img));
      a = Rect{a.x0 + shx, a.y0 + shy, a.x1 + shx, a.y1 + shy};
    }
    if (dir == 0) g->nbars_h = g->nbars;
  }
  return true;
}

// ---------------------------------------------------------------------------
// Per-sheet scratch: [hsum: W | vsum: H] u32, the head (u32 "some bar is a
// candidate" flag, then the candidate bits of the bars from byte 8), the
// planes RM, RP (H rows of wpr words: x = 64w + bit, word w of row y at
// y * wpr + w) and CM, CP (W columns of hpc words: y = 64w + bit, word w of
// column x at w * W + x, so that neighbouring columns' words are adjacent),
// the DFS stack frames.
UPH_HD int32_t black_wpr(const BlackGeom& g) { return (g.W + 63) >> 6; }
UPH_HD int32_t black_hpc(const BlackGeom& g) { return (g.H + 63) >> 6; }
UPH_HD size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
UPH_HD size_t black_head_off(const BlackGeom& g) { return align256(((size_t)g.W + g.H) * 4); }
UPH_HD size_t black_rows_bytes(const BlackGeom& g) { return align256((size_t)g.H * black_wpr(g) * 8); }
UPH_HD size_t black_cols_bytes(const BlackGeom& g) { return align256((size_t)g.W * black_hpc(g) * 8); }
UPH_HD size_t black_rm_off(const BlackGeom& g) {
  return black_head_off(g) + align256(8 + (((size_t)g.nbars + 63) / 64) * 8);
}
UPH_HD size_t black_rp_off(const BlackGeom& g) { return black_rm_off(g) + black_rows_bytes(g); }
UPH_HD size_t black_cm_off(const BlackGeom& g) { return black_rp_off(g) + black_rows_bytes(g); }
UPH_HD size_t black_cp_off(const BlackGeom& g) { return black_cm_off(g) + black_cols_bytes(g); }
UPH_HD size_t black_stack_off(const BlackGeom& g) { return black_cp_off(g) + black_cols_bytes(g); }
size_t black_scratch_bytes(const BlackGeom& g) {
  return align256(black_stack_off(g) + (size_t)g.stack_capacity * 32);
}

// darkness of a bar on the original image (darkness_rect, blit.c:131-146)
// from the stripe's column / row sums, and the scan's test (filters.c:76-78)
__device__ __forceinline__ bool bar_candidate(const BlackGeom& g, const BlackBar& bb,
                                              const uint32_t* hsum, const uint32_t* vsum) {
  const Rect c = clip(bb.r, g.W, g.H);
  uint64_t sum = 0;
  if (c.x0 <= c.x1 && c.y0 <= c.y1) {
    if (bb.dir == 0)
      for (int32_t x = c.x0; x <= c.x1; x++) sum += hsum[x];
    else
      for (int32_t y = c.y0; y <= c.y1; y++) sum += vsum[y];
  }
  const uint8_t dark = (uint8_t)(0xFFull - sum / count_pixels(c));
  return dark >= g.abs_threshold && !bb.excluded;
}

// The candidate bits of every bar, and whether a sheet has any: only those
// sheets get planes, a replay and a paint pass.
constexpr int kCandThreads = 256;
__global__ void __launch_bounds__(kCandThreads) k_black_cand(BlackGeom g, const BlackBar* bars,
                                                             uint8_t* scratch, int64_t sstride,
                                                             const int32_t* active) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  uint8_t* scr = scratch + s * sstride;
  const uint32_t* hsum = (const uint32_t*)scr;
  uint8_t* head = scr + black_head_off(g);
  uint64_t* cand = (uint64_t*)(head + 8);
  bool any = false;
  for (int32_t b0 = 0; b0 < g.nbars; b0 += kCandThreads) {
    const int32_t bi = b0 + (int32_t)threadIdx.x;
    const bool c = bi < g.nbars && bar_candidate(g, bars[bi], hsum, hsum + g.W);
    const unsigned long long m = __ballot(c);
    if ((threadIdx.x & 63) == 0 && bi < g.nbars) cand[bi >> 6] = m;
    any |= c;
  }
  any = __syncthreads_or(any);
  if (threadIdx.x == 0) *(int32_t*)head = any;
}

__device__ __forceinline__ bool sheet_has_candidate(const BlackGeom& g, const uint8_t* scr) {
  return *(const int32_t*)(scr + black_head_off(g)) != 0;
}

// The planes of the candidate sheets, a block per 256x64 pixels: thread t
// makes row word t & 3 of row t >> 2 (M from the image, P clear; a row's
// four words from 256 contiguous bytes), then the column word of column t
// from the 64 row words in LDS.  Both planes are written in whole lines.
// RM_READY: the decode wrote RM (GRAY8 page = sheet, nothing between): the
// row words are read from it instead of from the image.
template <int FMT, bool RM_READY>
__global__ void __launch_bounds__(256) k_black_planes(PlaneRef img, BlackGeom g, uint8_t* scratch,
                                                      int64_t sstride, const int32_t* active) {
  const int s = blockIdx.z;
  if (active && !active[s]) return;
  uint8_t* scr = scratch + s * sstride;
  if (!sheet_has_candidate(g, scr)) return;
  __shared__ uint64_t rw[64][4];
  const int32_t wpr = black_wpr(g);
  const int t = threadIdx.x, r = t >> 2, q = t & 3;
  const int32_t xw = 4 * blockIdx.x + q, y = 64 * blockIdx.y + r, x0 = 64 * xw;
  uint64_t m = 0;
  if (RM_READY) {
    if (y < g.H && xw < wpr) {
      const int64_t i = (int64_t)y * wpr + xw;
      m = ((const uint64_t*)(scr + black_rm_off(g)))[i];
      ((uint64_t*)(scr + black_rp_off(g)))[i] = 0;
    }
  } else if (y < g.H && xw < wpr) {
    const uint8_t* row = plane_ptr(img, s) + (int64_t)y * img.P.pitch;
    if (FMT == F_GRAY8 && x0 + 64 <= g.W && ((uintptr_t)(row + x0) & 15) == 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint4 v = *(const uint4*)(row + x0 + 16 * k);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 16; c++)
          m |= (uint64_t)(((w4[c >> 2] >> (8 * (c & 3))) & 0xFFu) <= g.mask_max) << (16 * k + c);
      }
    } else {
      for (int c = 0; c < 64 && x0 + c < g.W; c++)
        m |= (uint64_t)(gray_of(load_px_row<FMT>(row, x0 + c)) <= g.mask_max) << c;
    }
    const int64_t i = (int64_t)y * wpr + xw;
    ((uint64_t*)(scr + black_rm_off(g)))[i] = m;
    ((uint64_t*)(scr + black_rp_off(g)))[i] = 0;
  }
  rw[r][q] = m;
  __syncthreads();
  // column x: bit k = row 64 blockIdx.y + k's bit x & 63 (a wave reads one
  // word of each row: LDS broadcasts)
  const int32_t x = 256 * blockIdx.x + t;
  const int qc = t >> 6, c = t & 63;
  uint64_t col = 0;
#pragma unroll 16
  for (int k = 0; k < 64; k++) col |= ((rw[k][qc] >> c) & 1ull) << k;
  if (x < g.W) {
    const int64_t i = (int64_t)blockIdx.y * g.W + x;
    ((uint64_t*)(scr + black_cm_off(g)))[i] = col;
    ((uint64_t*)(scr + black_cp_off(g)))[i] = 0;
  }
}

// The image from RP: painted pixels become white; the noisefilter's dark
// bit-plane (GRAY8, one u32 per 32 pixels of a row) loses them too.  One
// thread per row word.
template <int FMT>
__global__ void __launch_bounds__(256) k_black_paint(PlaneRef img, BlackGeom g, uint8_t* scratch,
                                                     int64_t sstride, const int32_t* active,
                                                     uint32_t* nbits, int64_t nbits_stride,
                                                     uint32_t* bbits, int64_t bb_stride) {
  const int s = blockIdx.z;
  if (active && !active[s]) return;
  uint8_t* scr = scratch + s * sstride;
  if (!sheet_has_candidate(g, scr)) return;
  const int32_t wpr = black_wpr(g);
  const int32_t xw = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (xw >= wpr || y >= g.H) return;
  const uint64_t p = ((const uint64_t*)(scr + black_rp_off(g)))[(int64_t)y * wpr + xw];
  if (!p) return;
  uint8_t* row = plane_ptr(img, s) + (int64_t)y * img.P.pitch;
  const int32_t x0 = 64 * xw;
  if (FMT == F_GRAY8 && x0 + 64 <= g.W && ((uintptr_t)(row + x0) & 15) == 0) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t b16 = (uint32_t)(p >> (16 * q)) & 0xFFFFu;
      if (!b16) continue;
      uint4* a = (uint4*)(row + x0 + 16 * q);
      const uint4 v = *a;
      uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int c = 0; c < 16; c++)
        if ((b16 >> c) & 1) w4[c >> 2] |= 0xFFu << (8 * (c & 3));
      *a = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  } else {
    for (uint64_t r = p; r; r &= r - 1)
      store_px_row<FMT>(row, x0 + __ffsll((long long)r) - 1, Px{255, 255, 255});
  }
  if (FMT == F_GRAY8 && nbits) {
    const int32_t nwr = (g.W + 31) >> 5;
    uint32_t* nb = nbits + s * nbits_stride + (int64_t)y * nwr + 2 * xw;
    nb[0] &= ~(uint32_t)p;
    if (2 * xw + 1 < nwr) nb[1] &= ~(uint32_t)(p >> 32);
  }
  if (FMT == F_GRAY8 && bbits) {  // the blurfilter's plane (pixel <= white < 255)
    const int32_t nwr = (g.W + 31) >> 5;
    uint32_t* bb = bbits + s * bb_stride + (int64_t)y * nwr + 2 * xw;
    bb[0] &= ~(uint32_t)p;
    if (2 * xw + 1 < nwr) bb[1] &= ~(uint32_t)(p >> 32);
  }
}

// ---------------------------------------------------------------------------
// The replay: one wave per sheet.  Control values are uniform (scalar).
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// Values the whole wave holds alike but loaded from memory (frames, bars)
// count as per-lane to the compiler: made scalar, the control built on them
// stays on the scalar unit instead of exec-masked vector code.
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)(uint32_t)uni((int32_t)(v >> 32)) << 32) | (uint32_t)uni((int32_t)v);
}
__device__ __forceinline__ Rect uni_rect(Rect r) { return Rect{uni(r.x0), uni(r.y0), uni(r.x1), uni(r.y1)}; }
__device__ __forceinline__ int ctz64(uint64_t v) { return __ffsll((long long)v) - 1; }
__device__ __forceinline__ int hib64(uint64_t v) { return 63 - __clzll((long long)v); }
template <class T>
__device__ __forceinline__ T pick4(const T (&a)[4], int d) {
  return d == 0 ? a[0] : d == 1 ? a[1] : d == 2 ? a[2] : a[3];
}
// lanes [lo, lo + n)
__device__ __forceinline__ uint64_t lane_range(int lo, int n) {
  return (n >= 64 ? ~0ull : ((1ull << n) - 1)) << lo;
}

constexpr int kStackLds = 1024;  // the lowest frames of the DFS stack live in LDS
constexpr size_t kStackLdsBytes = (size_t)kStackLds * 32;  // 32 KiB: deeper frames go to HBM

struct Frame {
  int32_t x, y;
  int32_t dist[4];
  int32_t cursor;  // next neighbour check, over the four lines' checks in order
  int32_t pad;
};

__device__ __forceinline__ int4* stack_lds() {
  extern __shared__ int4 black_stack[];
  return black_stack;
}
__device__ __forceinline__ void frame_put(Frame* hbm, int32_t i, const Frame& f) {
  const int4 a = make_int4(f.x, f.y, f.dist[0], f.dist[1]);
  const int4 b = make_int4(f.dist[2], f.dist[3], f.cursor, 0);
  if (i < kStackLds) {
    stack_lds()[2 * i] = a;
    stack_lds()[2 * i + 1] = b;
  } else {
    hbm[i] = f;
  }
}
__device__ __forceinline__ Frame frame_pop(const Frame* hbm, int32_t i) {
  Frame f;
  if (i >= kStackLds) {
    f = hbm[i];
  } else {
    const int4 a = stack_lds()[2 * i], b = stack_lds()[2 * i + 1];
    f.x = a.x;
    f.y = a.y;
    f.dist[0] = a.z;
    f.dist[1] = a.w;
    f.dist[2] = b.x;
    f.dist[3] = b.y;
    f.cursor = b.z;
  }
  f.x = uni(f.x);
  f.y = uni(f.y);
#pragma unroll
  for (int d = 0; d < 4; d++) f.dist[d] = uni(f.dist[d]);
  f.cursor = uni(f.cursor);
  f.pad = 0;
  return f;
}

struct BlackStats {
  uint32_t frames, fill_trips, check_trips, bar_trips, remeasures;
  uint64_t t_fill, t_check, t_bar, t_remeasure, t_wait0, t_paint, t_wait1;
};
#ifdef UPHIP_DIAG
#define BSTAT(...) __VA_ARGS__
#else
#define BSTAT(...)
#endif

// left, up, right, down (fill.c:88-95)
__device__ __forceinline__ constexpr int dir_dx(int d) { return d == 0 ? -1 : d == 2 ? 1 : 0; }
__device__ __forceinline__ constexpr int dir_dy(int d) { return d == 1 ? -1 : d == 3 ? 1 : 0; }

struct Sheet {
  const uint64_t* RM;
  uint64_t* RP;
  const uint64_t* CM;
  uint64_t* CP;
  int32_t wpr, hpc, W, H;
  int32_t I;  // intensity, clamped to 2^30 (lines are shorter)
  bool live;  // mask_max < 255: a painted (white) pixel stops matching
  // P is read and written by this wave alone.  Paints are no-return atomics
  // (they execute at the memory side: issued and forgotten, and in order
  // with the wave's later loads of the same word); loads bypass L1.
  __device__ __forceinline__ static uint64_t pload(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ static void por(uint64_t* p, uint64_t bits) {
    __hip_atomic_fetch_or(p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// A lane's window: 64 positions of a line, loaded as two words of M and P of
// the line's plane (row lines: the row planes, column lines: the column
// planes), issued by `issue` and combined by `bits` so that the loads of a
// round trip are in flight together.  Line `ln` (row y or column x) holds
// coordinates 0 .. len-1; the window holds coordinates s .. s+63 (bit i is
// s + i; zero outside).
struct Win {
  uint64_t m0, m1, p0, p1;
  int32_t sh;
  bool ok0, ok1;
  __device__ __forceinline__ void issue(const Sheet& S, bool col, int32_t ln, int32_t s) {
    // plain values first: a per-lane choice between two members of S would
    // otherwise become a per-lane address into a private copy of S
    const int32_t W = S.W, H = S.H, hpc = S.hpc, wpr = S.wpr;
    const uint64_t *CM = S.CM, *RM = S.RM, *CP = S.CP, *RP = S.RP;
    const int32_t nl = col ? W : H, nw = col ? hpc : wpr;
    const uint64_t* M = col ? CM : RM;
    const uint64_t* P = col ? CP : RP;
    const int32_t w0 = s >> 6;  // floor
    const bool lok = ln >= 0 && ln < nl;
    ok0 = lok && w0 >= 0 && w0 < nw;
    ok1 = lok && w0 + 1 >= 0 && w0 + 1 < nw;
    sh = s & 63;
    // row planes: word w of row ln at ln * wpr + w; column planes: word w of
    // column ln at w * W + ln
    const int32_t l = lok ? ln : 0, wa = ok0 ? w0 : 0, wb = ok1 ? w0 + 1 : 0;
    const int64_t i0 = col ? (int64_t)wa * W + l : (int64_t)l * wpr + wa;
    const int64_t i1 = col ? (int64_t)wb * W + l : (int64_t)l * wpr + wb;
    m0 = M[i0];
    m1 = M[i1];
    p0 = Sheet::pload(P + i0);
    p1 = Sheet::pload(P + i1);
  }
  __device__ __forceinline__ uint64_t bits(const Sheet& S) const {
    const uint64_t e0 = ok0 ? (S.live ? m0 & ~p0 : m0) : 0;
    const uint64_t e1 = ok1 ? (S.live ? m1 & ~p1 : m1) : 0;
    return sh ? (e0 >> sh) | (e1 << (64 - sh)) : e0;
  }
};

// Positions j = base .. base+63 along a line from (cx, cy) in direction d,
// at perpendicular offset `off` (a neighbour side): the lane's window issue,
// and its bits in position order.
__device__ __forceinline__ void ray_issue(const Sheet& S, Win& w, int d, int32_t cx, int32_t cy,
                                          int32_t off, int32_t base) {
  const bool col = d & 1;
  const int32_t ln = col ? cx + off : cy + off;  // the row / column the positions lie on
  const int32_t c0 = col ? cy : cx;
  const bool dec = d < 2;  // left, up: coordinates fall with the position
  w.issue(S, col, ln, dec ? c0 - base - 63 : c0 + base);
}
__device__ __forceinline__ uint64_t ray_bits(const Sheet& S, const Win& w, int d) {
  const uint64_t v = w.bits(S);
  return d < 2 ? __builtin_bitreverse64(v) : v;
}

// A window of 64 positions base .. base+63 of a fill line (E: bit k set iff
// position base+k matches), with L the last matching position before it
// (1 - I when none: the counter starts at 1, fill.c:20): the line's stop in
// this window, or INT_MAX.  The counter reaches 0 at the first non-matching
// position j with j - L >= I; before the window's first match f that is
// max(base, L + I) if it lies below base + f, after it the first position
// with no match in the I positions ending at it (the smear of E over I - 1
// positions, exact inside the window since a run reaching back past f holds f).
__device__ __forceinline__ int32_t window_stop(uint64_t E, int32_t base, int32_t L, int32_t I) {
  const int f = E ? ctz64(E) : 64;
  const int32_t j = imax(base, L + I);
  if (j < base + f) return j;
  if (I >= 64 || f >= 63) return INT_MAX;
  uint64_t cur = E;
  int len = 1;
  while (2 * len <= I) {
    cur |= cur << len;
    len *= 2;
  }
  if (len < I) cur |= cur << (I - len);
  const uint64_t cand = ~cur & (~0ull << (f + 1));
  return cand ? base + ctz64(cand) : INT_MAX;
}

// Paint the cross at (px, py): the start and positions 1 .. dist[d] of its
// four lines.  In the own planes (row py: [px - dist0, px + dist2], column
// px: [py - dist1, py + dist3]) a word per lane; in the crossing planes a bit
// per lane (column words of the row's pixels, row words of the column's).
template <bool LONG>
__device__ __forceinline__ void paint_cross(const Sheet& S, int32_t px, int32_t py,
                                            const int32_t (&dist)[4]) {
  const int lane = lane_id();
  const int32_t xa = px - dist[0], xb = px + dist[2], ya = py - dist[1], yb = py + dist[3];
  const int32_t nrw = (xb >> 6) - (xa >> 6) + 1, nown = nrw + (yb >> 6) - (ya >> 6) + 1;
  const int32_t nrx = dist[0] + dist[2];
  uint64_t *RP = S.RP, *CP = S.CP;
  const int32_t wpr = S.wpr, W = S.W;
  const int32_t ncross = nrx + dist[1] + dist[3];
  if (!LONG) {  // the one lane loop over everything (round 5)
    for (int32_t i0 = 0; i0 < imax(nown, ncross); i0 += 64) {
      const int32_t i = i0 + lane;
      if (i < nown) {
        const bool row = i < nrw;
        const int32_t lo = row ? xa : ya, hi = row ? xb : yb;
        const int32_t w = (lo >> 6) + (row ? i : i - nrw);
        const int a = imax(lo - 64 * w, 0), b = imin(hi - 64 * w, 63);
        Sheet::por(row ? RP + (int64_t)py * wpr + w : CP + (int64_t)w * W + px,
                   (~0ull >> (63 - b)) & (~0ull << a));
      }
      if (i < nrx) {
        const int32_t x = i < dist[0] ? px - 1 - i : px + 1 + (i - dist[0]);
        Sheet::por(CP + (int64_t)(py >> 6) * W + x, 1ull << (py & 63));
      } else if (i < ncross) {
        const int32_t j = i - nrx;
        const int32_t y = j < dist[1] ? py - 1 - j : py + 1 + (j - dist[1]);
        Sheet::por(RP + (int64_t)y * wpr + (px >> 6), 1ull << (px & 63));
      }
    }
    return;
  }
  if (nown <= 64 && ncross <= 64) {
    // a short cross (the common frame): one lane step does everything
    const int32_t i = lane;
    if (i < nown) {
      const bool row = i < nrw;
      const int32_t lo = row ? xa : ya, hi = row ? xb : yb;
      const int32_t w = (lo >> 6) + (row ? i : i - nrw);
      const int a = imax(lo - 64 * w, 0), b = imin(hi - 64 * w, 63);
      Sheet::por(row ? RP + (int64_t)py * wpr + w : CP + (int64_t)w * W + px,
                 (~0ull >> (63 - b)) & (~0ull << a));
    }
    if (i < nrx) {
      const int32_t x = i < dist[0] ? px - 1 - i : px + 1 + (i - dist[0]);
      Sheet::por(CP + (int64_t)(py >> 6) * W + x, 1ull << (py & 63));
    } else if (i < ncross) {
      const int32_t j = i - nrx;
      const int32_t y = j < dist[1] ? py - 1 - j : py + 1 + (j - dist[1]);
      Sheet::por(RP + (int64_t)y * wpr + (px >> 6), 1ull << (px & 63));
    }
    return;
  }
  // own planes: a word per lane
  for (int32_t i = lane; i < nown; i += 64) {
    const bool row = i < nrw;
    const int32_t lo = row ? xa : ya, hi = row ? xb : yb;
    const int32_t w = (lo >> 6) + (row ? i : i - nrw);
    const int a = imax(lo - 64 * w, 0), b = imin(hi - 64 * w, 63);
    Sheet::por(row ? RP + (int64_t)py * wpr + w : CP + (int64_t)w * W + px,
               (~0ull >> (63 - b)) & (~0ull << a));
  }
  // crossing planes, a bit per lane: the row's pixels in the column planes
  const uint64_t bit_y = 1ull << (py & 63);
  uint64_t* const crow = CP + (int64_t)(py >> 6) * W;
  for (int32_t i = lane; i < nrx; i += 64)
    Sheet::por(crow + (i < dist[0] ? px - 1 - i : px + 1 + (i - dist[0])), bit_y);
  // ... and the column's pixels in the row planes: straight pointer walks up
  // and down (a C3 band column is ~3500 pixels: this is most of a frame's
  // paint)
  const uint64_t bit_x = 1ull << (px & 63);
  const int64_t step = (int64_t)64 * wpr;
  uint64_t* up = RP + (int64_t)(py - 1 - lane) * wpr + (px >> 6);
  for (int32_t j = lane; j < dist[1]; j += 64, up -= step) Sheet::por(up, bit_x);
  uint64_t* dn = RP + (int64_t)(py + 1 + lane) * wpr + (px >> 6);
  for (int32_t j = lane; j < dist[3]; j += 64, dn += step) Sheet::por(dn, bit_x);
}

// The four fill_lines of a frame at (px, py) (fill.c:16-43, :88-95): left,
// up, right, down.  They touch disjoint pixels, so they run together: lanes
// 16d .. 16d+15 hold line d's windows of a round trip (1024 positions), each
// lane finds its window's stop given the last match of the lanes before it
// (or of the trips before), and the first lane with a stop has the line's.
// `w` holds the first trip's windows, issued by the caller (fill_issue).
// dist[d]: pixels painted (positions 1 .. dist); the paints (the start too)
// are issued here.
__device__ __forceinline__ void fill_issue(const Sheet& S, Win& w, int32_t px, int32_t py) {
  const int lane = lane_id();
  ray_issue(S, w, lane >> 4, px, py, 0, 1 + 64 * (lane & 15));
}
template <bool LONG>
__device__ __forceinline__ void fill_cross(const Sheet& S, int32_t px, int32_t py, int32_t (&dist)[4],
                                           Win& w, BlackStats* bs) {
  const int lane = lane_id();
  if (S.I == 0) {  // the counter is 0 after the first position, whatever it holds
#pragma unroll
    for (int d = 0; d < 4; d++) dist[d] = 0;
    return;
  }
  BSTAT({ const uint64_t tw = wall_clock64(); __builtin_amdgcn_s_waitcnt(0); bs->t_wait0 += wall_clock64() - tw; })
  const int32_t edge[4] = {px + 1, py + 1, S.W - px, S.H - py};  // first position outside
  int32_t pos0[4] = {1, 1, 1, 1}, carry[4], stop[4];
#pragma unroll
  for (int d = 0; d < 4; d++) carry[d] = 1 - S.I;
  uint32_t done = 0;
  {
    // trip 0: 16 lanes a line, the windows issued with the frame's first
    // check windows (a short cross ends here)
    BSTAT(bs->fill_trips++;)
    const int ln = lane >> 4, k = lane & 15;
    const int32_t base = 1 + 64 * k;
    const uint64_t E = ray_bits(S, w, ln);
    const int32_t lastabs = E ? base + hib64(E) : INT_MIN;
    const uint64_t hasb = __ballot(E != 0);
    const uint64_t before = hasb & lane_range(16 * ln, k);
    const int32_t lsrc = __shfl(lastabs, before ? hib64(before) : lane, 64);
    const int32_t L = before ? lsrc : 1 - S.I;
    const int32_t st = window_stop(E, base, L, S.I);
    const uint64_t stb = __ballot(st != INT_MAX);
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint64_t rng = lane_range(16 * d, 16);
      int32_t sd = (stb & rng) ? __builtin_amdgcn_readlane(st, ctz64(stb & rng)) : INT_MAX;
      const int32_t end = 1 + 64 * 16;  // first position not read
      if (sd == INT_MAX && end > edge[d]) sd = edge[d];
      if (sd != INT_MAX) {
        stop[d] = imin(sd, edge[d]);
        done |= 1u << d;
      } else {
        if (hasb & rng) carry[d] = __builtin_amdgcn_readlane(lastabs, hib64(hasb & rng));
        pos0[d] = end;
      }
    }
  }
  // later trips: the lines still open share all 64 lanes (one open line:
  // 4096 positions a trip, two: 2048; three or four: 16 lanes each)
  while (uni(done) != 15) {
    BSTAT(bs->fill_trips++;)
#pragma unroll
    for (int d = 0; d < 4; d++) {
      pos0[d] = uni(pos0[d]);
      carry[d] = uni(carry[d]);
    }
    done = uni(done);
    const int nopen = __popc(~done & 15u);
    const int32_t per = (!LONG || nopen > 2) ? 16 : 64 / nopen;
    int32_t lo[4], cnt[4];
    int32_t next = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const bool open = !((done >> d) & 1);
      lo[d] = per == 16 ? 16 * d : next;
      cnt[d] = open ? per : 0;
      if (open) next += per;
    }
    int mln = -1;
#pragma unroll
    for (int d = 0; d < 4; d++)
      if (lane >= lo[d] && lane < lo[d] + cnt[d]) mln = d;
    const bool run = mln >= 0;
    const int lnx = run ? mln : 0;
    const int32_t lol = pick4(lo, lnx), kk = lane - lol;
    const int32_t base = pick4(pos0, lnx) + 64 * kk;
    if (run) ray_issue(S, w, lnx, px, py, 0, base);
    const uint64_t E = run ? ray_bits(S, w, lnx) : 0;
    // the last match of this line's lanes before this one, or the carry
    const int32_t lastabs = E ? base + hib64(E) : INT_MIN;
    const uint64_t hasb = __ballot(E != 0);
    const uint64_t before = hasb & lane_range(lol, kk);
    const int32_t lsrc = __shfl(lastabs, before ? hib64(before) : lane, 64);
    const int32_t L = before ? lsrc : pick4(carry, lnx);
    const int32_t st = run ? window_stop(E, base, L, S.I) : INT_MAX;
    const uint64_t stb = __ballot(st != INT_MAX);
#pragma unroll
    for (int d = 0; d < 4; d++) {
      if ((done >> d) & 1) continue;
      const uint64_t rng = lane_range(lo[d], cnt[d]);
      int32_t sd = (stb & rng) ? __builtin_amdgcn_readlane(st, ctz64(stb & rng)) : INT_MAX;
      const int32_t end = pos0[d] + 64 * cnt[d];  // first position not read
      if (sd == INT_MAX && end > edge[d]) sd = edge[d];
      if (sd != INT_MAX) {
        stop[d] = imin(sd, edge[d]);
        done |= 1u << d;
      } else {
        if (hasb & rng) carry[d] = __builtin_amdgcn_readlane(lastabs, hib64(hasb & rng));
        pos0[d] = end;
      }
    }
  }
#pragma unroll
  for (int d = 0; d < 4; d++) dist[d] = uni(stop[d] - 1);
  // the paints are issued by the caller after the frame's first check
  // evaluation: a wait for the check windows' loads would otherwise wait for
  // every paint atomic issued after them (one vector memory counter)
}

// Neighbour checks (flood_fill_around_line, fill.c:54-74): the checks of line
// 0, then 1, 2, 3; along a line two per position, below then above (row line)
// or right then left (column line).  A round trip reads 8 windows of both
// sides of the cursor's line dc from position p[dc] and of each later line
// from its start (lanes 16d + 8side + k).  Checks that do not match now
// cannot match later (paints only clear), and the cross's own paints touch
// none of its checks, so a frame's first round trip is issued with its fill.
constexpr int kChkWin = 8;
__device__ __forceinline__ void check_issue(const Sheet& S, Win& w, const Frame& f, int dc,
                                            const int32_t (&p)[4], bool dist_known) {
  const int lane = lane_id(), ln = lane >> 4, side = (lane >> 3) & 1, k = lane & 7;
  const int32_t base = pick4(p, ln) + 64 * k;
  if (ln >= dc && (!dist_known || base <= pick4(f.dist, ln)))
    ray_issue(S, w, ln, f.x, f.y, side == 0 ? 1 : -1, base);
}
// The loaded windows' first match at or after the cursor (line dc, position
// t, side sub), in check order; INT_MAX when none, with *next the first check
// not read.  *resume: where the frame goes on after that match's child: the
// next check, or, when the windows hold no other match, the first check not
// read (the checks between stay non-matching).
__device__ __forceinline__ int32_t check_eval(const Sheet& S, const Win& w, const Frame& f,
                                              const int32_t (&cs)[5], int dc, int32_t sub,
                                              const int32_t (&p)[4], int32_t* resume,
                                              int32_t* next) {
  const int lane = lane_id(), ln = lane >> 4, side = (lane >> 3) & 1, k = lane & 7;
  const int32_t dl = pick4(f.dist, ln);
  const int32_t base = pick4(p, ln) + 64 * k;
  const bool on = ln >= dc && base <= dl;
  uint64_t E = on ? ray_bits(S, w, ln) : 0;
  const int32_t lim = dl - base + 1;  // this window's positions on the line
  if (lim < 64) E &= lim > 0 ? (1ull << lim) - 1 : 0;
  if (ln == dc && side == 0 && k == 0 && sub) E &= ~1ull;  // behind the cursor
  const int32_t fp = E ? base + ctz64(E) : INT_MAX;
  const uint64_t hasb = __ballot(E != 0);
  const bool multi = __ballot(__popcll(E) >= 2) != 0 || __popcll(hasb) >= 2;
  int32_t cov = cs[4];  // the first check not read
#pragma unroll
  for (int d = 3; d >= 0; d--)
    if (d >= dc && p[d] + 64 * kChkWin <= f.dist[d]) cov = cs[d] + 2 * (p[d] + 64 * kChkWin - 1);
  *next = cov;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    if (d < dc) continue;
    const uint64_t r0 = hasb & lane_range(16 * d, 8), r1 = hasb & lane_range(16 * d + 8, 8);
    const int32_t f0 = r0 ? __builtin_amdgcn_readlane(fp, ctz64(r0)) : INT_MAX;
    const int32_t f1 = r1 ? __builtin_amdgcn_readlane(fp, ctz64(r1)) : INT_MAX;
    if (f0 != INT_MAX || f1 != INT_MAX) {
      const int32_t c = f0 <= f1 ? cs[d] + 2 * (f0 - 1) : cs[d] + 2 * (f1 - 1) + 1;
      *resume = multi ? c + 1 : cov;
      return c;
    }
    if (p[d] + 64 * kChkWin <= f.dist[d]) return INT_MAX;  // the line goes on past the windows
  }
  return INT_MAX;
}
__device__ __forceinline__ void check_cursor(const int32_t (&cs)[5], int32_t c, int* dc,
                                             int32_t (&p)[4], int32_t* sub) {
  *dc = c < cs[1] ? 0 : c < cs[2] ? 1 : c < cs[3] ? 2 : 3;
  const int32_t cd = *dc == 0 ? 0 : *dc == 1 ? cs[1] : *dc == 2 ? cs[2] : cs[3];
#pragma unroll
  for (int d = 0; d < 4; d++) p[d] = d == *dc ? ((c - cd) >> 1) + 1 : 1;
  *sub = (c - cd) & 1;
}
// Later check trips of a frame (its lines' lengths known): the 32 window
// slots of a trip (lane = 2 * slot + side) go to the checks in order -- the
// cursor's line from the cursor, then the following lines from their first
// position -- as many windows as each needs, so a long line is read 2048
// positions a trip instead of 512 (a C3 band column is 3508 long).
#ifndef UPH_BLACK_PLAN
#define UPH_BLACK_PLAN 1
#endif
// positions a lane reads on one side of a line per scan trip: UPH_BLACK_SPAN
// windows of 64 (32 lanes a side: 4096 positions a trip at 2)
#ifndef UPH_BLACK_SPAN
#define UPH_BLACK_SPAN 2
#endif
constexpr int kSpan = UPH_BLACK_SPAN;
constexpr int kSpanPos = 64 * kSpan;
struct ChkPlan {
  int32_t start[4], cnt[4], p0[4];  // slot range and first position per line
  int32_t cov;                      // the first check the windows do not reach
};
__device__ __forceinline__ ChkPlan check_plan(const Frame& f, const int32_t (&cs)[5], int dc,
                                              int32_t pc) {
  ChkPlan pl;
  int32_t left = 32;
  pl.cov = cs[4];
  bool open = true;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    pl.p0[d] = d == dc ? pc : 1;
    const int32_t rem = d < dc ? 0 : f.dist[d] - pl.p0[d] + 1;  // positions to read
    const int32_t need = rem > 0 ? (rem + kSpanPos - 1) / kSpanPos : 0;
    pl.start[d] = 32 - left;
    pl.cnt[d] = open ? imin(need, left) : 0;
    if (open && need > left) {  // this line runs past the trip's windows
      pl.cov = cs[d] + 2 * (pl.p0[d] + kSpanPos * left - 1);
      open = false;
    }
    left -= pl.cnt[d];
  }
  return pl;
}
__device__ __forceinline__ void check_issue_plan(const Sheet& S, Win (&w)[kSpan], const Frame& f,
                                                 const ChkPlan& pl, int* ln_out, int32_t* base_out) {
  const int lane = lane_id(), j = lane >> 1, side = lane & 1;
  int ln = -1;
  int32_t base = 0;
#pragma unroll
  for (int d = 0; d < 4; d++)
    if (j >= pl.start[d] && j < pl.start[d] + pl.cnt[d]) {
      ln = d;
      base = pl.p0[d] + kSpanPos * (j - pl.start[d]);
    }
  if (ln >= 0) {
#pragma unroll
    for (int h = 0; h < kSpan; h++) ray_issue(S, w[h], ln, f.x, f.y, side == 0 ? 1 : -1, base + 64 * h);
  }
  *ln_out = ln;
  *base_out = base;
}
// The first matching check in the planned windows (INT_MAX: none, *next =
// the plan's coverage); *resume as in check_eval.
__device__ __forceinline__ int32_t check_eval_plan(const Sheet& S, const Win (&w)[kSpan], const Frame& f,
                                                   const int32_t (&cs)[5], int dc, int32_t sub,
                                                   int32_t pc, const ChkPlan& pl, int ln, int32_t base,
                                                   int32_t* resume, int32_t* next) {
  const int lane = lane_id(), side = lane & 1;
  int32_t fpos = INT_MAX;  // the lane's first matching position
  int nm = 0;              // its matches (0, 1, or 2 = more than one)
  int32_t csd = 0;
  if (ln >= 0) {
    const int32_t dl = pick4(f.dist, ln);
#pragma unroll
    for (int h = kSpan - 1; h >= 0; h--) {
      uint64_t E = ray_bits(S, w[h], ln);
      const int32_t bh = base + 64 * h;
      const int32_t lim = dl - bh + 1;  // this window's positions on the line
      if (lim < 64) E &= lim > 0 ? (1ull << lim) - 1 : 0;
      if (h == 0 && ln == dc && side == 0 && base == pc && sub) E &= ~1ull;  // behind the cursor
      if (E) {
        fpos = bh + ctz64(E);
        nm += __popcll(E);
      }
    }
    csd = ln == 0 ? cs[0] : ln == 1 ? cs[1] : ln == 2 ? cs[2] : cs[3];
  }
  // check index of the lane's first match; slots follow the check order, so
  // the first match is in the lowest slot with one: the smaller of its two
  // sides' first matches
  const int32_t cl = fpos != INT_MAX ? csd + 2 * (fpos - 1) + side : INT_MAX;
  const uint64_t hasb = __ballot(fpos != INT_MAX);
  *next = pl.cov;
  if (!hasb) return INT_MAX;
  const int l0 = ctz64(hasb) & ~1;
  const int32_t c = imin(__builtin_amdgcn_readlane(cl, l0), __builtin_amdgcn_readlane(cl, l0 + 1));
  const bool multi = __ballot(nm >= 2) != 0 || __popcll(hasb) >= 2;
  *resume = multi ? c + 1 : pl.cov;
  return c;
}

// One planned scan trip, out of line: it is taken for long lines only, and
// inlined it costs every frame of the replay SGPR spills.
#ifndef UPH_BLACK_PLAN_NOINLINE
#define UPH_BLACK_PLAN_NOINLINE 0
#endif
#if UPH_BLACK_PLAN_NOINLINE
__device__ __attribute__((noinline))
#else
__device__ __forceinline__
#endif
int32_t check_trip_plan(const Sheet& S, const Frame& f, const int32_t (&cs)[5], int dc, int32_t sub,
                        int32_t pc, int32_t* resume, int32_t* next) {
  const ChkPlan pl = check_plan(f, cs, dc, pc);
  Win w[kSpan];
  int ln;
  int32_t base;
  check_issue_plan(S, w, f, pl, &ln, &base);
  return check_eval_plan(S, w, f, cs, dc, sub, pc, pl, ln, base, resume, next);
}

// The first matching check of frame f at or after check c, or n (none).
template <bool LONG>
__device__ __forceinline__ int32_t check_scan(const Sheet& S, const Frame& f,
                                              const int32_t (&cs)[5], int32_t c, int32_t* resume,
                                              BlackStats* bs) {
  while (c < cs[4]) {
    BSTAT(bs->check_trips++;)
    c = uni(c);
    int dc;
    int32_t p[4], sub;
    check_cursor(cs, c, &dc, p, &sub);
    const int32_t pc = pick4(p, dc);
    int32_t nx, r;
    // a line the fixed layout (8 windows a side of every line from the
    // cursor's) cannot finish in this trip: planned slots instead
    bool longl = pick4(f.dist, dc) - pc + 1 > 64 * kChkWin;
#pragma unroll
    for (int d = 0; d < 4; d++) longl |= d > dc && f.dist[d] > 64 * kChkWin;
    if (LONG && UPH_BLACK_PLAN && longl) {
      r = check_trip_plan(S, f, cs, dc, sub, pc, resume, &nx);
    } else {
      Win w;
      check_issue(S, w, f, dc, p, true);
      r = check_eval(S, w, f, cs, dc, sub, p, resume, &nx);
    }
    if (r != INT_MAX) return r;
    c = uni(nx);
  }
  return cs[4];
}

// flood_fill (fill.c:81-107) + flood_fill_around_line (fill.c:54-74), depth
// first with an explicit stack.  The caller has just read (sx, sy) as
// matching.  Returns false on a stack overflow.
template <bool LONG>
__device__ __forceinline__ bool flood(const Sheet& S, int32_t sx, int32_t sy, Frame* stack,
                                      int32_t capacity, BlackStats* bs) {
  Frame top;
  int32_t sp = 0;  // frames on the stack, `top` included; those below it in stack[0 .. sp-2]
  int32_t nx = sx, ny = sy;
  bool start = true;
  for (;;) {
    sp = uni(sp);
    nx = uni(nx);
    ny = uni(ny);
    int32_t c, resume = 0;
    int32_t cs[5];
    if (start) {
      // a new frame: save the parent; one round trip for the fill's first
      // windows and the first check windows
      if (sp >= capacity) return false;
      if (sp > 0 && lane_id() == 0) frame_put(stack, sp - 1, top);
      top.x = nx;
      top.y = ny;
      Win wf, wc;
      fill_issue(S, wf, nx, ny);
      const int32_t p1[4] = {1, 1, 1, 1};
      check_issue(S, wc, top, 0, p1, false);
      BSTAT(const uint64_t t0 = wall_clock64();)
      fill_cross<LONG>(S, nx, ny, top.dist, wf, bs);
      BSTAT(bs->t_fill += wall_clock64() - t0; bs->frames++;)
      cs[0] = 0;
#pragma unroll
      for (int d = 0; d < 4; d++) cs[d + 1] = cs[d] + 2 * top.dist[d];
      BSTAT({ const uint64_t tw = wall_clock64(); __builtin_amdgcn_s_waitcnt(0); bs->t_wait1 += wall_clock64() - tw; })
      BSTAT(const uint64_t t1 = wall_clock64(); bs->check_trips++;)
      int32_t nxt;
      c = uni(check_eval(S, wc, top, cs, 0, 0, p1, &resume, &nxt));
      // the cross's paints touch none of its checks: issued now, before any
      // later load (this wave's memory operations stay in order)
      BSTAT(const uint64_t tp = wall_clock64();)
      paint_cross<LONG>(S, nx, ny, top.dist);
      BSTAT(bs->t_paint += wall_clock64() - tp;)
      if (c == INT_MAX) c = uni(check_scan<LONG>(S, top, cs, nxt, &resume, bs));
      BSTAT(bs->t_check += wall_clock64() - t1;)
      sp++;
      start = false;
    } else {
      cs[0] = 0;
#pragma unroll
      for (int d = 0; d < 4; d++) cs[d + 1] = cs[d] + 2 * top.dist[d];
      BSTAT(const uint64_t t1 = wall_clock64();)
      c = uni(check_scan<LONG>(S, top, cs, top.cursor, &resume, bs));
      BSTAT(bs->t_check += wall_clock64() - t1;)
    }
    if (c >= cs[4]) {
      if (--sp == 0) return true;
      top = frame_pop(stack, sp - 1);
      continue;
    }
    int d = 0;
    int32_t cl = c;
    while (cl >= 2 * pick4(top.dist, d)) cl -= 2 * pick4(top.dist, d++);
    const int32_t pos = (cl >> 1) + 1, sd = cl & 1;
    if (d & 1) {
      nx = sd == 0 ? top.x + 1 : top.x - 1;
      ny = top.y + dir_dy(d) * pos;
    } else {
      nx = top.x + dir_dx(d) * pos;
      ny = sd == 0 ? top.y + 1 : top.y - 1;
    }
    top.cursor = uni(resume);
    start = true;
  }
}

template <int FMT, bool LONG>
__global__ void __launch_bounds__(64) k_black_resolve(PlaneRef img, BlackGeom g,
                                                      const BlackBar* bars, uint8_t* scratch,
                                                      int64_t sstride, const int32_t* active,
                                                      SheetCtl* ctl) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  uint8_t* scr = scratch + s * sstride;
  if (!sheet_has_candidate(g, scr)) return;
  const int lane = lane_id();
  const uint64_t* cand = (const uint64_t*)(scr + black_head_off(g) + 8);
  Frame* stack = (Frame*)(scr + black_stack_off(g));
  const uint8_t* const base = plane_ptr(img, s);
  const int64_t pitch = img.P.pitch;
  const Sheet S{(const uint64_t*)(scr + black_rm_off(g)), (uint64_t*)(scr + black_rp_off(g)),
                (const uint64_t*)(scr + black_cm_off(g)), (uint64_t*)(scr + black_cp_off(g)),
                black_wpr(g), black_hpc(g), g.W, g.H,
                (int32_t)(g.intensity > (1u << 30) ? (1u << 30) : g.intensity), g.mask_max < 255};
  BlackStats bstat{};
  BlackStats* bs = &bstat;
  (void)bs;
  BSTAT(const uint64_t t_all = wall_clock64();)
  bool dirty = false;
  for (int32_t cw = 0; cw < (g.nbars + 63) / 64; cw++) {
    for (uint64_t cm = uni64(cand[cw]); cm; cm &= cm - 1) {
      BlackBar bb = bars[64 * cw + ctz64(cm)];
      bb.r = uni_rect(bb.r);
      if (dirty) {
        // darkness on the current image: painted pixels are white
        BSTAT(const uint64_t tr = wall_clock64(); bs->remeasures++;)
        const Rect c = clip(bb.r, g.W, g.H);
        uint64_t sum = 0;
        if (c.x0 <= c.x1 && c.y0 <= c.y1 && FMT == F_GRAY8 && pitch % 16 == 0 &&
            ((uintptr_t)base & 15) == 0) {
          // GRAY8: a lane per (row, 64-pixel word of the row plane): the P
          // word and the segment's 64 bytes as four 16-byte loads, four
          // segments' loads in flight at once (a bar is ~10^4 pixels: a
          // load round trip a pixel made a remeasure ~40 us)
          const int32_t w0 = c.x0 >> 6, nw = (c.x1 >> 6) - w0 + 1;
          const int32_t nseg = nw * (c.y1 - c.y0 + 1);
          constexpr int kU = 4;
          for (int32_t i0 = lane; i0 < nseg; i0 += 64 * kU) {
            uint64_t pw[kU];
            uint4 px[kU][4];
            int32_t lo[kU], hi[kU];
#pragma unroll
            for (int u = 0; u < kU; u++) {
              const int32_t i = i0 + 64 * u;
              const bool ok = i < nseg;
              const int32_t y = c.y0 + (ok ? i / nw : 0), w = w0 + (ok ? i % nw : 0);
              lo[u] = ok ? imax(c.x0 - 64 * w, 0) : 64;
              hi[u] = ok ? imin(c.x1 - 64 * w, 63) : -1;
              pw[u] = ok ? Sheet::pload(S.RP + (int64_t)y * S.wpr + w) : 0ull;
              const uint4* q = reinterpret_cast<const uint4*>(base + (int64_t)y * pitch + 64 * w);
#pragma unroll
              for (int k = 0; k < 4; k++) {
                // the row's last word may reach past the pitch: only bytes
                // at or below x1 are summed, and loads stay inside the row
                const bool in = ok && 64 * w + 16 * k < (int32_t)pitch;
                px[u][k] = in ? q[k] : make_uint4(0, 0, 0, 0);
              }
            }
            // painted pixels count 255 (white); the others' bytes are summed
            // four at a time (v_sad_u8 over the bytes the mask keeps)
            uint32_t acc = 0;
#pragma unroll
            for (int u = 0; u < kU; u++) {
              const uint64_t rmask =
                  hi[u] >= lo[u] ? (~0ull >> (63 - hi[u])) & (~0ull << lo[u]) : 0ull;
              sum += 255u * (uint32_t)__popcll(pw[u] & rmask);
              const uint64_t keep = rmask & ~pw[u];
#pragma unroll
              for (int k = 0; k < 4; k++) {
                const uint32_t d4[4] = {px[u][k].x, px[u][k].y, px[u][k].z, px[u][k].w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                  const uint32_t m = (uint32_t)(keep >> (16 * k + 4 * j)) & 0xFu;
                  const uint32_t M = ((m * 0x00204081u) & 0x01010101u) * 0xFFu;
                  acc = __builtin_amdgcn_sad_u8(d4[j] & M, 0u, acc);
                }
              }
            }
            sum += acc;
          }
        } else if (c.x0 <= c.x1 && c.y0 <= c.y1) {
          const int32_t cwid = c.x1 - c.x0 + 1;
          const int64_t npx = (int64_t)cwid * (c.y1 - c.y0 + 1);
          const int32_t q64 = 64 / cwid, r64 = 64 % cwid;
          int32_t y = c.y0 + lane / cwid, x = c.x0 + lane % cwid;
          for (int64_t i = lane; i < npx; i += 64) {
            const uint64_t pw = Sheet::pload(S.RP + (int64_t)y * S.wpr + (x >> 6));
            const uint32_t v = dark_of(load_px_row<FMT>(base + (int64_t)y * pitch, x));
            sum += ((pw >> (x & 63)) & 1) ? 255u : v;
            x += r64;
            y += q64;
            if (x > c.x1) {
              x -= cwid;
              y++;
            }
          }
        }
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
        sum = uni64(sum);  // every lane holds the total: the decision is the wave's
        const uint8_t dark = (uint8_t)(0xFFull - sum / count_pixels(c));
        BSTAT(bs->t_remeasure += wall_clock64() - tr;)
        if (dark < g.abs_threshold) continue;
      }
      // flood fill from every pixel of the bar in scan order (filters.c:86-89):
      // lanes are 64-pixel segments of the bar's rows, row-major
      const int32_t bw = bb.r.x1 - bb.r.x0 + 1, bh = bb.r.y1 - bb.r.y0 + 1;
      if (bw <= 0 || bh <= 0) continue;
      const int32_t nseg = (bw + 63) >> 6;
      const int32_t total = nseg * bh;
      int32_t cy = bb.r.y0, cx = bb.r.x0;  // next pixel to look at
      for (;;) {
        BSTAT(const uint64_t tb = wall_clock64(); bs->bar_trips++;)
        cy = uni(cy);
        cx = uni(cx);
        const int32_t k0 = (cy - bb.r.y0) * nseg + ((cx - bb.r.x0) >> 6);
        if (k0 >= total) break;
        const int32_t kk = k0 + lane;
        const int32_t ry = bb.r.y0 + kk / nseg, sx = bb.r.x0 + 64 * (kk % nseg);
        Win w;
        const bool on = kk < total;
        if (on) w.issue(S, false, ry, sx);
        uint64_t e = on ? w.bits(S) : 0;
        const int32_t wlim = bb.r.x1 - sx + 1;  // pixels of this segment in the bar
        if (wlim < 64) e &= (1ull << wlim) - 1;
        if (lane == 0 && cx > sx) e &= ~0ull << (cx - sx);  // before the cursor: done
        const uint64_t hit = __ballot(e != 0);
        BSTAT(bs->t_bar += wall_clock64() - tb;)
        if (!hit) {
          const int32_t kn = k0 + 64;
          if (kn >= total) break;
          cy = bb.r.y0 + kn / nseg;
          cx = bb.r.x0 + 64 * (kn % nseg);
          continue;
        }
        const int hl = ctz64(hit);
        const int32_t fx = __builtin_amdgcn_readlane(sx + (e ? ctz64(e) : 0), hl);
        const int32_t fy = __builtin_amdgcn_readlane(ry, hl);
        if (!flood<LONG>(S, fx, fy, stack, g.stack_capacity, bs)) {
          if (lane == 0 && ctl) atomicOr(&ctl[s].status, STATUS_FLOOD_OVERFLOW);
          return;
        }
        dirty = true;
        cy = fy;
        cx = fx + 1;
        if (cx > bb.r.x1) {
          cx = bb.r.x0;
          cy++;
        }
      }
    }
  }
#ifdef UPHIP_DIAG
  if ((g.diag & 16) && lane == 0 && bstat.frames)
    printf("uphip black: sheet %d frames %u fill %u (%.1f us) check %u (%.1f us) bar %u (%.1f us) "
           "remeasure %u (%.1f us) wait0 %.1f paint %.1f wait1 %.1f total %.1f us\n",
           s, bstat.frames, bstat.fill_trips, bstat.t_fill * 0.01, bstat.check_trips,
           bstat.t_check * 0.01, bstat.bar_trips, bstat.t_bar * 0.01, bstat.remeasures,
           bstat.t_remeasure * 0.01, bstat.t_wait0 * 0.01, bstat.t_paint * 0.01,
           bstat.t_wait1 * 0.01, (wall_clock64() - t_all) * 0.01);
#endif
}

template <int FMT>
static void launch_black_t(const PlaneRef& img, const BlackGeom& g, const BlackBar* bars,
                           uint8_t* scr, int64_t ss, const int32_t* active, SheetCtl* ctl,
                           int count, hipStream_t st, const AxisArgs* hargs,
                           const AxisArgs* vargs, bool vsum_ready, uint32_t* nbits,
                           int64_t nbits_stride, uint32_t* bbits, int64_t bb_stride,
                           bool rm_ready) {
  // column sums of max(rgb) over the h-stripe rows, row sums over the v-stripe cols
  if (g.hregion.x1 >= g.hregion.x0 && g.hregion.y1 >= g.hregion.y0)
    launch_axis_reduce(img, hargs, 0, M_DARKINV_SUM, g.W, g.H, (uint32_t*)scr, ss / 4, count, st);
  if (g.vregion.x1 >= g.vregion.x0 && g.vregion.y1 >= g.vregion.y0 && !vsum_ready)
    launch_axis_reduce(img, vargs, 1, M_DARKINV_SUM, g.vregion.x1 - g.vregion.x0 + 1, g.H,
                       (uint32_t*)scr + g.W, ss / 4, count, st);
  hipLaunchKernelGGL(k_black_cand, dim3(count), dim3(kCandThreads), 0, st, g, bars, scr, ss, active);
  if (FMT == F_GRAY8 && rm_ready)
    hipLaunchKernelGGL((k_black_planes<FMT, true>), dim3((black_wpr(g) + 3) / 4, black_hpc(g), count),
                       dim3(256), 0, st, img, g, scr, ss, active);
  else
    hipLaunchKernelGGL((k_black_planes<FMT, false>), dim3((black_wpr(g) + 3) / 4, black_hpc(g), count),
                       dim3(256), 0, st, img, g, scr, ss, active);
  BlackGeom gd = g;
  gd.diag = diag_noise();
  // LONG: the long-line machinery (open fill lines sharing the wave, planned
  // two-window scan trips, pointer-walk paints).  Exact either way; chosen by
  // sheet size as measured: A4 pages (a solid band: ~40 frames of 3508-long
  // columns) 877 -> ~540 us a 64-sheet launch, while on C4's 70-Mpixel sheets
  // (floods percolating through specks: ~17k short crosses) its register
  // pressure made every frame slower (heaviest sheet 75 -> 88 ms).
  const bool longl = (int64_t)g.W * g.H <= (16 << 20);
  if (!(diag_skip() & 1)) {
    if (longl) {
      allow_dynamic_lds((const void*)k_black_resolve<FMT, true>, kStackLdsBytes);
      hipLaunchKernelGGL((k_black_resolve<FMT, true>), dim3(count), dim3(64), kStackLdsBytes, st, img, gd,
                         bars, scr, ss, active, ctl);
    } else {
      allow_dynamic_lds((const void*)k_black_resolve<FMT, false>, kStackLdsBytes);
      hipLaunchKernelGGL((k_black_resolve<FMT, false>), dim3(count), dim3(64), kStackLdsBytes, st, img, gd,
                         bars, scr, ss, active, ctl);
    }
  }
  hipLaunchKernelGGL(k_black_paint<FMT>, dim3((black_wpr(g) + 63) / 64, (g.H + 3) / 4, count),
                     dim3(256), 0, st, img, g, scr, ss, active, FMT == F_GRAY8 ? nbits : nullptr,
                     nbits_stride, FMT == F_GRAY8 ? bbits : nullptr, bb_stride);
}

uint32_t* black_rm_plane(const BlackGeom& g, void* scratch) {
  return (uint32_t*)((uint8_t*)scratch + black_rm_off(g));
}

__global__ void k_black_prep(uint8_t* scr, int64_t ss, int32_t words, int count) {
  // zero the column sums (atomic accumulation) of every sheet
  const int s = blockIdx.y;
  uint32_t* p = (uint32_t*)(scr + s * ss);
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += gridDim.x * blockDim.x)
    p[i] = 0;
}

void launch_blackfilter_impl(const PlaneRef& img, const BlackGeom& g, const BlackBar* bars,
                             void* scratch, int64_t ss, const int32_t* active, SheetCtl* ctl,
                             int count, hipStream_t st, const AxisArgs* hargs,
                             const AxisArgs* vargs, bool vsum_ready, uint32_t* nbits,
                             int64_t nbits_stride, uint32_t* bbits, int64_t bb_stride,
                             bool rm_ready) {
  uint8_t* scr = (uint8_t*)scratch;
  hipLaunchKernelGGL(k_black_prep, dim3(8, count), dim3(256), 0, st, scr, ss, g.W, count);
  switch (img.P.fmt) {
    case F_GRAY8:
      launch_black_t<F_GRAY8>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs,
                              vsum_ready, nbits, nbits_stride, bbits, bb_stride, rm_ready);
      break;
    case F_Y400A:
      launch_black_t<F_Y400A>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs,
                              vsum_ready, nbits, nbits_stride, bbits, bb_stride, rm_ready);
      break;
    default:
      launch_black_t<F_RGB24>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs,
                              vsum_ready, nbits, nbits_stride, bbits, bb_stride, rm_ready);
      break;
  }
}

}  // namespace uph
