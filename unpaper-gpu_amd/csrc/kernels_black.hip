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
// non-matching pixels), so one wave replays it: an explicit stack of frames in
// HBM, one workgroup per sheet: the four fill_lines of a frame together, and
// the neighbour and bar-pixel checks in windows of 4096 read ahead, 64 pixels
// per ballot, the window's slices spread over the workgroup's waves.
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

size_t black_scratch_bytes(const BlackGeom& g) {
  // [sums: W (h-stripe columns) + H (v-stripe rows)] u32 + DFS stack frames
  size_t b = ((size_t)g.W + g.H) * 4;
  b = (b + 255) & ~(size_t)255;
  b += (size_t)g.stack_capacity * 32;
  return (b + 255) & ~(size_t)255;
}

struct Frame {
  int32_t x, y;
  int32_t dist[4];
  int32_t cursor;  // next neighbour check, over the four lines' checks in order
  int32_t pad;
};

// left, up, right, down (fill.c:92-106)
__device__ __forceinline__ constexpr int dir_dx(int d) { return d == 0 ? -1 : d == 2 ? 1 : 0; }
__device__ __forceinline__ constexpr int dir_dy(int d) { return d == 1 ? -1 : d == 3 ? 1 : 0; }

template <class T>
__device__ __forceinline__ T pick4(const T (&a)[4], int d) {
  return d == 0 ? a[0] : d == 1 ? a[1] : d == 2 ? a[2] : a[3];
}
template <class T>
__device__ __forceinline__ void set4(T (&a)[4], int d, T v) {
  if (d == 0) a[0] = v;
  else if (d == 1) a[1] = v;
  else if (d == 2) a[2] = v;
  else a[3] = v;
}

// The replay is one workgroup of kWaves waves per sheet.  Control (the DFS
// stack, the current frame, the bar loop) is uniform: every wave runs it on
// the same values, read from LDS after a barrier.  The per-pixel work of a
// round trip is a window of kSlices 64-pixel slices, kGroup per wave.
constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kGroup = 8;
constexpr int kSlices = kWaves * kGroup;  // 64 slices = 4096 pixels per round trip
static_assert(kSlices == 64, "lane-parallel reads of the per-slice tables assume 64 slices");

// Per-round-trip tables in LDS (the window's results of each wave).
constexpr int kOffStop = 0;                       // i32[2][3][kWaves] fill-trip posts + 12 more
constexpr int kOffFirst = kOffStop + 4 * kWaves;  // i32[2][kWaves] first matches
constexpr int kOffRed = kOffFirst + kWaves;       // u64[kWaves] sums
constexpr int kOffCand = kOffRed + kWaves;        // u64[kWaves] candidate bars
constexpr int kOffMail = kOffCand + kWaves;       // i32[16] driver -> helper commands
constexpr int kReplayWords = kOffMail + 8;        // in 8-byte units

__device__ __forceinline__ uint64_t* lds64() {
  __shared__ uint64_t black_tables[kReplayWords];
  return black_tables;
}
__device__ __forceinline__ int32_t* tab_stop() { return (int32_t*)(lds64() + kOffStop); }
__device__ __forceinline__ int32_t* tab_first() { return (int32_t*)(lds64() + kOffFirst); }
__device__ __forceinline__ uint64_t* tab_red() { return lds64() + kOffRed; }
__device__ __forceinline__ uint64_t* tab_cand() { return lds64() + kOffCand; }
__device__ __forceinline__ int32_t* mailbox() { return (int32_t*)(lds64() + kOffMail); }

// The lowest kStackLds frames of the DFS stack live in LDS (dynamic), the
// rest in HBM: a pop is then an LDS read instead of a memory round trip.
constexpr int kStackLds = 3072;
constexpr size_t kStackLdsBytes = (size_t)kStackLds * 32;  // 96 KiB
__device__ __forceinline__ int4* stack_lds() {
  extern __shared__ int4 black_stack[];
  return black_stack;
}
__device__ __forceinline__ void frame_put(int4* lds, Frame* hbm, int32_t i, const Frame& f) {
  const int4 a = make_int4(f.x, f.y, f.dist[0], f.dist[1]);
  const int4 b = make_int4(f.dist[2], f.dist[3], f.cursor, 0);
  if (i < kStackLds) {
    lds[2 * i] = a;
    lds[2 * i + 1] = b;
  } else {
    hbm[i] = f;
  }
}
__device__ __forceinline__ Frame frame_get(const int4* lds, const Frame* hbm, int32_t i) {
  if (i >= kStackLds) return hbm[i];
  const int4 a = lds[2 * i], b = lds[2 * i + 1];
  Frame f;
  f.x = a.x;
  f.y = a.y;
  f.dist[0] = a.z;
  f.dist[1] = a.w;
  f.dist[2] = b.x;
  f.dist[3] = b.y;
  f.cursor = b.z;
  f.pad = 0;
  return f;
}

// scalar (readfirstlane), so everything derived from it stays in SGPRs
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int32_t wave_min(int32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = imin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// barrier with a workgroup fence: paints (image stores) of every wave are
// visible to every wave after it
__device__ __forceinline__ void block_sync() { __syncthreads(); }
// replay counters, tuning build only (UPHIP_DIAG_NOISE bit 16)
struct BlackStats {
  uint32_t frames, fill_trips, check_trips, bar_trips, remeasures, lookups;
  uint64_t t_fill, t_check, t_bar, t_remeasure, t_fa, t_fb, t_fc, t_fd, t_fa0, t_fa1, t_local, t_pop;
};
#ifdef UPHIP_DIAG
#define BSTAT(...) __VA_ARGS__
#else
#define BSTAT(...)
#endif

template <int FMT>
struct Canvas {
  uint8_t* base;
  int64_t pitch;
  int32_t W, H;
  uint8_t mmax;  // mask_max (mask_min is 0)
  BlackStats* bs;  // tuning build counters
  uint32_t* nbits;  // the noisefilter's dark bit-plane of this sheet (or null)
  int32_t nwr;      // its words per row
  __device__ __forceinline__ bool inside(int32_t x, int32_t y) const {
    return x >= 0 && y >= 0 && x < W && y < H;
  }
  // N matches of this wave: the loads of all are issued before any is used,
  // so one memory round trip serves the group.  x < 0 means "no position"
  // (no match).
  template <int N>
  __device__ __forceinline__ void match_group(const int32_t (&x)[N], const int32_t (&y)[N],
                                              bool (&m)[N]) const {
    uint8_t g[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
      const int32_t cy = imin(imax(y[k], 0), H - 1), cx = imin(imax(x[k], 0), W - 1);
      g[k] = gray_of(load_px_row<FMT>(base + (int64_t)cy * pitch, cx));
    }
#pragma unroll
    for (int k = 0; k < N; k++) m[k] = inside(x[k], y[k]) && g[k] <= mmax;
    BSTAT(bs->lookups += N;)
  }
  __device__ __forceinline__ void paint(int32_t x, int32_t y) const {
    if (!inside(x, y)) return;
    store_px_row<FMT>(base + (int64_t)y * pitch, x, Px{255, 255, 255});
    // white is not dark: the bit-plane follows the fill
    if (nbits) atomicAnd(nbits + (int64_t)y * nwr + (x >> 5), ~(1u << (x & 31)));
  }
};

// The four fill_lines (fill.c:16-52) from (px,py); dist[d] = pixels painted.
// Per line a counter starts at 1, resets to `intensity` on a match and
// decrements otherwise; the line stops (unpainted) where it reaches 0 or
// leaves the image: at the first position p that is outside, or does not
// match and lies `intensity` or more past the last match (the first
// non-matching position if there was none).  The four lines touch disjoint
// pixels (left, up, right, down of the start), so they share each round trip:
// the window's slices are split evenly over the lines still running, whole
// waves per line (16, 32 or 64 slices a line, 8 a wave).  A round trip is
//   A: each wave reads its slices and posts their first match F, last match
//      L, and the first stop I after F (which needs no carry from before);
//   C: one barrier, then every wave walks each line's posts in order with
//      the carry (last match so far) to find the line's stop, uniformly;
//   D: paint up to the stop.
// The posts alternate between two buffers, so a round trip has one barrier;
// the paints are published by the barrier after the four lines.
// The four fill_lines (fill.c:16-52) from (px,py); dist[d] = pixels painted.
// Per line a counter starts at 1, resets to `intensity` on a match and
// decrements otherwise; the line stops (unpainted) where it reaches 0 or
// leaves the image: at the first position p that is outside, or does not
// match and lies `intensity` or more past the last match (the first
// non-matching position if there was none).  The four lines touch disjoint
// pixels (left, up, right, down of the start), so they share each round trip.
//
// fill_local: the first round trip, by the driving wave alone: the first
// 64 kLocalSl positions of each line.  Most lines of most frames end there.  The lines' state goes to `lpost`; returns
// whether a line runs on.
constexpr int kLocalSl = 2;  // slices per line of a frame's first round trip (1: more lines go cooperative, slower overall)

template <int FMT>
__device__ __forceinline__ bool fill_local(const Canvas<FMT>& C, int32_t px, int32_t py,
                                           uint64_t intensity, int32_t (&dist)[4],
                                           BlackStats* bs) {
  const int lane = lane_id();
  const uint64_t upto_mask = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  int32_t* lpost = tab_stop() + 6 * kWaves;  // [4] stop | [4] has_last | [4] last
  bool more = false;
  int32_t qx[4 * kLocalSl], qy[4 * kLocalSl];
  bool m[4 * kLocalSl];
#pragma unroll
  for (int i = 0; i < 4 * kLocalSl; i++) {
    const int dd = i / kLocalSl;
    const int32_t j = 1 + 64 * (i % kLocalSl) + lane;
    qx[i] = dd == 0 ? px - j : dd == 2 ? px + j : px;
    qy[i] = dd == 1 ? py - j : dd == 3 ? py + j : py;
  }
  C.match_group(qx, qy, m);
#pragma unroll
  for (int dd = 0; dd < 4; dd++) {
    bool hl = false;
    int32_t lm = 0, stop = INT_MAX;
#pragma unroll
    for (int k = 0; k < kLocalSl; k++) {
      const int i = kLocalSl * dd + k;
      const unsigned long long Mi = __ballot(m[i]);
      if (stop == INT_MAX) {
        const int32_t p0 = 1 + 64 * k, j = p0 + lane;
        const unsigned long long upto = Mi & upto_mask;
        bool lhl = hl;
        int32_t llm = lm;
        if (upto) {
          lhl = true;
          llm = p0 + (63 - __clzll((long long)upto));
        }
        bool st = !C.inside(qx[i], qy[i]);
        if (lhl) st |= (uint64_t)(uint32_t)(j - llm) >= intensity;
        else st |= j >= 1;
        const unsigned long long S = __ballot(st);
        if (S) stop = p0 + __ffsll((long long)S) - 1;
        if (Mi) {
          hl = true;
          lm = p0 + (63 - __clzll((long long)Mi));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kLocalSl; k++)
      if (1 + 64 * k + lane < stop) C.paint(qx[kLocalSl * dd + k], qy[kLocalSl * dd + k]);
    if (lane == 0) {
      lpost[dd] = stop;
      lpost[4 + dd] = hl;
      lpost[8 + dd] = lm;
    }
    if (stop != INT_MAX) set4(dist, dd, stop - 1);
    else more = true;
  }
  BSTAT(bs->fill_trips++;)
  return more;
}

// fill_coop: the rest of the lines, by the whole workgroup, from the state in
// `lpost`: the window's slices are split evenly over the lines still running,
// whole waves per line (16, 32 or 64 slices a line, 8 a wave).  A round trip is
//   A: each wave reads its slices and posts their first match F, last match
//      L, and the first stop I after F (which needs no carry from before);
//   C: one barrier, then every wave walks each line's posts in order with
//      the carry (last match so far) to find the line's stop, uniformly;
//   D: paint up to the stop.
// The posts alternate between two buffers, so a round trip has one barrier;
// the paints are published by the barrier after the four lines.
template <int FMT>
__device__ __forceinline__ void fill_coop(const Canvas<FMT>& C, int32_t px, int32_t py,
                                          uint64_t intensity, int32_t (&dist)[4],
                                          BlackStats* bs) {
  const int w = wave_id(), lane = lane_id();
  BSTAT(const uint64_t t0 = wall_clock64();)
  uint32_t done = 0, has_last = 0;  // per line bits (bool arrays indexed by a
                                    // run-time line would live in scratch)
  int32_t last[4] = {0, 0, 0, 0};   // positions along a line fit 31 bits
  constexpr int32_t kFirst = 1 + 64 * kLocalSl;  // fill_local read positions 1 .. kFirst - 1
  int32_t pos0[4] = {kFirst, kFirst, kFirst, kFirst};
  // first position outside the image, per line
  const int32_t edge[4] = {px + 1, py + 1, C.W - px, C.H - py};
  const uint64_t upto_mask = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  {
    const int32_t* lpost = tab_stop() + 6 * kWaves;
    const int32_t v = lane < 12 ? lpost[lane] : 0;
#pragma unroll
    for (int dd = 0; dd < 4; dd++) {
      const int32_t stop = __builtin_amdgcn_readlane(v, dd);
      if (stop != INT_MAX) {
        done |= 1u << dd;
        set4(dist, dd, stop - 1);
      } else {
        if (__builtin_amdgcn_readlane(v, 4 + dd)) has_last |= 1u << dd;
        set4(last, dd, __builtin_amdgcn_readlane(v, 8 + dd));
      }
    }
  }
  int parity = 0;
  for (;;) {
    uint32_t actp = 0;  // running lines, a nibble each
    int nact = 0;
#pragma unroll
    for (int d = 0; d < 4; d++)
      if (!((done >> d) & 1)) actp |= (uint32_t)d << (4 * nact++);
    if (nact == 0) break;
    const int lg = nact == 1 ? 6 : nact == 2 ? 5 : 4;  // log2 slices per line
    const int spd = 1 << lg, wpl = spd / kGroup;        // slices, waves per line
    // this wave's line and first slice (uniform)
    const int a = (w * kGroup) >> lg, k0 = (w * kGroup) & (spd - 1);
    const bool valid = a < nact;
    const int d = (int)((actp >> (4 * (valid ? a : 0))) & 15);
    const int32_t base0 = pick4(pos0, d) + 64 * k0;  // position of lane 0, slice 0
    int32_t* post = tab_stop() + parity * 3 * kWaves;  // F | L | I, per wave
    parity ^= 1;
    BSTAT(uint64_t tp = wall_clock64();)
    // A
    int32_t qx[kGroup], qy[kGroup];
    bool m[kGroup];
#pragma unroll
    for (int i = 0; i < kGroup; i++) {
      const int32_t j = base0 + 64 * i + lane;
      qx[i] = !valid ? -1 : d == 0 ? px - j : d == 2 ? px + j : px;
      qy[i] = d == 1 ? py - j : d == 3 ? py + j : py;
    }
    BSTAT(bs->t_fa0 += wall_clock64() - tp;)
    C.match_group(qx, qy, m);
    BSTAT(bs->t_fa1 += wall_clock64() - tp;)
    int32_t F = -1, L = -1, I = INT_MAX;
    {
      bool hl = false;  // a match earlier in this wave's slices
      int32_t lm = 0;
#pragma unroll
      for (int i = 0; i < kGroup; i++) {
        const unsigned long long Mi = __ballot(m[i]);
        const int32_t p0 = base0 + 64 * i, j = p0 + lane;
        if (I == INT_MAX) {
          const unsigned long long upto = Mi & upto_mask;
          bool lhl = hl;
          int32_t llm = lm;
          if (upto) {
            lhl = true;
            llm = p0 + (63 - __clzll((long long)upto));
          }
          // after the wave's first match only: before it the carry decides
          const unsigned long long S = __ballot(lhl && (uint64_t)(uint32_t)(j - llm) >= intensity);
          if (S) I = p0 + __ffsll((long long)S) - 1;
        }
        if (Mi) {
          if (F < 0) F = p0 + __ffsll((long long)Mi) - 1;
          L = p0 + (63 - __clzll((long long)Mi));
          hl = true;
          lm = L;
        }
      }
    }
    if (lane == 0) {
      post[w] = valid ? F : -1;
      post[kWaves + w] = valid ? L : -1;
      post[2 * kWaves + w] = valid ? I : INT_MAX;
    }
    block_sync();
    BSTAT(bs->t_fa += wall_clock64() - tp; tp = wall_clock64();)
    // C (uniform): per line, lanes stand for its waves; each lane takes the
    // carry from the line's earlier waves (or the previous round trip) and
    // finds its wave's stop; the first lane with one has the line's stop
    const int32_t vF = lane < kWaves ? post[lane] : -1;
    const int32_t vL = lane < kWaves ? post[kWaves + lane] : -1;
    const int32_t vI = lane < kWaves ? post[2 * kWaves + lane] : INT_MAX;
    const unsigned long long withL = __ballot(vL >= 0);
    int32_t sd[4] = {INT_MAX, INT_MAX, INT_MAX, INT_MAX};
#pragma unroll
    for (int aa = 0; aa < 4; aa++) {
      if (aa >= nact) break;
      const int dd = (int)((actp >> (4 * aa)) & 15);
      const int lo = aa * wpl;
      const unsigned long long range = ((1ull << wpl) - 1) << lo;
      const bool inr = (range >> lane) & 1;
      const unsigned long long before = withL & range & ((1ull << lane) - 1);
      const int src = before ? 63 - __clzll((long long)before) : lane;
      const int32_t lmv = __shfl(vL, src, 64);
      const bool has = before ? true : ((has_last >> dd) & 1);
      const int32_t lm = before ? lmv : pick4(last, dd);
      const int32_t Pv = pick4(pos0, dd) + 64 * kGroup * (lane - lo);
      const int32_t end = vF >= 0 ? vF : Pv + 64 * kGroup;  // no match in [Pv, end)
      const int32_t cand =
          has ? imax(Pv, (int32_t)imin((int64_t)lm + (int64_t)intensity, (int64_t)INT_MAX)) : Pv;
      const int32_t sv = cand < end ? cand : vI;
      const unsigned long long stops = __ballot(inr && sv != INT_MAX);
      int32_t stop = stops ? __shfl(sv, __ffsll((long long)stops) - 1, 64) : INT_MAX;
      stop = imin(stop, pick4(edge, dd));
      if (stop < pick4(pos0, dd) + 64 * spd) {
        set4(sd, dd, stop);
        done |= 1u << dd;
        set4(dist, dd, stop - 1);
      } else {
        const unsigned long long mine = withL & range;
        if (mine) {
          has_last |= 1u << dd;
          set4(last, dd, __shfl(vL, 63 - __clzll((long long)mine), 64));
        }
        set4(pos0, dd, pick4(pos0, dd) + 64 * spd);
      }
    }
    BSTAT(bs->t_fc += wall_clock64() - tp; tp = wall_clock64();)
    // D
    if (valid) {
      const int32_t lim = pick4(sd, d);
#pragma unroll
      for (int i = 0; i < kGroup; i++)
        if (base0 + 64 * i + lane < lim) C.paint(qx[i], qy[i]);
    }
    BSTAT(bs->t_fd += wall_clock64() - tp; bs->fill_trips++;)
  }
  block_sync();  // the lines' paints, before any check reads them
  BSTAT(bs->t_fill += wall_clock64() - t0;)
}

// Neighbour check number c of a frame (flood_fill_around_line, fill.c:62-79):
// the checks of line 0, then 1, 2, 3; along a line two per position, below
// then above (horizontal line) or right then left (vertical line).
__device__ __forceinline__ void check_pos(const Frame& f, int32_t c, int32_t* qx, int32_t* qy) {
  const int32_t n0 = 2 * f.dist[0], n1 = n0 + 2 * f.dist[1], n2 = n1 + 2 * f.dist[2];
  const int d = c < n0 ? 0 : c < n1 ? 1 : c < n2 ? 2 : 3;
  const int32_t cc = c - (d == 0 ? 0 : d == 1 ? n0 : d == 2 ? n1 : n2);
  const int32_t t = (cc >> 1) + 1, sub = cc & 1;
  const int dx = dir_dx(d), dy = dir_dy(d);
  int32_t x = f.x + t * dx, y = f.y + t * dy;
  if (dx != 0) y += sub == 0 ? 1 : -1;  // below, then above
  else x += sub == 0 ? 1 : -1;           // right, then left
  *qx = x;
  *qy = y;
}

// First match of a window whose slices were looked up by every wave: each
// wave posts the index of its first matching position (or INT_MAX) into the
// buffer of this round trip's parity, then all read the minimum.  M[i] is
// the ballot of slice i; with pairs (every lane two consecutive positions),
// M0[i] says which lanes matched their first one.
template <bool kPairs>
__device__ __forceinline__ int32_t window_first(const uint64_t (&M)[kGroup],
                                                const uint64_t (&M0)[kGroup], int parity) {
  const int w = wave_id(), lane = lane_id();
  int32_t lf = INT_MAX;
#pragma unroll
  for (int i = kGroup - 1; i >= 0; i--) {
    if (M[i]) {
      const int L = __ffsll((long long)M[i]) - 1;
      const int32_t u = 64 * (w * kGroup + i) + L;
      lf = kPairs ? 2 * u + (((M0[i] >> L) & 1) ? 0 : 1) : u;
    }
  }
  int32_t* first = tab_first() + parity * kWaves;
  if (lane == 0) first[w] = lf;
  block_sync();
  // waves hold consecutive slices: the first wave that found one has the minimum
  const int32_t v = lane < kWaves ? first[lane] : INT_MAX;
  const unsigned long long any = __ballot(v != INT_MAX);
  return any ? __shfl(v, __ffsll((long long)any) - 1, 64) : INT_MAX;
}

// The flood fill is driven by wave 0 alone.  Its small steps (a frame's
// first 128 pixels per line, a check window of at most 512 checks) need no
// other wave and no barrier; a long line or a long run of checks is posted as
// a command, and the other waves, parked in `flood_help`, join for it.
// A command's operation ends in a barrier that every wave reaches, so the
// driver never rewrites the mailbox before the helpers have read it.
enum : int32_t { CMD_DONE = 0, CMD_FILL = 1, CMD_CHECK = 2 };
// mailbox: [0] sequence, [1] command, [2..3] fill start, [4..11] frame
// (x, y, dist[4], cursor, checks), [12] flood result

__device__ __forceinline__ void post_command(int32_t* seq, int32_t cmd) {
  int32_t* mb = mailbox();
  if (lane_id() == 0) mb[1] = cmd;
  // arguments and paints before the sequence number that publishes them
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane_id() == 0) __hip_atomic_store(&mb[0], ++*seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else ++*seq;
}

// One check window of the whole workgroup (64 slices, 4096 checks).
template <int FMT>
__device__ __forceinline__ int32_t check_coop(const Canvas<FMT>& C, const Frame& top, int32_t n,
                                              int* parity, BlackStats* bs) {
  const int w = wave_id(), lane = lane_id();
  int32_t qx[kGroup], qy[kGroup];
  bool m[kGroup];
#pragma unroll
  for (int i = 0; i < kGroup; i++) {
    const int32_t c = top.cursor + 64 * (w * kGroup + i) + lane;
    check_pos(top, imin(c, n - 1), &qx[i], &qy[i]);
    if (c >= n) qx[i] = -1;
  }
  C.match_group(qx, qy, m);
  uint64_t M[kGroup];
#pragma unroll
  for (int i = 0; i < kGroup; i++) M[i] = __ballot(m[i]);
  return window_first<false>(M, M, (*parity)++ & 1);
}

// The helpers' side: run the driver's commands until CMD_DONE.
template <int FMT>
__device__ void flood_help(const Canvas<FMT>& C, uint64_t intensity, int32_t* seen, int* parity,
                           BlackStats* bs) {
  int32_t* mb = mailbox();
  for (;;) {
    int32_t sq;
    while ((sq = __hip_atomic_load(&mb[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) ==
           *seen)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    *seen = sq;
    const int32_t cmd = mb[1];
    if (cmd == CMD_DONE) return;
    if (cmd == CMD_FILL) {
      int32_t dist[4];
      fill_coop<FMT>(C, mb[2], mb[3], intensity, dist, bs);
    } else {
      Frame f;
      f.x = mb[4];
      f.y = mb[5];
      f.dist[0] = mb[6];
      f.dist[1] = mb[7];
      f.dist[2] = mb[8];
      f.dist[3] = mb[9];
      f.cursor = mb[10];
      check_coop<FMT>(C, f, mb[11], parity, bs);
    }
  }
}

// flood_fill (fill.c:81-107) + flood_fill_around_line (fill.c:62-79), depth
// first with an explicit stack in HBM, driven by wave 0.  Returns false on a
// stack overflow.
template <int FMT>
__device__ bool flood_drive(const Canvas<FMT>& C, int32_t sx, int32_t sy, uint64_t intensity,
                            Frame* stack, int32_t capacity, int32_t* seq, int* parity,
                            BlackStats* bs) {
  const int lane = lane_id();
  int32_t* mb = mailbox();
  Frame top;
  int32_t sp = 0;  // frames on the stack, `top` included; those below it live in stack[0 .. sp-2]
  int32_t nx = sx, ny = sy;
  bool start = true;
  for (;;) {
    if (start) {  // a new frame: save the parent, paint the start, fill the cross
      if (sp >= capacity) return false;  // stack overflow: flagged by the caller
      if (sp > 0 && lane == 0) frame_put(stack_lds(), stack, sp - 1, top);
      // the caller has just read the start pixel as matching (a neighbour
      // check or a bar pixel) and nothing has painted since
      if (lane == 0) C.paint(nx, ny);
      top.x = nx;
      top.y = ny;
      BSTAT(const uint64_t tl = wall_clock64();)
      const bool more = fill_local<FMT>(C, nx, ny, intensity, top.dist, bs);
      BSTAT(bs->t_local += wall_clock64() - tl;)
      if (more) {
        if (lane == 0) {
          mb[2] = nx;
          mb[3] = ny;
        }
        post_command(seq, CMD_FILL);
        fill_coop<FMT>(C, nx, ny, intensity, top.dist, bs);
      }
      top.cursor = 0;
      BSTAT(bs->frames++;)
      sp++;
      start = false;
    }
    const int32_t n = 2 * (top.dist[0] + top.dist[1] + top.dist[2] + top.dist[3]);
    if (top.cursor >= n) {
      if (--sp == 0) return true;
      BSTAT(const uint64_t tq = wall_clock64();)
      top = frame_get(stack_lds(), stack, sp - 1);
      BSTAT(bs->t_pop += wall_clock64() - tq;)
      continue;
    }
    BSTAT(const uint64_t tc = wall_clock64(); bs->check_trips++;)
    int32_t f;
    int32_t span;
    // this wave alone when its 8 slices cover the rest, and for a frame's
    // first window (a new frame's first checks usually start its child)
    if (n - top.cursor <= 64 * kGroup || top.cursor == 0) {
      span = 64 * kGroup;
      const int nsl = imin((n - top.cursor + 63) >> 6, kGroup);  // slices holding checks
      int32_t qx[kGroup], qy[kGroup];
      bool m[kGroup];
#pragma unroll
      for (int i = 0; i < kGroup; i++) {
        qx[i] = -1;
        qy[i] = 0;
        if (i < nsl) {
          const int32_t c = top.cursor + 64 * i + lane;
          check_pos(top, imin(c, n - 1), &qx[i], &qy[i]);
          if (c >= n) qx[i] = -1;
        }
      }
      C.match_group(qx, qy, m);
      // the first match and the one after it: painting only turns pixels
      // white, so checks that did not match now cannot match after the
      // child's fill either, and the frame resumes at the second match (or,
      // with none, is done) without reading its checks again
      f = INT_MAX;
      int32_t f2 = INT_MAX;
#pragma unroll
      for (int i = kGroup - 1; i >= 0; i--) {
        const unsigned long long Mi = __ballot(m[i]);
        if (Mi) {
          const unsigned long long rest = Mi & (Mi - 1);
          f2 = rest ? 64 * i + __ffsll((long long)rest) - 1 : f;
          f = 64 * i + __ffsll((long long)Mi) - 1;
        }
      }
      if (f != INT_MAX) {
        const int32_t cidx = top.cursor + f;
        check_pos(top, cidx, &nx, &ny);
        top.cursor = f2 != INT_MAX ? top.cursor + f2 : imin(n, top.cursor + 64 * nsl);
        BSTAT(bs->t_check += wall_clock64() - tc;)
        start = true;
        continue;
      }
    } else {
      span = 64 * kSlices;
      if (lane == 0) {
        mb[4] = top.x;
        mb[5] = top.y;
        mb[6] = top.dist[0];
        mb[7] = top.dist[1];
        mb[8] = top.dist[2];
        mb[9] = top.dist[3];
        mb[10] = top.cursor;
        mb[11] = n;
      }
      post_command(seq, CMD_CHECK);
      f = check_coop<FMT>(C, top, n, parity, bs);
    }
    BSTAT(bs->t_check += wall_clock64() - tc;)
    if (f == INT_MAX) {
      top.cursor += span;
      continue;
    }
    const int32_t cidx = top.cursor + f;
    check_pos(top, cidx, &nx, &ny);
    top.cursor = cidx + 1;
    start = true;
  }
}

template <int FMT>
__global__ void __launch_bounds__(kThreads) k_black_resolve(PlaneRef img, BlackGeom g,
                                                            const BlackBar* bars,
                                                            uint8_t* scratch, int64_t sstride,
                                                            const int32_t* active,
                                                            SheetCtl* ctl, uint32_t* nbits,
                                                            int64_t nbits_stride) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  const int w = wave_id(), lane = lane_id();
  uint8_t* scr = scratch + s * sstride;
  const uint32_t* hsum = (const uint32_t*)scr;        // W entries
  const uint32_t* vsum = hsum + g.W;                  // H entries
  size_t off = (((size_t)g.W + g.H) * 4 + 255) & ~(size_t)255;
  Frame* stack = (Frame*)(scr + off);
  uint8_t* const base = plane_ptr(img, s);
  BlackStats bstat{};
  BlackStats* bs = &bstat;
  (void)bs;
  const Canvas<FMT> C{base, img.P.pitch, g.W, g.H, g.mask_max,
                      bs, nbits ? nbits + s * nbits_stride : nullptr, (g.W + 31) >> 5};
  BSTAT(const uint64_t t_all = wall_clock64();)
  uint64_t* red = tab_red();
  int parity = 0;
  int32_t seq = 0;  // last command number (driver) / last one seen (helpers)
  if (threadIdx.x == 0) mailbox()[0] = 0;
  block_sync();
  bool dirty = false;
  for (int32_t b0 = 0; b0 < g.nbars; b0 += kThreads) {
    // darkness of kThreads bars on the original image (darkness_rect,
    // blit.c:131-146)
    bool cand = false;
    const int32_t bi = b0 + (int32_t)threadIdx.x;
    if (bi < g.nbars) {
      const BlackBar bb = bars[bi];
      const Rect c = clip(bb.r, g.W, g.H);
      uint64_t sum = 0;
      if (c.x0 <= c.x1 && c.y0 <= c.y1) {
        if (bb.dir == 0)
          for (int32_t x = c.x0; x <= c.x1; x++) sum += hsum[x];
        else
          for (int32_t y = c.y0; y <= c.y1; y++) sum += vsum[y];
      }
      const uint8_t dark = (uint8_t)(0xFFull - sum / count_pixels(c));
      cand = dark >= g.abs_threshold && !bb.excluded;
    }
    const unsigned long long cw = __ballot(cand);
    if (lane == 0) tab_cand()[w] = cw;
    block_sync();
#pragma unroll 1
    for (int v = 0; v < kWaves; v++) {
      uint64_t Mv = tab_cand()[v];
      while (Mv) {
        const int k = __ffsll((long long)Mv) - 1;
        Mv &= Mv - 1;
        const BlackBar bb = bars[b0 + v * 64 + k];
        if (dirty) {  // re-measure on the current image, every thread a share
          BSTAT(const uint64_t tr = wall_clock64(); bs->remeasures++;)
          const Rect c = clip(bb.r, g.W, g.H);
          uint64_t sum = 0;
          if (c.x0 <= c.x1 && c.y0 <= c.y1) {
            for (int32_t x0 = c.x0; x0 <= c.x1; x0 += 64) {
              const int32_t xx = x0 + lane;
              if (xx > c.x1) continue;
              for (int32_t y0 = c.y0 + w * 4; y0 <= c.y1; y0 += 4 * kWaves) {
                uint32_t d[4];
#pragma unroll
                for (int r = 0; r < 4; r++)
                  d[r] = dark_of(load_px_row<FMT>(C.base + (int64_t)imin(y0 + r, c.y1) * C.pitch, xx));
#pragma unroll
                for (int r = 0; r < 4; r++) sum += y0 + r <= c.y1 ? d[r] : 0u;
              }
            }
          }
          sum = wave_sum(sum);
          if (lane == 0) red[w] = sum;
          block_sync();
          uint64_t tot = 0;
#pragma unroll
          for (int v2 = 0; v2 < kWaves; v2++) tot += red[v2];
          block_sync();
          const uint8_t dark = (uint8_t)(0xFFull - tot / count_pixels(c));
          BSTAT(bs->t_remeasure += wall_clock64() - tr;)
          if (dark < g.abs_threshold) continue;
        }
        // flood fill from every pixel of the bar, in scan order
        // (filters.c:81-86): the bar's pixels row-major, a window at a time
        const int32_t bw = bb.r.x1 - bb.r.x0 + 1;
        const int64_t npx = (int64_t)bw * (bb.r.y1 - bb.r.y0 + 1);
        if (bw <= 0 || npx <= 0) continue;
        const int32_t q64 = 64 / bw, r64 = 64 % bw;  // one slice = q64 rows + r64 pixels
        for (int64_t i0 = 0; i0 < npx;) {
          BSTAT(const uint64_t tb = wall_clock64(); bs->bar_trips++;)
          const int64_t i = i0 + 64 * (int64_t)(w * kGroup) + lane;
          int32_t y = bb.r.y0 + (int32_t)(i / bw), x = bb.r.x0 + (int32_t)(i % bw);
          int32_t qx[kGroup], qy[kGroup];
          bool m[kGroup];
#pragma unroll
          for (int k2 = 0; k2 < kGroup; k2++) {
            qx[k2] = i + 64 * k2 < npx ? x : -1;
            qy[k2] = y;
            x += r64;
            y += q64;
            if (x > bb.r.x1) {
              x -= bw;
              y++;
            }
          }
          C.match_group(qx, qy, m);
          uint64_t M[kGroup];
#pragma unroll
          for (int k2 = 0; k2 < kGroup; k2++) M[k2] = __ballot(m[k2]);
          const int32_t f = window_first<false>(M, M, parity++ & 1);
          BSTAT(bs->t_bar += wall_clock64() - tb;)
          if (f == INT_MAX) {
            i0 += 64 * kSlices;
            continue;
          }
          const int64_t hit = i0 + f;
          // wave 0 drives the fill, the others help on its commands
          if (w == 0) {
            const bool ok = flood_drive<FMT>(C, bb.r.x0 + (int32_t)(hit % bw),
                                             bb.r.y0 + (int32_t)(hit / bw), g.intensity, stack,
                                             g.stack_capacity, &seq, &parity, bs);
            if (lane == 0) mailbox()[12] = ok;
            post_command(&seq, CMD_DONE);
          } else {
            flood_help<FMT>(C, g.intensity, &seq, &parity, bs);
          }
          block_sync();  // the fill's paints, and the result, for every wave
          if (!mailbox()[12]) {
            if (threadIdx.x == 0 && ctl) atomicOr(&ctl[s].status, STATUS_FLOOD_OVERFLOW);
            return;
          }
          dirty = true;
          i0 = hit + 1;
        }
      }
    }
    block_sync();  // the candidate table is rewritten by the next chunk
  }
#ifdef UPHIP_DIAG
  if ((g.diag & 16) && threadIdx.x == 0 && bstat.frames)
    printf("uphip black: sheet %d frames %u fill %u (%.1f us) check %u (%.1f us) bar %u (%.1f us) "
           "remeasure %u (%.1f us) total %.1f us lookups %u "
           "fillA %.1f (pos %.1f lookup %.1f) B %.1f C %.1f D %.1f us local %.1f pop %.1f us\n",
           s, bstat.frames, bstat.fill_trips, bstat.t_fill * 0.01, bstat.check_trips,
           bstat.t_check * 0.01, bstat.bar_trips, bstat.t_bar * 0.01, bstat.remeasures,
           bstat.t_remeasure * 0.01, (wall_clock64() - t_all) * 0.01, bstat.lookups * 64,
           bstat.t_fa * 0.01, bstat.t_fa0 * 0.01,
           bstat.t_fa1 * 0.01, bstat.t_fb * 0.01,
           bstat.t_fc * 0.01, bstat.t_fd * 0.01, bstat.t_local * 0.01, bstat.t_pop * 0.01);
#endif
}

template <int FMT>
static void launch_black_t(const PlaneRef& img, const BlackGeom& g, const BlackBar* bars,
                           uint8_t* scr, int64_t ss, const int32_t* active, SheetCtl* ctl,
                           int count, hipStream_t st, const AxisArgs* hargs,
                           const AxisArgs* vargs, bool vsum_ready, uint32_t* nbits,
                           int64_t nbits_stride) {
  // column sums of max(rgb) over the h-stripe rows, row sums over the v-stripe cols
  if (g.hregion.x1 >= g.hregion.x0 && g.hregion.y1 >= g.hregion.y0)
    launch_axis_reduce(img, hargs, 0, M_DARKINV_SUM, g.W, g.H, (uint32_t*)scr, ss / 4, count, st);
  if (g.vregion.x1 >= g.vregion.x0 && g.vregion.y1 >= g.vregion.y0 && !vsum_ready)
    launch_axis_reduce(img, vargs, 1, M_DARKINV_SUM, g.vregion.x1 - g.vregion.x0 + 1, g.H,
                       (uint32_t*)scr + g.W, ss / 4, count, st);
  BlackGeom gd = g;
  gd.diag = diag_noise();
  allow_dynamic_lds((const void*)k_black_resolve<FMT>, kStackLdsBytes);
  if (!(diag_skip() & 1))
    hipLaunchKernelGGL(k_black_resolve<FMT>, dim3(count), dim3(kThreads), kStackLdsBytes, st, img, gd,
                       bars, scr, ss, active, ctl, FMT == F_GRAY8 ? nbits : nullptr, nbits_stride);
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
                             int64_t nbits_stride) {
  uint8_t* scr = (uint8_t*)scratch;
  hipLaunchKernelGGL(k_black_prep, dim3(8, count), dim3(256), 0, st, scr, ss, g.W, count);
  switch (img.P.fmt) {
    case F_GRAY8:
      launch_black_t<F_GRAY8>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs, vsum_ready,
                         nbits, nbits_stride);
      break;
    case F_Y400A:
      launch_black_t<F_Y400A>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs, vsum_ready,
                         nbits, nbits_stride);
      break;
    default:
      launch_black_t<F_RGB24>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs, vsum_ready,
                         nbits, nbits_stride);
      break;
  }
}

}  // namespace uph
