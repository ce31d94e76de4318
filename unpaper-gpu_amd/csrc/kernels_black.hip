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
// HBM, every fill_line and every run of neighbour checks done 64 pixels per
// step with ballots.
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
  int32_t dir;
  int32_t idx;  // next child: 2*d + sub along line `dir`
};

// left, up, right, down (fill.c:92-106)
__constant__ int kDX[4] = {-1, 0, 1, 0};
__constant__ int kDY[4] = {0, -1, 0, 1};

template <int FMT>
struct Canvas {
  uint8_t* base;
  int64_t pitch;
  int32_t W, H;
  uint8_t mmax;  // mask_max (mask_min is 0)
  __device__ __forceinline__ bool inside(int32_t x, int32_t y) const {
    return x >= 0 && y >= 0 && x < W && y < H;
  }
  __device__ __forceinline__ uint8_t gray(int32_t x, int32_t y) const {
    if (!inside(x, y)) return 255;
    return gray_of(load_px_row<FMT>(base + (int64_t)y * pitch, x));
  }
  __device__ __forceinline__ bool match(int32_t x, int32_t y) const { return gray(x, y) <= mmax; }
  // match() as an unconditional load at a clamped position (no divergent
  // branch around the load, so a batch of them is in flight together)
  __device__ __forceinline__ bool match_nb(int32_t x, int32_t y) const {
    const bool in = (x >= 0) & (y >= 0) & (x < W) & (y < H);
    const int32_t cx = imin(imax(x, 0), W - 1), cy = imin(imax(y, 0), H - 1);
    return in & (gray_of(load_px_row<FMT>(base + (int64_t)cy * pitch, cx)) <= mmax);
  }
  __device__ __forceinline__ void paint(int32_t x, int32_t y) const {
    if (inside(x, y)) store_px_row<FMT>(base + (int64_t)y * pitch, x, Px{255, 255, 255});
  }
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

constexpr int kSlices = 8;  // 64-pixel slices evaluated per memory round trip

// fill_line (fill.c:16-52) for one wave: returns the distance painted.  The
// 512 positions of a round are loaded together; they are consumed slice by
// slice in order (a line never revisits its pixels, so painting a slice does
// not change the matches of the next).
template <int FMT>
__device__ int32_t fill_line(const Canvas<FMT>& C, int32_t px, int32_t py, int dir,
                             uint64_t intensity) {
  const int lane = threadIdx.x & 63;
  const int dx = kDX[dir], dy = kDY[dir];
  bool has_last = false;
  int64_t last = 0;  // position of the last matching pixel so far
  for (int64_t pos0 = 1;; pos0 += 64 * kSlices) {
    bool mk[kSlices];
#pragma unroll
    for (int k = 0; k < kSlices; k++) {
      const int64_t j = pos0 + 64 * k + lane;
      mk[k] = C.match_nb(px + (int32_t)(j * dx), py + (int32_t)(j * dy));
    }
#pragma unroll
    for (int k = 0; k < kSlices; k++) {
      const int64_t pos = pos0 + 64 * k, j = pos + lane;
      const int32_t qx = px + (int32_t)(j * dx), qy = py + (int32_t)(j * dy);
      const bool in = C.inside(qx, qy);
      const unsigned long long M = __ballot(mk[k]);
      // last match at or before this lane within the slice
      const unsigned long long upto = M & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
      bool hl = has_last;
      int64_t lm = last;
      if (upto) {
        hl = true;
        lm = pos + (63 - __clzll((long long)upto));
      }
      // counter starts at 1, resets to `intensity` on a match, decrements
      // otherwise; the line stops (unpainted) where it reaches 0 or leaves
      bool stop = !in;
      if (hl) stop |= (uint64_t)(j - lm) >= intensity;
      else stop |= j >= 1;
      const unsigned long long S = __ballot(stop);
      const int first = S ? __ffsll((long long)S) - 1 : 64;
      if (lane < first) C.paint(qx, qy);
      if (S) {
        wave_sync();
        return (int32_t)(pos + first - 1);
      }
      if (M) {
        has_last = true;
        last = pos + (63 - __clzll((long long)M));
      }
    }
    wave_sync();
  }
}

template <int FMT>
__device__ bool frame_start(const Canvas<FMT>& C, int32_t x, int32_t y, uint64_t intensity,
                            Frame* f) {
  // first half of flood_fill (fill.c:81-96)
  if (!C.match(x, y)) return false;
  if ((threadIdx.x & 63) == 0) C.paint(x, y);
  wave_sync();
  f->x = x;
  f->y = y;
  for (int d = 0; d < 4; d++) f->dist[d] = fill_line<FMT>(C, x, y, d, intensity);
  f->dir = 0;
  f->idx = 0;
  return true;
}

// flood_fill (fill.c:81-107) + flood_fill_around_line (fill.c:62-79), one wave.
template <int FMT>
__device__ bool flood_fill(const Canvas<FMT>& C, int32_t sx, int32_t sy, uint64_t intensity,
                           Frame* stack, int32_t capacity, bool* painted) {
  const int lane = threadIdx.x & 63;
  Frame top;
  if (!frame_start<FMT>(C, sx, sy, intensity, &top)) return true;
  *painted = true;
  int32_t sp = 1;  // frames below `top` live in stack[0 .. sp-2]
  while (sp > 0) {
    while (top.dir < 4 && top.idx >= 2 * top.dist[top.dir]) {
      top.dir++;
      top.idx = 0;
    }
    if (top.dir >= 4) {
      sp--;
      if (sp > 0) top = stack[sp - 1];
      continue;
    }
    const int dx = kDX[top.dir], dy = kDY[top.dir];
    const int32_t n = 2 * top.dist[top.dir];
    // the next 512 neighbour checks of the line in one round trip; the first
    // match (in order) starts the child frame, later ones are re-read after it
    bool mk[kSlices];
#pragma unroll
    for (int k = 0; k < kSlices; k++) {
      const int32_t c = top.idx + 64 * k + lane;
      const int32_t d = c >> 1, sub = c & 1;
      int32_t qx = top.x + (d + 1) * dx, qy = top.y + (d + 1) * dy;
      if (dx != 0) qy += sub == 0 ? 1 : -1;  // below, then above
      else qx += sub == 0 ? 1 : -1;           // right, then left
      mk[k] = (c < n) & C.match_nb(qx, qy);
    }
    int kf = -1;
    unsigned long long M = 0;
#pragma unroll
    for (int k = kSlices - 1; k >= 0; k--) {
      const unsigned long long b = __ballot(mk[k]);
      if (b) {
        kf = k;
        M = b;
      }
    }
    if (kf < 0) {
      top.idx += 64 * kSlices;
      continue;
    }
    const int first = __ffsll((long long)M) - 1;
    const int32_t cidx = top.idx + 64 * kf + first;
    int32_t cx, cy;
    {
      const int32_t d = cidx >> 1, sub = cidx & 1;
      cx = top.x + (d + 1) * dx;
      cy = top.y + (d + 1) * dy;
      if (dx != 0) cy += sub == 0 ? 1 : -1;
      else cx += sub == 0 ? 1 : -1;
    }
    top.idx = cidx + 1;
    if (sp >= capacity) return false;  // stack overflow: flagged by the caller
    Frame child;
    if (frame_start<FMT>(C, cx, cy, intensity, &child)) {
      if (lane == 0) stack[sp - 1] = top;
      wave_sync();
      top = child;
      sp++;
    }
  }
  return true;
}

template <int FMT>
__global__ void __launch_bounds__(64) k_black_resolve(PlaneRef img, BlackGeom g,
                                                      const BlackBar* bars, uint8_t* scratch,
                                                      int64_t sstride, const int32_t* active,
                                                      SheetCtl* ctl) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  const int lane = threadIdx.x;
  uint8_t* scr = scratch + s * sstride;
  const uint32_t* hsum = (const uint32_t*)scr;        // W entries
  const uint32_t* vsum = hsum + g.W;                  // H entries
  size_t off = (((size_t)g.W + g.H) * 4 + 255) & ~(size_t)255;
  Frame* stack = (Frame*)(scr + off);
  Canvas<FMT> C{plane_ptr(img, s), img.P.pitch, g.W, g.H, g.mask_max};
  bool dirty = false;
  for (int32_t b0 = 0; b0 < g.nbars; b0 += 64) {
    // darkness of 64 bars on the original image (darkness_rect, blit.c:131-146)
    bool cand = false;
    const int32_t bi = b0 + lane;
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
    unsigned long long M = __ballot(cand);
    while (M) {
      const int k = __ffsll((long long)M) - 1;
      M &= M - 1;
      const BlackBar bb = bars[b0 + k];
      if (dirty) {  // re-measure on the current image
        const Rect c = clip(bb.r, g.W, g.H);
        uint64_t sum = 0;
        if (c.x0 <= c.x1 && c.y0 <= c.y1) {
          const int32_t w = c.x1 - c.x0 + 1;
          const int64_t npx = (int64_t)w * (c.y1 - c.y0 + 1);
          for (int64_t i = lane; i < npx; i += 64) {
            const int32_t yy = c.y0 + (int32_t)(i / w), xx = c.x0 + (int32_t)(i % w);
            sum += dark_of(load_px_row<FMT>(C.base + (int64_t)yy * C.pitch, xx));
          }
        }
        for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o, 64);
        sum = __shfl(sum, 0, 64);
        const uint8_t dark = (uint8_t)(0xFFull - sum / count_pixels(c));
        if (dark < g.abs_threshold) continue;
      }
      // flood fill from every pixel of the bar, in scan order (filters.c:81-86)
      for (int32_t y = bb.r.y0; y <= bb.r.y1; y++) {
        for (int32_t x0 = bb.r.x0; x0 <= bb.r.x1; x0 += 64) {
          int32_t from = 0;
          for (;;) {
            const int32_t x = x0 + from + lane;
            const bool m = (from + lane) < 64 && x <= bb.r.x1 && C.match(x, y);
            const unsigned long long S = __ballot(m);
            if (!S) break;
            const int f = __ffsll((long long)S) - 1;
            bool painted = false;
            if (!flood_fill<FMT>(C, x0 + f, y, g.intensity, stack, g.stack_capacity,
                                 &painted)) {
              if (lane == 0 && ctl) atomicOr(&ctl[s].status, STATUS_FLOOD_OVERFLOW);
              return;
            }
            dirty |= painted;
            from = f + 1;
            if (from >= 64) break;
          }
        }
      }
    }
  }
}

template <int FMT>
static void launch_black_t(const PlaneRef& img, const BlackGeom& g, const BlackBar* bars,
                           uint8_t* scr, int64_t ss, const int32_t* active, SheetCtl* ctl,
                           int count, hipStream_t st, const AxisArgs* hargs,
                           const AxisArgs* vargs) {
  // column sums of max(rgb) over the h-stripe rows, row sums over the v-stripe cols
  if (g.hregion.x1 >= g.hregion.x0 && g.hregion.y1 >= g.hregion.y0)
    launch_axis_reduce(img, hargs, 0, M_DARKINV_SUM, g.W, g.H, (uint32_t*)scr, ss / 4, count, st);
  if (g.vregion.x1 >= g.vregion.x0 && g.vregion.y1 >= g.vregion.y0)
    launch_axis_reduce(img, vargs, 1, M_DARKINV_SUM, g.vregion.x1 - g.vregion.x0 + 1, g.H,
                       (uint32_t*)scr + g.W, ss / 4, count, st);
  if (!(diag_skip() & 1)) hipLaunchKernelGGL(k_black_resolve<FMT>, dim3(count), dim3(64), 0, st, img, g, bars, scr, ss,
                     active, ctl);
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
                             const AxisArgs* vargs) {
  uint8_t* scr = (uint8_t*)scratch;
  hipLaunchKernelGGL(k_black_prep, dim3(8, count), dim3(256), 0, st, scr, ss, g.W, count);
  switch (img.P.fmt) {
    case F_GRAY8:
      launch_black_t<F_GRAY8>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs);
      break;
    case F_Y400A:
      launch_black_t<F_Y400A>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs);
      break;
    default:
      launch_black_t<F_RGB24>(img, g, bars, scr, ss, active, ctl, count, st, hargs, vargs);
      break;
  }
}

}  // namespace uph
