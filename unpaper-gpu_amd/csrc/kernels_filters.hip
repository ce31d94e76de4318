// kernels_filters.hip — grayfilter, blurfilter and noisefilter for gfx950.
//
// All three are raster-order scans in the reference whose later decisions can
// depend on earlier writes.  Each is split into (1) one streaming pass that
// computes every decision input in parallel on the unmodified image and (2) an
// exact resolution of the order dependence on small per-sheet data, proven
// equivalent to the sequential scan (DESIGN.md §Order-dependent scans).
#include <climits>

#include "filters.h"

namespace uph {

__host__ __device__ static inline int32_t gcd_i(int32_t a, int32_t b) {
  a = a < 0 ? -a : a;
  b = b < 0 ? -b : b;
  while (b) {
    int32_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

template <int FMT>
__device__ __forceinline__ void white_px(uint8_t* row, int32_t x) {
  store_px_row<FMT>(row, x, Px{255, 255, 255});
}

// =========================================================================
// GRAYFILTER (filters.c:370-402)
//   tile T at (i*sx, j*sy), visited x-fastest for x = 0.. first x >= W and
//   y = 0.. <= H.  T is wiped iff it holds no pixel with gray <= black_thr and
//   255 - lightness_sum/count(clip T) < abs_thr, evaluated on the image as
//   left by the wipes of EARLIER tiles.  A wipe never changes a dark count
//   (wiped tiles had none) and only raises lightness, so T's predicate is
//   monotone in the set of earlier wipes.  The exact result is the unique
//   fixed point of "wiped(T) = pred(T, {earlier wiped})", reached by Jacobi
//   iteration from the tiles that pass on the original image.
// =========================================================================
bool gray_geometry(int32_t W, int32_t H, const UphipGrayfilterParameters& p, uint8_t black_thr,
                   GrayGeom* g) {
  if (p.scan_size.width <= 0 || p.scan_size.height <= 0 || p.scan_step.horizontal <= 0 ||
      p.scan_step.vertical <= 0)
    return false;
  g->W = W;
  g->H = H;
  g->scan_w = p.scan_size.width;
  g->scan_h = p.scan_size.height;
  g->step_x = p.scan_step.horizontal;
  g->step_y = p.scan_step.vertical;
  g->cw = gcd_i(g->step_x, g->scan_w);
  g->ch = gcd_i(g->step_y, g->scan_h);
  g->ncx = (W + g->cw - 1) / g->cw;
  g->ncy = (H + g->ch - 1) / g->ch;
  g->tw = g->scan_w / g->cw;
  g->th = g->scan_h / g->ch;
  g->tsx = g->step_x / g->cw;
  g->tsy = g->step_y / g->ch;
  // x = 0, sx, ... up to and including the first value >= W (filters.c:392-399)
  g->ntx = (W + g->step_x - 1) / g->step_x + 1;
  g->nty = H / g->step_y + 1;  // y = 0.. <= H
  g->black_thr = black_thr;
  g->abs_thr = p.abs_threshold;
  return true;
}

size_t gray_scratch_bytes(const GrayGeom& g) {
  const size_t cells = (size_t)g.ncx * g.ncy;
  const size_t tiles = (size_t)g.ntx * g.nty;
  size_t b = cells * 8 + tiles;  // dark+light (2 x u32), tile state
  b = (b + 3) & ~(size_t)3;
  b += 4;                        // undecided-tile counter
  return (b + 255) & ~(size_t)255;
}

struct GrayPtrs {
  uint32_t* dark;
  uint32_t* light;
  uint8_t* tile;     // 0 = never, 1 = undecided, 2 = wiped (3 = newly wiped, transient)
  uint32_t* nund;    // undecided tiles
};
__device__ __forceinline__ GrayPtrs gray_ptrs(const GrayGeom& g, uint8_t* base) {
  const size_t cells = (size_t)g.ncx * g.ncy;
  const size_t tiles = (size_t)g.ntx * g.nty;
  GrayPtrs p;
  p.dark = (uint32_t*)base;
  p.light = p.dark + cells;
  p.tile = (uint8_t*)(p.light + cells);
  p.nund = (uint32_t*)(base + ((cells * 8 + tiles + 3) & ~(size_t)3));
  return p;
}

template <int FMT>
__global__ void __launch_bounds__(256) k_gray_cells(PlaneRef img, GrayGeom g, uint8_t* scratch,
                                                    int64_t sstride, const int32_t* active) {
  const int s = blockIdx.z;
  if (active && !active[s]) return;
  const int32_t cx = blockIdx.x * 256 + threadIdx.x, cy = blockIdx.y;
  GrayPtrs P = gray_ptrs(g, scratch + s * sstride);
  if (cx == 0 && cy == 0) *P.nund = 0;
  if (cx >= g.ncx) return;
  const uint8_t* base = plane_ptr(img, s);
  const int32_t x0 = cx * g.cw, x1 = imin(x0 + g.cw, g.W);
  const int32_t y0 = cy * g.ch, y1 = imin(y0 + g.ch, g.H);
  uint32_t dark = 0, light = 0;
  for (int32_t y = y0; y < y1; y++) {
    const uint8_t* row = base + (int64_t)y * img.P.pitch;
    for (int32_t x = x0; x < x1; x++) {
      Px p = load_px_row<FMT>(row, x);
      dark += gray_of(p) <= g.black_thr ? 1u : 0u;
      light += light_of(p);
    }
  }
  const size_t c = (size_t)cy * g.ncx + cx;
  P.dark[c] = dark;
  P.light[c] = light;
}

// k_gray_cells for a gray plane: one workgroup per kGrayStrips strips of cell
// rows, a lane per 8-byte column group (the block is as wide as a row's
// groups, so nearly every lane has one).  A lane adds its columns over the
// strip's rows as 16-bit lanes of four words (bytes 0/2 and 1/3 of each
// dword), counting bytes above the dark threshold as bit 8 of byte + 256 -
// (thr+1) (ch <= 255 keeps both in 16 bits), and posts the 16-bit column
// totals to LDS; then one lane per cell adds its cw columns.
// With `colsum`, the block's strips also add up per-column gray sums over all
// rows: the sums the next mask scan takes (detect_mask, masks.c:54-100, on
// the image the grayfilter leaves; k_gray_wipe adds what its wipes change), so
// that scan needs no pass of its own.  kGrayStrips strips per block keep the
// atomics at W per kGrayStrips * ch rows.
#ifndef UPH_GRAY_ROWS
#define UPH_GRAY_ROWS 1  // k_gray_tiles_rows (0: a thread per tile reading its cells)
#endif
constexpr int kGrayStripMaxW = 16384;
constexpr int kGrayStrips = 8;
constexpr int kGrayMaxCh = 255;
__global__ void __launch_bounds__(1024) k_gray_cells_g(PlaneRef img, GrayGeom g, uint8_t* scratch,
                                                       int64_t sstride, const int32_t* active,
                                                       uint32_t* colsum, int64_t colsum_stride) {
  const int s = blockIdx.z;
  if (active && !active[s]) return;
  GrayPtrs P = gray_ptrs(g, scratch + s * sstride);
  if (blockIdx.x == 0 && threadIdx.x == 0) *P.nund = 0;
  const uint8_t* base = plane_ptr(img, s);
  const int64_t pitch = img.P.pitch;
  // [wq] dark counts, [wq] lightness sums (u16), then [W] u32 totals
  extern __shared__ __attribute__((aligned(16))) uint16_t cols16[];
  const int32_t wq = (g.W + 7) & ~7;
  uint16_t* cdark = cols16;
  uint16_t* clight = cols16 + wq;
  uint32_t* ctot = reinterpret_cast<uint32_t*>(cols16 + 2 * wq);
  if (colsum)
    for (int32_t x = threadIdx.x; x < g.W; x += blockDim.x) ctot[x] = 0;
  const int32_t n8 = (g.W + 7) >> 3;
  const uint32_t kadd = (256u - ((uint32_t)g.black_thr + 1u)) * 0x00010001u;
  const int32_t cy_end = imin((int32_t)(blockIdx.x + 1) * kGrayStrips, g.ncy);
  for (int32_t cy = blockIdx.x * kGrayStrips; cy < cy_end; cy++) {
    const int32_t y0 = cy * g.ch, y1 = imin(y0 + g.ch, g.H);
    for (int32_t d = threadIdx.x; d < n8; d += blockDim.x) {
      // words: bytes 0/2 and 1/3 of the group's dword 0, then of dword 1
      uint32_t l[4] = {0, 0, 0, 0}, ge[4] = {0, 0, 0, 0};
      auto add = [&](uint2 v) {
        const uint32_t w[4] = {v.x & 0x00FF00FFu, (v.x >> 8) & 0x00FF00FFu, v.y & 0x00FF00FFu,
                               (v.y >> 8) & 0x00FF00FFu};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          l[j] += w[j];
          ge[j] += (w[j] + kadd) & 0x01000100u;
        }
      };
      const uint8_t* p = base + (int64_t)y0 * pitch + 8 * d;
      int32_t y = y0;
      for (; y + 4 <= y1; y += 4, p += 4 * pitch) {
        uint2 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = *reinterpret_cast<const uint2*>(p + k * pitch);
#pragma unroll
        for (int k = 0; k < 4; k++) add(v[k]);
      }
      for (; y < y1; y++, p += pitch) add(*reinterpret_cast<const uint2*>(p));
      const uint32_t rows2 = (uint32_t)(y1 - y0) * 0x00010001u;
      uint32_t dk[4];
#pragma unroll
      for (int j = 0; j < 4; j++) dk[j] = rows2 - (ge[j] >> 8);
      // columns 8d + 4k + b sit in word 2k + (b & 1), half b >> 1
      const uint32_t sel_lo = 0x05040100u, sel_hi = 0x07060302u;  // (a.lo, b.lo), (a.hi, b.hi)
      const uint4 dv = make_uint4(__builtin_amdgcn_perm(dk[1], dk[0], sel_lo),
                                  __builtin_amdgcn_perm(dk[1], dk[0], sel_hi),
                                  __builtin_amdgcn_perm(dk[3], dk[2], sel_lo),
                                  __builtin_amdgcn_perm(dk[3], dk[2], sel_hi));
      const uint4 lv = make_uint4(__builtin_amdgcn_perm(l[1], l[0], sel_lo),
                                  __builtin_amdgcn_perm(l[1], l[0], sel_hi),
                                  __builtin_amdgcn_perm(l[3], l[2], sel_lo),
                                  __builtin_amdgcn_perm(l[3], l[2], sel_hi));
      *reinterpret_cast<uint4*>(cdark + 8 * d) = dv;
      *reinterpret_cast<uint4*>(clight + 8 * d) = lv;
    }
    __syncthreads();
    for (int32_t cx = threadIdx.x; cx < g.ncx; cx += blockDim.x) {
      const int32_t x0 = cx * g.cw, x1 = imin(x0 + g.cw, g.W);
      uint32_t dark = 0, light = 0;
      for (int32_t x = x0; x < x1; x++) {
        dark += cdark[x];
        light += clight[x];
      }
      const size_t c = (size_t)cy * g.ncx + cx;
      P.dark[c] = dark;
      P.light[c] = light;
    }
    if (colsum)
      for (int32_t x = threadIdx.x; x < g.W; x += blockDim.x) ctot[x] += clight[x];
    __syncthreads();  // the next strip rewrites the column tables
  }
  if (colsum) {
    uint32_t* out = colsum + (int64_t)s * colsum_stride;
    for (int32_t x = threadIdx.x; x < g.W; x += blockDim.x)
      if (ctot[x]) atomicAdd(out + x, ctot[x]);
  }
}

__device__ __forceinline__ uint32_t cell_pixels(const GrayGeom& g, int32_t cx, int32_t cy) {
  const int32_t w = imin((cx + 1) * g.cw, g.W) - cx * g.cw;
  const int32_t h = imin((cy + 1) * g.ch, g.H) - cy * g.ch;
  return (w > 0 && h > 0) ? (uint32_t)(w * h) : 0u;
}

// inverse_lightness_rect of tile (tx,ty) on the original image, the cells'
// lightness sums from light(cx, cy)
template <class Light>
__device__ __forceinline__ uint8_t gray_tile_inv0(const GrayGeom& g, int32_t tx, int32_t ty,
                                                  Light light) {
  const Rect r = clip(rect_from_size(tx * g.step_x, ty * g.step_y, g.scan_w, g.scan_h), g.W, g.H);
  const uint64_t count = count_pixels(r);
  uint64_t sum = 0;
  const int32_t cx0 = tx * g.tsx, cy0 = ty * g.tsy;
  for (int32_t j = 0; j < g.th; j++) {
    const int32_t cy = cy0 + j;
    if (cy >= g.ncy) break;
    for (int32_t i = 0; i < g.tw; i++) {
      const int32_t cx = cx0 + i;
      if (cx >= g.ncx) break;
      sum += light(cx, cy);
    }
  }
  if (r.x1 < r.x0 || r.y1 < r.y0) sum = 0;  // loop body never runs
  return (uint8_t)(0xFFull - sum / count);
}

// inverse_lightness_rect of tile (tx,ty) with wiped cells reading 255.
// mode 0: original image; mode 1: cells covered by an EARLIER wiped tile are white.
__device__ uint8_t gray_tile_inv(const GrayGeom& g, const GrayPtrs& P, int32_t tx, int32_t ty,
                                 int mode) {
  const Rect r = clip(rect_from_size(tx * g.step_x, ty * g.step_y, g.scan_w, g.scan_h), g.W, g.H);
  const uint64_t count = count_pixels(r);
  uint64_t sum = 0;
  const int32_t cx0 = tx * g.tsx, cy0 = ty * g.tsy;
  for (int32_t j = 0; j < g.th; j++) {
    const int32_t cy = cy0 + j;
    if (cy >= g.ncy) break;
    for (int32_t i = 0; i < g.tw; i++) {
      const int32_t cx = cx0 + i;
      if (cx >= g.ncx) break;
      const size_t c = (size_t)cy * g.ncx + cx;
      bool white = false;
      if (mode) {
        // tiles covering cell (cx,cy) that precede (tx,ty) and are wiped
        for (int32_t oy = cy - g.th + 1; oy <= cy && !white; oy++) {
          if (oy < 0 || oy % g.tsy) continue;
          const int32_t uy = oy / g.tsy;
          if (uy >= g.nty || uy > ty) continue;
          for (int32_t ox = cx - g.tw + 1; ox <= cx; ox++) {
            if (ox < 0 || ox % g.tsx) continue;
            const int32_t ux = ox / g.tsx;
            if (ux >= g.ntx) continue;
            if (uy == ty && ux >= tx) continue;
            if (P.tile[(size_t)uy * g.ntx + ux] == 2) {
              white = true;
              break;
            }
          }
        }
      }
      sum += white ? 255u * cell_pixels(g, cx, cy) : P.light[c];
    }
  }
  if (r.x1 < r.x0 || r.y1 < r.y0) sum = 0;  // loop body never runs
  return (uint8_t)(0xFFull - sum / count);
}

// Whether cell (cx, cy) lies in a wiped tile (2): the tiles covering it are
// ux in [ceil((cx - tw + 1) / tsx), cx / tsx], likewise uy.
__device__ __forceinline__ bool gray_cell_wiped(const GrayGeom& g, const uint8_t* tile, int32_t cx,
                                                int32_t cy) {
  const int32_t uy0 = imax(0, (cy - g.th + g.tsy) / g.tsy), uy1 = imin(cy / g.tsy, g.nty - 1);
  const int32_t ux0 = imax(0, (cx - g.tw + g.tsx) / g.tsx), ux1 = imin(cx / g.tsx, g.ntx - 1);
  for (int32_t uy = uy0; uy <= uy1; uy++)
    for (int32_t ux = ux0; ux <= ux1; ux++)
      if (tile[(size_t)uy * g.ntx + ux] == 2) return true;
  return false;
}

// Every tile decided on the original image, one thread per tile: tiles with
// a dark pixel never wipe; tiles light enough on the original always wipe
// (wipes only brighten); the rest are undecided and counted.
__global__ void __launch_bounds__(256) k_gray_tiles(GrayGeom g, uint8_t* scratch, int64_t sstride,
                                                    const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  GrayPtrs P = gray_ptrs(g, scratch + s * sstride);
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  const int32_t ntiles = g.ntx * g.nty;
  bool und = false;
  if (t < ntiles) {
    const int32_t tx = t % g.ntx, ty = t / g.ntx;
    uint32_t dark = 0;
    for (int32_t j = 0; j < g.th; j++) {
      const int32_t cy = ty * g.tsy + j;
      if (cy >= g.ncy) break;
      for (int32_t i = 0; i < g.tw; i++) {
        const int32_t cx = tx * g.tsx + i;
        if (cx >= g.ncx) break;
        dark += P.dark[(size_t)cy * g.ncx + cx];
      }
    }
    uint8_t st = 0;
    if (dark == 0) {
      st = gray_tile_inv(g, P, tx, ty, 0) < g.abs_thr ? 2 : 1;
      und = st == 1;
    }
    P.tile[t] = st;
  }
  const unsigned long long M = __ballot(und);
  if (M && (threadIdx.x & 63) == __ffsll((long long)M) - 1) atomicAdd(P.nund, (uint32_t)__popcll(M));
}

// k_gray_tiles with a workgroup per tile row: the th cell rows it covers
// (dark counts and lightness sums) staged in LDS once instead of every tile
// reading its tw x th cells from the scratch (the host takes it when those
// rows fit kGrayRowLds).
constexpr int kGrayRowLds = 32 * 1024;
__global__ void __launch_bounds__(256) k_gray_tiles_rows(GrayGeom g, uint8_t* scratch, int64_t sstride,
                                                         const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  GrayPtrs P = gray_ptrs(g, scratch + s * sstride);
  const int32_t ty = blockIdx.x, cy0 = ty * g.tsy;
  const int32_t nr = imax(0, imin(g.th, g.ncy - cy0));  // cell rows inside the image
  extern __shared__ uint32_t gcl[];
  uint32_t* sd = gcl;                 // [nr][ncx] dark
  uint32_t* sl = gcl + nr * g.ncx;    // [nr][ncx] light
  for (int32_t i = threadIdx.x; i < nr * g.ncx; i += 256) {
    const size_t c = (size_t)cy0 * g.ncx + i;  // rows cy0.. are consecutive
    sd[i] = P.dark[c];
    sl[i] = P.light[c];
  }
  __syncthreads();
  bool und_any = false;
  for (int32_t tx = threadIdx.x; tx - (int32_t)threadIdx.x < g.ntx; tx += 256) {
    bool und = false;
    if (tx < g.ntx) {
      const int32_t cx0 = tx * g.tsx;
      uint32_t dark = 0;
      for (int32_t j = 0; j < nr; j++)
        for (int32_t i = 0; i < g.tw && cx0 + i < g.ncx; i++) dark += sd[j * g.ncx + cx0 + i];
      uint8_t st = 0;
      if (dark == 0) {
        const uint8_t inv = gray_tile_inv0(g, tx, ty, [&](int32_t cx, int32_t cy) {
          return sl[(cy - cy0) * g.ncx + cx];
        });
        st = inv < g.abs_thr ? 2 : 1;
        und = st == 1;
      }
      P.tile[(size_t)ty * g.ntx + tx] = st;
    }
    const unsigned long long M = __ballot(und);
    if (M && (threadIdx.x & 63) == __ffsll((long long)M) - 1) atomicAdd(P.nund, (uint32_t)__popcll(M));
    und_any |= und;
  }
  (void)und_any;
}

// The wipe feedback: Jacobi sweeps over the undecided tiles until nothing
// changes (one block per sheet; returns at once when none is undecided).
__global__ void __launch_bounds__(1024) k_gray_decide(GrayGeom g, uint8_t* scratch, int64_t sstride,
                                                      const int32_t* active) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  GrayPtrs P = gray_ptrs(g, scratch + s * sstride);
  if (*P.nund == 0) return;
  const int32_t ntiles = g.ntx * g.nty;
  __shared__ int32_t changed;
  for (int iter = 0; iter < ntiles + 1; iter++) {
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    for (int32_t t = threadIdx.x; t < ntiles; t += blockDim.x) {
      if (P.tile[t] != 1) continue;
      const int32_t tx = t % g.ntx, ty = t / g.ntx;
      if (gray_tile_inv(g, P, tx, ty, 1) < g.abs_thr) {
        P.tile[t] = 3;
        changed = 1;
      }
    }
    __threadfence_block();
    __syncthreads();
    if (!changed) break;
    for (int32_t t = threadIdx.x; t < ntiles; t += blockDim.x)
      if (P.tile[t] == 3) P.tile[t] = 2;
    __threadfence_block();
    __syncthreads();
  }
}

template <int FMT>
__global__ void __launch_bounds__(256) k_gray_wipe(PlaneRef img, GrayGeom g, uint8_t* scratch,
                                                   int64_t sstride, const int32_t* active,
                                                   uint32_t* colsum, int64_t colsum_stride) {
  const int s = blockIdx.z;
  if (active && !active[s]) return;
  const int32_t cx = blockIdx.x * 256 + threadIdx.x, cy = blockIdx.y;
  if (cx >= g.ncx) return;
  GrayPtrs P = gray_ptrs(g, scratch + s * sstride);
  // a cell whose lightness sum is all white is white already (Y400A wipes
  // also set alpha, so its cells are always written): one load decides the
  // blank paper before the covering tiles' states are read
  if (FMT != F_Y400A && P.light[(size_t)cy * g.ncx + cx] == 255u * cell_pixels(g, cx, cy)) return;
  if (!gray_cell_wiped(g, P.tile, cx, cy)) return;
  uint8_t* base = plane_ptr(img, s);
  const int32_t x0 = cx * g.cw, x1 = imin(x0 + g.cw, g.W);
  const int32_t y0 = cy * g.ch, y1 = imin(y0 + g.ch, g.H);
  if (FMT == F_GRAY8 && colsum) {
    // the column gray sums (k_gray_cells_g) follow the wipe: + (255 - old)
    uint32_t* out = colsum + (int64_t)s * colsum_stride;
    for (int32_t x = x0; x < x1; x++) {
      uint32_t add = 0;
      for (int32_t y = y0; y < y1; y++) add += 255u - base[(int64_t)y * img.P.pitch + x];
      if (add) atomicAdd(out + x, add);
    }
  }
  for (int32_t y = y0; y < y1; y++) {
    uint8_t* row = base + (int64_t)y * img.P.pitch;
    for (int32_t x = x0; x < x1; x++) white_px<FMT>(row, x);
  }
}

template <int FMT>
static bool launch_gray_t(const PlaneRef& img, const GrayGeom& g, uint8_t* scr, int64_t ss,
                          const int32_t* active, int count, hipStream_t st, uint32_t* colsum,
                          int64_t cs) {
  dim3 grid((g.ncx + 255) / 256, g.ncy, count);
  const bool strips = FMT == F_GRAY8 && g.W <= kGrayStripMaxW && g.ch <= kGrayMaxCh;
  if (!strips) colsum = nullptr;
  if (strips) {
    const size_t wq = (size_t)((g.W + 7) & ~7);
    // a lane per 8-byte column group, up to 1024
    const int n8 = (g.W + 7) >> 3;
    const int threads = imin(1024, (n8 + 63) & ~63);
    UPH_LAUNCH_DIAG(32, k_gray_cells_g, dim3((g.ncy + kGrayStrips - 1) / kGrayStrips, 1, count),
                    dim3(threads), 4 * wq + (colsum ? 4 * (size_t)g.W : 0), st, img, g, scr, ss,
                    active, colsum, cs);
  } else {
    hipLaunchKernelGGL(k_gray_cells<FMT>, grid, dim3(256), 0, st, img, g, scr, ss, active);
  }
  const int32_t ntiles = g.ntx * g.nty;
  const size_t rows_lds = 2 * sizeof(uint32_t) * (size_t)g.th * g.ncx;
  if (UPH_GRAY_ROWS && rows_lds <= (size_t)kGrayRowLds)
    hipLaunchKernelGGL(k_gray_tiles_rows, dim3(g.nty, count), dim3(256), rows_lds, st, g, scr, ss, active);
  else
    hipLaunchKernelGGL(k_gray_tiles, dim3((ntiles + 255) / 256, count), dim3(256), 0, st, g, scr, ss,
                       active);
  if (!(diag_skip() & 4)) hipLaunchKernelGGL(k_gray_decide, dim3(count), dim3(1024), 0, st, g, scr, ss, active);
  hipLaunchKernelGGL(k_gray_wipe<FMT>, grid, dim3(256), 0, st, img, g, scr, ss, active, colsum, cs);
  return colsum != nullptr;
}

bool launch_grayfilter(const PlaneRef& img, const GrayGeom& g, void* scratch,
                       int64_t scratch_stride, const int32_t* active, int count, hipStream_t st,
                       uint32_t* colsum, int64_t colsum_stride) {
  uint8_t* scr = (uint8_t*)scratch;
  switch (img.P.fmt) {
    case F_GRAY8:
      return launch_gray_t<F_GRAY8>(img, g, scr, scratch_stride, active, count, st, colsum,
                                    colsum_stride);
    case F_Y400A:
      return launch_gray_t<F_Y400A>(img, g, scr, scratch_stride, active, count, st, nullptr, 0);
    default:
      return launch_gray_t<F_RGB24>(img, g, scr, scratch_stride, active, count, st, nullptr, 0);
  }
}

// =========================================================================
// BLURFILTER (filters.c:149-232)
//   Every count the reference takes is of the unmodified image (no wipe ever
//   overlaps a rectangle counted later), so all counts are computed in
//   parallel; the reference's three count rows are pointers into ONE row of
//   its VLA at offsets 0/1/2 that rotate every row, so the wipe decisions are
//   the literal pointer recurrence replayed by one lane over those counts.
//   The slot read before it is written (prev[0] on the first row, an
//   uninitialised stack value in the reference) is 0 here.
// =========================================================================
bool blur_geometry(int32_t W, int32_t H, const UphipBlurfilterParameters& p, uint8_t white,
                   BlurGeom* g) {
  if (p.scan_size.width <= 0 || p.scan_size.height <= 0) return false;
  g->W = W;
  g->H = H;
  g->sw = p.scan_size.width;
  g->sh = p.scan_size.height;
  g->step_y = p.scan_step.vertical;
  g->bpr = (int32_t)((uint32_t)(W / g->sw));
  g->T = H >= g->sh ? (H - g->sh) / g->sh + 1 : 0;
  g->nrect = g->bpr + g->T * (g->bpr + 1);
  g->white = white;
  g->intensity = p.intensity;
  return true;
}

size_t blur_scratch_bytes(const BlurGeom& g) {
  size_t b = (size_t)g.nrect * 4 + (size_t)g.T * (g.bpr > 0 ? g.bpr : 1);
  return (b + 255) & ~(size_t)255;
}

__device__ __forceinline__ void blur_rect_origin(const BlurGeom& g, int32_t r, int32_t* x,
                                                 int32_t* y) {
  if (r < g.bpr) {
    *x = r * g.sw;
    *y = 0;
  } else {
    const int32_t q = r - g.bpr, t = q / (g.bpr + 1), j = q % (g.bpr + 1);
    *x = j * g.sw;
    *y = t * g.sh + g.step_y;
  }
}

// k_blur_counts for a gray plane: one workgroup per row of rectangles (the
// first row at y = 0, row t at step_y + t*sh).  Lanes count dark pixels
// (gray <= white) of aligned dwords over the strip's rows into per-column
// 16-bit totals in LDS, then one lane per rectangle adds its sw columns.
// V16: 16-byte loads, 16 columns a lane (A/B 146.5 -> 140.6 us a launch
// against 4-byte loads); the host takes it only for planes whose bases,
// stride and pitch are 16-byte aligned with pitch >= round16(W), so the last
// vector of a row stays inside the row.
template <bool V16>
__global__ void __launch_bounds__(256) k_blur_counts_g(PlaneRef img, BlurGeom g, uint8_t* scratch,
                                                       int64_t sstride, const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  const int32_t row = blockIdx.x;  // 0: the top row of rectangles, 1 + t: row t
  const int32_t ry = row == 0 ? 0 : (row - 1) * g.sh + g.step_y;
  const int32_t y0 = imax(ry, 0), y1 = imin(ry + g.sh, g.H);  // [y0, y1)
  const uint8_t* base = plane_ptr(img, s);
  extern __shared__ uint16_t ccount[];
  // V16: a lane counts 16 columns, 8 rows' loads in flight
  const int32_t nv = V16 ? (g.W + 15) >> 4 : 0;
  for (int32_t vi = threadIdx.x; vi < nv; vi += 256) {
    uint32_t c[16];
#pragma unroll
    for (int j = 0; j < 16; j++) c[j] = 0;
    for (int32_t y = y0; y < y1; y += 8) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; k++)
        v[k] = *reinterpret_cast<const uint4*>(base + (int64_t)imin(y + k, y1 - 1) * img.P.pitch + 16 * vi);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t keep = y + k < y1 ? 1u : 0u;
        const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
          for (int j = 0; j < 4; j++) c[4 * q + j] += keep & (((w4[q] >> (8 * j)) & 0xFF) <= g.white ? 1u : 0u);
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j++)
      if (16 * vi + j < g.W) ccount[16 * vi + j] = (uint16_t)c[j];
  }
  const int32_t nd = V16 ? 0 : (g.W + 3) >> 2;
  for (int32_t d = threadIdx.x; d < nd; d += 256) {
    uint32_t c[4] = {0, 0, 0, 0};
    for (int32_t y = y0; y < y1; y += 8) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; k++)
        v[k] = *reinterpret_cast<const uint32_t*>(base + (int64_t)imin(y + k, y1 - 1) * img.P.pitch +
                                                  4 * d);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t keep = y + k < y1 ? 1u : 0u;
#pragma unroll
        for (int j = 0; j < 4; j++) c[j] += keep & (((v[k] >> (8 * j)) & 0xFF) <= g.white ? 1u : 0u);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) ccount[4 * d + j] = (uint16_t)c[j];
  }
  __syncthreads();
  const int32_t nr = row == 0 ? g.bpr : g.bpr + 1;
  uint32_t* counts = (uint32_t*)(scratch + s * sstride);
  for (int32_t j = threadIdx.x; j < nr; j += 256) {
    const int32_t x0 = imax(j * g.sw, 0), x1 = imin(j * g.sw + g.sw, g.W);
    uint32_t n = 0;
    if (y0 < y1)
      for (int32_t x = x0; x < x1; x++) n += ccount[x];
    counts[row == 0 ? j : g.bpr + (row - 1) * (g.bpr + 1) + j] = n;
  }
}

// k_blur_counts_g from the bit-plane of pixels <= white (1/8 of the plane's
// bytes; NoiseGeom::bbits, kept current by the black- and noisefilter's
// clears).  Rectangles at least 32 wide, so a 32-pixel word meets at most two
// of them: a lane per (word column, row phase) keeps two popcount sums over
// its rows of the strip, then adds them into per-rectangle LDS counters.
__global__ void __launch_bounds__(256) k_blur_counts_bits(BlurGeom g, const uint32_t* bbits,
                                                          int64_t bb_stride, uint8_t* scratch,
                                                          int64_t sstride, const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  const int32_t row = blockIdx.x;
  const int32_t ry = row == 0 ? 0 : (row - 1) * g.sh + g.step_y;
  const int32_t y0 = imax(ry, 0), y1 = imin(ry + g.sh, g.H);
  const int32_t nr = row == 0 ? g.bpr : g.bpr + 1;
  const int32_t nwr = (g.W + 31) >> 5;
  extern __shared__ uint32_t rcount[];
  for (int32_t j = threadIdx.x; j < nr + 1; j += 256) rcount[j] = 0;
  __syncthreads();
  const uint32_t* plane = bbits + s * bb_stride;
  const int32_t nph = nwr >= 256 ? 1 : 256 / nwr;  // row phases
  const int32_t lanes = nph * nwr;
  for (int32_t t = threadIdx.x; t < (nwr >= 256 ? nwr : lanes); t += 256) {
    const int32_t wi = nwr >= 256 ? t : t % nwr, ph = nwr >= 256 ? 0 : t / nwr;
    const int32_t x0 = 32 * wi;
    const int32_t j0 = x0 / g.sw;
    // bits [0, cut) of a word belong to rectangle j0, [cut, 32) to j0 + 1
    const int32_t cut = imin((j0 + 1) * g.sw - x0, 32);
    const uint32_t m0 = cut >= 32 ? ~0u : (1u << cut) - 1u;
    uint32_t a0 = 0, a1 = 0;
    const uint32_t* col = plane + wi;
    int32_t y = y0 + ph;
    for (; y + 3 * nph < y1; y += 4 * nph) {
      uint32_t v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = col[(int64_t)(y + k * nph) * nwr];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        a0 += __popc(v[k] & m0);
        a1 += __popc(v[k] & ~m0);
      }
    }
    for (; y < y1; y += nph) {
      const uint32_t v = col[(int64_t)y * nwr];
      a0 += __popc(v & m0);
      a1 += __popc(v & ~m0);
    }
    if (a0 && j0 < nr) atomicAdd(&rcount[j0], a0);
    if (a1 && j0 + 1 < nr) atomicAdd(&rcount[j0 + 1], a1);
  }
  __syncthreads();
  uint32_t* counts = (uint32_t*)(scratch + s * sstride);
  for (int32_t j = threadIdx.x; j < nr; j += 256)
    counts[row == 0 ? j : g.bpr + (row - 1) * (g.bpr + 1) + j] = rcount[j];
}

template <int FMT>
__global__ void __launch_bounds__(256) k_blur_counts(PlaneRef img, BlurGeom g, uint8_t* scratch,
                                                     int64_t sstride, const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  const int32_t r = blockIdx.x;
  int32_t rx, ry;
  blur_rect_origin(g, r, &rx, &ry);
  const uint8_t* base = plane_ptr(img, s);
  // count_pixels_within_brightness(0, white): unclipped, outside = white
  const int32_t x0 = imax(rx, 0), x1 = imin(rx + g.sw - 1, g.W - 1);
  const int32_t y0 = imax(ry, 0), y1 = imin(ry + g.sh - 1, g.H - 1);
  uint32_t acc = 0;
  if (x0 <= x1 && y0 <= y1) {
    const int32_t w = x1 - x0 + 1;
    const int32_t n = w * (y1 - y0 + 1);
    for (int32_t i = threadIdx.x; i < n; i += 256) {
      const int32_t yy = y0 + i / w, xx = x0 + i % w;
      acc += gray_of(load_px_row<FMT>(base + (int64_t)yy * img.P.pitch, xx)) <= g.white ? 1u : 0u;
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
  __shared__ uint32_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* counts = (uint32_t*)(scratch + s * sstride);
    counts[r] = red[0] + red[1] + red[2] + red[3];
  }
}

__global__ void __launch_bounds__(256) k_blur_resolve(BlurGeom g, uint8_t* scratch, int64_t sstride,
                                                      const int32_t* active) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  const uint32_t* counts = (const uint32_t*)(scratch + s * sstride);
  uint8_t* wipe = scratch + s * sstride + (size_t)g.nrect * 4;
  extern __shared__ uint64_t sh[];  // [nrect] counts + [3*(bpr+2)] buffers
  uint64_t* cnt = sh;
  uint64_t* buf = sh + g.nrect;
  const int32_t nbuf = 3 * (g.bpr + 2);
  for (int32_t i = threadIdx.x; i < g.nrect; i += blockDim.x) cnt[i] = counts[i];
  for (int32_t i = threadIdx.x; i < nbuf; i += blockDim.x) buf[i] = 0;
  for (int32_t i = threadIdx.x; i < g.T * g.bpr; i += blockDim.x) wipe[i] = 0;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint64_t total = (uint64_t)(g.sw * g.sh);
  const int32_t bpr = g.bpr;
  int32_t op = 0, oc = 1, on = 2;  // prev / cur / next offsets into buf
  buf[oc + 0] = total;
  buf[oc + bpr] = total;
  buf[on + 0] = total;
  buf[on + bpr] = total;
  for (int32_t b = 0; b < bpr; b++) buf[oc + 1 + b] = cnt[b];
  for (int32_t t = 0; t < g.T; t++) {
    const int32_t base = bpr + t * (bpr + 1);
    buf[on + 0] = cnt[base + 0];
    for (int32_t block = 1; block <= bpr; block++) {
      buf[on + block + 1] = cnt[base + block];
      const uint64_t a = buf[op + block - 1], b = buf[op + block + 1], c = buf[oc + block];
      const uint64_t m1 = a > b ? (a > c ? a : c) : (b > c ? b : c);
      const uint64_t d = buf[on + block - 1], e = buf[on + block + 1];
      const uint64_t mx = d > e ? (d > m1 ? d : m1) : (e > m1 ? e : m1);
      if ((((float)mx) / total) <= g.intensity) {
        wipe[t * bpr + block - 1] = 1;
        buf[oc + block] = total;
      }
    }
    const int32_t tmp = op;
    op = oc;
    oc = on;
    on = tmp;
  }
}

// The same recurrence on the scalar unit, one wave per sheet, for rows of at
// most 56 blocks.  All three pointers of blurfilter_cpu index one array A
// (prev, cur, next at offsets op, oc, on, a rotation of 0, 1, 2), so block k
// of a row reads and writes only A[k-1 .. k+3]: that window lives in scalar
// registers and slides one entry a block.  A itself is one VGPR (lane j holds
// A[j]): the entry leaving the window is written into its lane, the one
// entering (untouched so far in this row) read from its lane; the row's
// counts are a second VGPR.  No memory access inside a row.  With the row's
// rotation the reads are
//   (0,1,2): next[k+1] = A[k+3]; the rest A[k-1], A[k+1] (three times); wipe A[k+1]
//   (1,2,0): next[k+1] = A[k+1]; A[k], A[k+2] (twice), A[k-1];          wipe A[k+2]
//   (2,0,1): next[k+1] = A[k+2]; A[k+1], A[k+3], A[k] (twice);          wipe A[k]
// and the float test ((float)max / total <= intensity) is monotone in max, so
// it is the integer compare max <= tmax with tmax found once per sheet.
constexpr int kBlurLanesMax = 120;  // bpr + 8 entries of A in two VGPRs
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t lane_get(uint32_t v, int32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int32_t)v, l);
}
__device__ __forceinline__ uint32_t lane_set(uint32_t v, uint32_t x, int32_t l) {
  return (int32_t)(threadIdx.x & 63) == l ? x : v;
}

// one row of type OP: blocks 1 .. bpr; returns the row's wipe bits (bit k-1)
// entries 0 .. 127 of an array over two VGPRs (lane l: entries l and 64 + l)
struct Lanes2 {
  uint32_t v0, v1;
};
__device__ __forceinline__ uint32_t lane_get(const Lanes2& v, int32_t l) {
  const uint32_t a = lane_get(v.v0, l & 63), b = lane_get(v.v1, l & 63);
  return l < 64 ? a : b;
}
__device__ __forceinline__ void lane_set(Lanes2& v, uint32_t x, int32_t l) {
  v.v0 = lane_set(v.v0, x, l);
  v.v1 = lane_set(v.v1, x, l - 64);
}

template <int OP>
__device__ __forceinline__ void blur_row(Lanes2& Av, Lanes2 rowv, int32_t bpr, uint32_t total,
                                         int32_t tmax, uint64_t (&wipes)[2]) {
  constexpr int ON = OP == 0 ? 2 : OP == 1 ? 0 : 1;
  uint32_t W0 = lane_get(Av, 0), W1 = lane_get(Av, 1), W2 = lane_get(Av, 2);
  uint32_t W3 = lane_get(Av, 3), W4 = lane_get(Av, 4);
  const uint32_t n0 = lane_get(rowv, 0);  // next[0] = A[on]
  if (ON == 0) W0 = n0;
  else if (ON == 1) W1 = n0;
  else W2 = n0;
  wipes[0] = wipes[1] = 0;  // bit k-1 of the pair: block k
#pragma unroll 4
  for (int32_t k = 1;; k++) {
    const uint32_t e = lane_get(rowv, k);
    uint32_t mx;
    bool w;
    if (OP == 0) {
      W4 = e;
      mx = umax(W0, umax(W2, W4));
      w = (int32_t)mx <= tmax;
      W2 = w ? total : W2;
    } else if (OP == 1) {
      W2 = e;
      mx = umax(umax(W0, W1), umax(W2, W3));
      w = (int32_t)mx <= tmax;
      W3 = w ? total : W3;
    } else {
      W3 = e;
      mx = umax(umax(W1, W2), umax(W3, W4));
      w = (int32_t)mx <= tmax;
      W1 = w ? total : W1;
    }
    const uint64_t bit = (uint64_t)w << ((k - 1) & 63);
    if (k <= 64) wipes[0] |= bit;
    else wipes[1] |= bit;
    if (k == bpr) break;
    lane_set(Av, W0, k - 1);
    W0 = W1;
    W1 = W2;
    W2 = W3;
    W3 = W4;
    W4 = lane_get(Av, k + 4);
  }
  lane_set(Av, W0, bpr - 1);
  lane_set(Av, W1, bpr);
  lane_set(Av, W2, bpr + 1);
  lane_set(Av, W3, bpr + 2);
  lane_set(Av, W4, bpr + 3);
}

// The same row for a row length known at compile time: the whole row's A in
// scalar registers (read from its lanes once, written back once), every
// block a handful of scalar operations.
template <int OP, int BPR>
__device__ __forceinline__ uint64_t blur_row_fixed(uint32_t& Av, uint32_t rowv, uint32_t total,
                                                   int32_t tmax) {
  constexpr int ON = OP == 0 ? 2 : OP == 1 ? 0 : 1;
  uint32_t a[BPR + 4];
#pragma unroll
  for (int j = 0; j < BPR + 4; j++) a[j] = lane_get(Av, j);
  a[ON] = lane_get(rowv, 0);  // next[0]
  uint64_t wipes = 0;
#pragma unroll
  for (int k = 1; k <= BPR; k++) {
    const uint32_t e = lane_get(rowv, k);
    uint32_t mx;
    if (OP == 0) {
      a[k + 3] = e;
      mx = umax(a[k - 1], umax(a[k + 1], a[k + 3]));
    } else if (OP == 1) {
      a[k + 1] = e;
      mx = umax(umax(a[k - 1], a[k]), umax(a[k + 1], a[k + 2]));
    } else {
      a[k + 2] = e;
      mx = umax(umax(a[k], a[k + 1]), umax(a[k + 2], a[k + 3]));
    }
    const bool w = (int32_t)mx <= tmax;
    if (OP == 0) a[k + 1] = w ? total : a[k + 1];
    else if (OP == 1) a[k + 2] = w ? total : a[k + 2];
    else a[k] = w ? total : a[k];
    wipes |= (uint64_t)w << (k - 1);
  }
#pragma unroll
  for (int j = 0; j < BPR + 4; j++) Av = lane_set(Av, a[j], j);
  return wipes;
}

// Rows of 33 .. 112 blocks.  Within a row the recurrence only READS A as it
// was before the row (an entry entering the window, A[k+4] at block k, has
// not been written in this row yet), so the scalar window reads the row's
// A and counts from their lanes and writes nothing back per block; the row's
// final A is then made lane-parallel from its counts and wipe bits (the last
// write of each entry, below), a handful of vector operations a row.
// 16 blocks KC+1 .. KC+16 of a row: their counts and the A entries entering
// the window read from lanes known at compile time up front, then a chain of
// scalar operations per block.  Blocks past bpr run too (their wipe bits are
// masked off; the row's state is rebuilt from the bits, not from the window).
__device__ __forceinline__ uint32_t lane_c(const Lanes2& v, int l) {
  return l < 64 ? lane_get(v.v0, l) : lane_get(v.v1, l - 64);
}
template <int OP, int KC>
__device__ __forceinline__ void blur_chunk_ro(const Lanes2& Aold, const Lanes2& rowv, int32_t bpr,
                                              uint32_t total, int32_t tmax, uint32_t (&W)[5],
                                              uint64_t& w0, uint64_t& w1) {
  if (KC + 1 > bpr) return;
  uint32_t e[16], nx[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int k = KC + 1 + i;
    e[i] = k < 128 ? lane_c(rowv, k) : 0u;
    nx[i] = k + 4 < 128 ? lane_c(Aold, k + 4) : 0u;
  }
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int k = KC + 1 + i;
    uint32_t mx;
    bool w;
    if (OP == 0) {
      W[4] = e[i];
      mx = umax(W[0], umax(W[2], W[4]));
      w = (int32_t)mx <= tmax;
      W[2] = w ? total : W[2];
    } else if (OP == 1) {
      W[2] = e[i];
      mx = umax(umax(W[0], W[1]), umax(W[2], W[3]));
      w = (int32_t)mx <= tmax;
      W[3] = w ? total : W[3];
    } else {
      W[3] = e[i];
      mx = umax(umax(W[1], W[2]), umax(W[3], W[4]));
      w = (int32_t)mx <= tmax;
      W[1] = w ? total : W[1];
    }
    if (k <= 64) w0 |= w ? 1ull << (k - 1) : 0ull;
    else if (k <= 128) w1 |= w ? 1ull << (k - 65) : 0ull;
    W[0] = W[1];
    W[1] = W[2];
    W[2] = W[3];
    W[3] = W[4];
    W[4] = nx[i];
  }
}
template <int OP>
__device__ __forceinline__ void blur_row_ro(const Lanes2& Aold, const Lanes2& rowv, int32_t bpr,
                                            uint32_t total, int32_t tmax, uint64_t (&wipes)[2]) {
  constexpr int ON = OP == 0 ? 2 : OP == 1 ? 0 : 1;
  uint32_t W[5];
#pragma unroll
  for (int j = 0; j < 5; j++) W[j] = lane_get(Aold.v0, j);
  W[ON] = lane_get(rowv.v0, 0);  // next[0] = A[on]
  uint64_t w0 = 0, w1 = 0;  // bit k-1: block k
  blur_chunk_ro<OP, 0>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  blur_chunk_ro<OP, 16>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  blur_chunk_ro<OP, 32>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  blur_chunk_ro<OP, 48>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  blur_chunk_ro<OP, 64>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  blur_chunk_ro<OP, 80>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  blur_chunk_ro<OP, 96>(Aold, rowv, bpr, total, tmax, W, w0, w1);
  wipes[0] = bpr >= 64 ? w0 : w0 & ((1ull << bpr) - 1);
  wipes[1] = bpr <= 64 ? 0 : bpr >= 128 ? w1 : w1 & ((1ull << (bpr - 64)) - 1);
}
// The row's final A, entry j per lane (j = lane, 64 + lane): the last write
// of entry j during the row of type OP (next[0] first, then per block k the
// count write and the wipe write):
//   OP 0: count A[k+3] = row[k], wipe A[k+1] = total, next[0] at A[2]
//   OP 1: count A[k+1] = row[k], wipe A[k+2] = total, next[0] at A[0]
//   OP 2: count A[k+2] = row[k], wipe A[k]   = total, next[0] at A[1]
template <int OP>
__device__ __forceinline__ Lanes2 blur_row_state(const Lanes2& Aold, const Lanes2& rowv,
                                                 int32_t bpr, uint32_t total,
                                                 const uint64_t (&wipes)[2]) {
  constexpr int S = OP == 0 ? 3 : OP == 1 ? 1 : 2;  // count shift: A[j] = row[j - S]
  constexpr int ON = OP == 0 ? 2 : OP == 1 ? 0 : 1;
  const int lane = threadIdx.x & 63;
  const uint32_t r0 = lane_get(rowv.v0, 0);
  auto wbit = [&](int32_t k) -> bool {  // block k wiped
    if (k < 1 || k > bpr) return false;
    const uint64_t m = k <= 64 ? wipes[0] : wipes[1];
    return (m >> ((k - 1) & 63)) & 1;
  };
  auto entry = [&](int32_t j, uint32_t old, uint32_t shifted) -> uint32_t {
    // shifted = row[j - S] (valid for j >= S)
    if (OP == 0) {
      if (j >= 2 && j <= bpr + 1 && wbit(j - 1)) return total;
      if (j >= 4 && j <= bpr + 3) return shifted;
      return j == ON ? r0 : old;
    } else if (OP == 1) {
      if (j >= 2 && j <= bpr + 1) return shifted;
      if (j == bpr + 2 && wbit(bpr)) return total;
      return j == ON ? r0 : old;
    } else {
      if (j >= 1 && j <= bpr && wbit(j)) return total;
      if (j >= 3 && j <= bpr + 2) return shifted;
      return j == ON ? r0 : old;
    }
  };
  // row[j - S] for j = lane and j = 64 + lane
  const int src0 = (lane - S) & 63;
  const uint32_t a0 = (uint32_t)__shfl((int)rowv.v0, src0, 64);
  const uint32_t b0 = (uint32_t)__shfl((int)rowv.v1, src0, 64);
  const uint32_t sh0 = a0;                      // lane >= S: row[lane - S] (v0)
  const uint32_t sh1 = lane >= S ? b0 : a0;     // row[64 + lane - S]: v1 or the top of v0
  Lanes2 r;
  r.v0 = entry(lane, Aold.v0, sh0);
  r.v1 = entry(64 + lane, Aold.v1, sh1);
  return r;
}

template <int BPR>
__device__ __forceinline__ void blur_rows_fixed(uint32_t Av, const uint32_t* counts, uint8_t* wipe,
                                                int32_t T, uint32_t total, int32_t tmax) {
  const int lane = threadIdx.x & 63;
  constexpr int32_t rl = BPR + 1;
  uint32_t rowv = T > 0 && lane < rl ? counts[BPR + lane] : 0;
  for (int32_t t = 0; t < T; t++) {
    const uint32_t cur = rowv;
    if (t + 1 < T) rowv = lane < rl ? counts[BPR + (t + 1) * rl + lane] : 0;
    const int op = t % 3;
    const uint64_t wipes = op == 0   ? blur_row_fixed<0, BPR>(Av, cur, total, tmax)
                           : op == 1 ? blur_row_fixed<1, BPR>(Av, cur, total, tmax)
                                     : blur_row_fixed<2, BPR>(Av, cur, total, tmax);
    if (lane < BPR) wipe[t * BPR + lane] = (uint8_t)((wipes >> lane) & 1);
  }
}

// CHUNKED: rows of 33 .. 112 blocks (blur_row_ro + blur_row_state); otherwise the fixed
// row lengths 12 .. 32 and the generic sliding window.  Separate kernels keep
// the chunked path's scalar registers free of the fixed rows' pressure.
template <bool CHUNKED>
__global__ void __launch_bounds__(64) k_blur_resolve_w(BlurGeom g, uint8_t* scratch,
                                                       int64_t sstride, const int32_t* active) {
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  const uint32_t* counts = (const uint32_t*)(scratch + s * sstride);
  uint8_t* wipe = scratch + s * sstride + (size_t)g.nrect * 4;
  const int lane = threadIdx.x;
  const int32_t bpr = g.bpr;
  const uint32_t total = (uint32_t)(g.sw * g.sh);
  // blurfilter_cpu's set-up (A zero where the reference reads uninitialised
  // stack, as the other resolver): cur[0], cur[bpr], next[0], next[bpr], then
  // cur[1 .. bpr] = the first row's counts (A[2] and A[bpr + 1] overwritten)
  // entries l (and 64 + l, for rows past 56 blocks) of A in lane l
  auto a_init = [&](int32_t j) -> uint32_t {
    uint32_t v = 0;
    if (j == 1 || j == bpr + 1 || j == 2 || j == bpr + 2) v = total;
    if (j >= 2 && j < 2 + bpr) v = counts[j - 2];
    return v;
  };
  uint32_t Av = a_init(lane);
  // the largest max that is wiped (-1: none)
  auto wiped = [&](uint32_t m) { return ((float)m) / (float)(uint64_t)total <= g.intensity; };
  int32_t tmax = -1;
  if (wiped(0u)) {
    uint32_t lo = 0, hi = total;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo + 1) / 2;
      if (wiped(mid)) lo = mid;
      else hi = mid - 1;
    }
    tmax = (int32_t)lo;
  }
  tmax = __builtin_amdgcn_readfirstlane(tmax);
  // row lengths of 150-400 dpi pages at the default 100-pixel blocks
  if (!CHUNKED) switch (bpr) {
#define UPH_BLUR_FIXED(n) \
  case n:                 \
    blur_rows_fixed<n>(Av, counts, wipe, g.T, total, tmax); \
    return;
    UPH_BLUR_FIXED(12) UPH_BLUR_FIXED(13) UPH_BLUR_FIXED(14) UPH_BLUR_FIXED(15)
    UPH_BLUR_FIXED(16) UPH_BLUR_FIXED(17) UPH_BLUR_FIXED(18) UPH_BLUR_FIXED(19)
    UPH_BLUR_FIXED(20) UPH_BLUR_FIXED(21) UPH_BLUR_FIXED(22) UPH_BLUR_FIXED(23)
    UPH_BLUR_FIXED(24) UPH_BLUR_FIXED(25) UPH_BLUR_FIXED(26) UPH_BLUR_FIXED(27)
    UPH_BLUR_FIXED(28) UPH_BLUR_FIXED(29) UPH_BLUR_FIXED(30) UPH_BLUR_FIXED(31)
    UPH_BLUR_FIXED(32)
#undef UPH_BLUR_FIXED
    default:
      break;
  }
  // the next row's counts one row ahead (entries l and 64 + l in lane l)
  const int32_t rl = bpr + 1;
  Lanes2 A2{Av, a_init(64 + lane)};
  auto row_of = [&](int32_t t) {
    const int64_t r0 = bpr + (int64_t)t * rl;
    return Lanes2{lane < rl ? counts[r0 + lane] : 0u, 64 + lane < rl ? counts[r0 + 64 + lane] : 0u};
  };
  Lanes2 rowv = g.T > 0 ? row_of(0) : Lanes2{0u, 0u};
  for (int32_t t = 0; t < g.T; t++) {
    const Lanes2 cur = rowv;
    if (t + 1 < g.T) rowv = row_of(t + 1);
    const int op = t % 3;
    uint64_t wipes[2];
    if (CHUNKED) {
      if (op == 0) {
        blur_row_ro<0>(A2, cur, bpr, total, tmax, wipes);
        A2 = blur_row_state<0>(A2, cur, bpr, total, wipes);
      } else if (op == 1) {
        blur_row_ro<1>(A2, cur, bpr, total, tmax, wipes);
        A2 = blur_row_state<1>(A2, cur, bpr, total, wipes);
      } else {
        blur_row_ro<2>(A2, cur, bpr, total, tmax, wipes);
        A2 = blur_row_state<2>(A2, cur, bpr, total, wipes);
      }
    } else if (op == 0) {
      blur_row<0>(A2, cur, bpr, total, tmax, wipes);
    } else if (op == 1) {
      blur_row<1>(A2, cur, bpr, total, tmax, wipes);
    } else {
      blur_row<2>(A2, cur, bpr, total, tmax, wipes);
    }
    if (lane < bpr) wipe[t * bpr + lane] = (uint8_t)((wipes[0] >> lane) & 1);
    if (64 + lane < bpr) wipe[t * bpr + 64 + lane] = (uint8_t)((wipes[1] >> lane) & 1);
  }
}

template <int FMT>
__global__ void __launch_bounds__(256) k_blur_wipe(PlaneRef img, BlurGeom g, uint8_t* scratch,
                                                   int64_t sstride, const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  const int32_t b = blockIdx.x;  // t*bpr + j
  const uint8_t* wipe = scratch + s * sstride + (size_t)g.nrect * 4;
  if (!wipe[b]) return;
  const int32_t t = b / g.bpr, j = b % g.bpr;
  const Rect r = clip(rect_from_size(j * g.sw, t * g.sh, g.sw, g.sh), g.W, g.H);
  uint8_t* base = plane_ptr(img, s);
  const int32_t w = r.x1 - r.x0 + 1;
  if (w <= 0 || r.y1 < r.y0) return;
  const int32_t n = w * (r.y1 - r.y0 + 1);
  for (int32_t i = threadIdx.x; i < n; i += 256) {
    const int32_t yy = r.y0 + i / w, xx = r.x0 + i % w;
    white_px<FMT>(base + (int64_t)yy * img.P.pitch, xx);
  }
}

template <int FMT>
static void launch_blur_t(const PlaneRef& img, const BlurGeom& g, uint8_t* scr, int64_t ss,
                          const int32_t* active, int count, hipStream_t st, const uint32_t* bbits,
                          int64_t bb_stride) {
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const bool v16 = img.P.pitch % 16 == 0 && img.P.stride % 16 == 0 && img.P.pitch >= ((g.W + 15) & ~15) &&
                   a16(img.P.base[0]) && a16(img.P.base[1]);
  if (g.nrect > 0 && FMT == F_GRAY8 && bbits && g.sw >= 32 && g.W <= (1 << 16))
    UPH_LAUNCH_DIAG(64, k_blur_counts_bits, dim3(1 + g.T, count), dim3(256),
                    4 * (size_t)(g.bpr + 2), st, g, bbits, bb_stride, scr, ss, active);
  else if (g.nrect > 0 && FMT == F_GRAY8 && g.sh <= 65535 && g.W <= (1 << 16) && v16)
    UPH_LAUNCH_DIAG(64, k_blur_counts_g<true>, dim3(1 + g.T, count), dim3(256),
                    2 * (size_t)((g.W + 3) & ~3), st, img, g, scr, ss, active);
  else if (g.nrect > 0 && FMT == F_GRAY8 && g.sh <= 65535 && g.W <= (1 << 16))
    UPH_LAUNCH_DIAG(64, k_blur_counts_g<false>, dim3(1 + g.T, count), dim3(256),
                    2 * (size_t)((g.W + 3) & ~3), st, img, g, scr, ss, active);
  else if (g.nrect > 0)
    hipLaunchKernelGGL(k_blur_counts<FMT>, dim3(g.nrect, count), dim3(256), 0, st, img, g, scr, ss,
                       active);
  const size_t lds = sizeof(uint64_t) * ((size_t)g.nrect + 3 * (size_t)(g.bpr + 2));
  const bool scalar = g.bpr >= 1 && g.bpr + 8 <= kBlurLanesMax && (int64_t)g.sw * g.sh < (1ll << 31);
  if (diag_skip() & 8) {
  } else if (scalar && g.bpr > 32 && g.bpr <= 112) {
    hipLaunchKernelGGL(k_blur_resolve_w<true>, dim3(count), dim3(64), 0, st, g, scr, ss, active);
  } else if (scalar) {
    hipLaunchKernelGGL(k_blur_resolve_w<false>, dim3(count), dim3(64), 0, st, g, scr, ss, active);
  } else {
    hipLaunchKernelGGL(k_blur_resolve, dim3(count), dim3(256), lds, st, g, scr, ss, active);
  }
  if (g.T * g.bpr > 0)
    hipLaunchKernelGGL(k_blur_wipe<FMT>, dim3(g.T * g.bpr, count), dim3(256), 0, st, img, g, scr,
                       ss, active);
}

void launch_blurfilter(const PlaneRef& img, const BlurGeom& g, void* scratch,
                       int64_t scratch_stride, const int32_t* active, int count, hipStream_t st,
                       const uint32_t* bbits, int64_t bb_stride) {
  uint8_t* scr = (uint8_t*)scratch;
  switch (img.P.fmt) {
    case F_GRAY8:
      launch_blur_t<F_GRAY8>(img, g, scr, scratch_stride, active, count, st, bbits, bb_stride);
      break;
    case F_Y400A:
      launch_blur_t<F_Y400A>(img, g, scr, scratch_stride, active, count, st, nullptr, 0);
      break;
    default: launch_blur_t<F_RGB24>(img, g, scr, scratch_stride, active, count, st, nullptr, 0); break;
  }
}

// =========================================================================
// NOISEFILTER (filters.c:238-338)
//   Raster scan; a pixel p with max(rgb) < white ("trigger") counts the
//   pixels with min(rgb) < white ("dark") in square rings of level 1..N
//   (N = intensity) until a ring is empty; if 1 + rings <= N the centre and
//   the counted rings are cleared.  Away from the left/top edge (where the
//   ring loops' unsigned comparisons drop whole rows, see oracle.c) an empty
//   ring separates its inside from everything else, so a clear removes whole
//   8-connected dark components of <= N pixels ("small").  Hence:
//     * triggers of large components outside the edge zone never clear;
//     * a small component C farther than 2N-1 from any other small pixel and
//       from the edge zone is cleared iff one of its triggers passes the test
//       on the ORIGINAL image (nothing that test reads ever changes);
//     * everything else (edge zone, clustered small components) is replayed
//       literally, in raster order, by one wave per sheet.
//   The parallel path is used for N <= 4 (radius constants below).
// =========================================================================
constexpr int kNT = 64;                    // tile height (and width for byte planes)
constexpr int kHalo = 14;                  // 4 (ring) + 7 (cluster) + 3 (component)
constexpr int kRW = kNT + 2 * kHalo;       // 92 region rows
// GRAY8 tiles are 100 wide: their region rows (from the bit-plane) fill the
// 128-bit row tables, so the per-row phases cover 100 interior columns
// instead of 64 for the same work (halo share 2.07 -> 1.84)
constexpr int kNTG = 100;
template <int FMT>
constexpr int noise_tile_w() { return FMT == F_GRAY8 ? kNTG : kNT; }
constexpr int kZone = 32;                  // sequential edge zone (x or y < 32)
constexpr int kEligible = kZone + 8;       // parallel only for components at >= 40

bool noise_geometry(int32_t W, int32_t H, uint64_t intensity, uint8_t white, NoiseGeom* g) {
  g->W = W;
  g->H = H;
  g->intensity = intensity > 64 ? 64 : (int32_t)intensity;
  g->white = white;
  // the parallel path only queues edge-zone and clustered triggers; the
  // all-sequential path (intensity > 4) may queue every pixel
  g->all_seq = intensity > 4 ? 1 : 0;
  int64_t cap = g->all_seq ? (int64_t)W * H + 64 : ((int64_t)W * H) / 4 + 1024;
  if (cap > (1 << 27)) cap = 1 << 27;
  g->capacity = (int32_t)cap;
  g->bbits = nullptr;
  g->bb_stride = 0;
  return true;
}

static size_t noise_list_bytes(const NoiseGeom& g) {
  // counters (2 x u32 padded to 256 B) + clear list + seq list
  size_t b = 256 + (size_t)g.capacity * 4 * 2;
  return (b + 255) & ~(size_t)255;
}

static size_t pow2_at_least(size_t n) {
  size_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// 32-pixel words per row of the GRAY8 dark bit-plane
static int32_t noise_bit_words(const NoiseGeom& g) { return noise_bit_words(g.W); }

// k_noise_group keeps up to 16 triggers a thread in LDS (more: in HBM)
constexpr int kCapPerThread = 16;
// Large sheets (C4's 9920 x 7016 double pages: several thousand triggers a
// sheet, never next to the code-block decode) keep 1024 threads and 16384
// triggers in LDS.
static int group_threads(int32_t W, int32_t H) { return (int64_t)W * H > (16 << 20) ? 1024 : 256; }
size_t noise_scratch_bytes(const NoiseGeom& g) {
  // lists + a global sort buffer for the rare > 8192-trigger sequential case;
  // the GRAY8 dark bit-plane shares the sort buffer's space (it is read by
  // k_noise_classify only, before k_noise_resolve may sort)
  // (and k_noise_group's keys / roots / last, 3 x its LDS cap words)
  size_t sort = 4 * pow2_at_least((size_t)g.capacity);
  const size_t cap3 = 12 * (size_t)kCapPerThread * (size_t)group_threads(g.W, g.H);
  if (sort < cap3) sort = cap3;
  const size_t bits = 4 * (size_t)noise_bit_words(g) * (size_t)g.H;
  return noise_list_bytes(g) + (sort > bits ? sort : bits);
}

struct NoisePtrs {
  uint32_t* nclear;
  uint32_t* nseq;
  uint32_t* clear;
  uint32_t* seq;
};
__device__ __forceinline__ NoisePtrs noise_ptrs(const NoiseGeom& g, uint8_t* base) {
  NoisePtrs p;
  p.nclear = (uint32_t*)base;
  p.nseq = p.nclear + 1;
  p.clear = (uint32_t*)(base + 256);
  p.seq = p.clear + g.capacity;
  return p;
}

// 9 bits of a region row bitmask starting at column c (bit i = column c+i)
__device__ __forceinline__ uint32_t row9(const uint32_t* w, int c) {
  const int word = c >> 5, off = c & 31;
  uint64_t v = ((uint64_t)w[word + 1] << 32) | w[word];
  return (uint32_t)(v >> off) & 0x1FFu;
}

// Dark component of (cx,cy) restricted to its 9x9 box; returns popcount
// (capped growth after 4 dilations) and the mask rows.  Every dilation step
// only adds pixels connected to the centre, so the search stops as soon as
// more than 4 are reached (the component is large; text strokes exit after
// the first step, whose 3x3 neighbourhood is all 8-adjacent to the centre).
__device__ __forceinline__ int flood9(const uint32_t (*drow)[4], int cx, int cy, uint32_t* comp) {
  uint32_t D[9], cur[9];
#pragma unroll
  for (int r = 0; r < 9; r++) {
    D[r] = row9(drow[cy - 4 + r], cx - 4);
    cur[r] = 0;
  }
  cur[4] = 1u << 4;
  for (int it = 0; it < 4; it++) {
    uint32_t nx[9];
    bool same = true;
    int n = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
      uint32_t u = cur[r] | (r > 0 ? cur[r - 1] : 0) | (r < 8 ? cur[r + 1] : 0);
      u = (u | (u << 1) | (u >> 1)) & D[r] & 0x1FFu;
      nx[r] = u;
      same &= (u == cur[r]);
      n += __popc(u);
    }
#pragma unroll
    for (int r = 0; r < 9; r++) cur[r] = nx[r];
    if (n > 4) {
#pragma unroll
      for (int r = 0; r < 9; r++) comp[r] = cur[r];
      return n;
    }
    if (same) break;
  }
  int n = 0;
#pragma unroll
  for (int r = 0; r < 9; r++) {
    comp[r] = cur[r];
    n += __popc(cur[r]);
  }
  return n;
}

// bits [c, c+n) of a 128-bit region row (n <= 32, c + n <= 128)
__device__ __forceinline__ uint32_t row_bits(const uint32_t* w, int c, int n) {
  const int word = c >> 5, off = c & 31;
  const uint64_t v = ((uint64_t)(word < 3 ? w[word + 1] : 0u) << 32) | w[word];
  return (uint32_t)(v >> off) & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
}

// Append the (gx, gy) keys of the lanes with `want` to a list: one atomic per
// wave, ballot-compacted.
__device__ __forceinline__ void wave_append(bool want, int32_t gx, int32_t gy, uint32_t* counter,
                                            uint32_t* list, int32_t capacity) {
  const unsigned long long M = __ballot(want);
  if (!M) return;
  const int lane = threadIdx.x & 63;
  uint32_t base = 0;
  const int leader = __ffsll((long long)M) - 1;
  if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(M));
  base = __shfl(base, leader, 64);
  if (want) {
    const uint32_t k = base + (uint32_t)__popcll(M & ((1ull << lane) - 1ull));
    if (k < (uint32_t)capacity) list[k] = ((uint32_t)gy << 16) | (uint32_t)gx;
  }
}

// Dark bits (byte < t) of 32 gray bytes (eight dwords) as one word, bit
// 4 d + q = byte q of dword d.  Per dword: 16-bit SWAR lanes hold
// (0x100 + t - 1) - byte, whose bit 8 is (byte < t) with nothing above it, so
// one byte permute gathers the four flags as bytes of 0 or 1; the eight
// dwords' flag bytes are stacked (bit 8 q + d), and four delta swaps
// transpose that 4 x 8 bit matrix into pixel order.
__device__ __forceinline__ uint32_t dark_bits32(const uint32_t (&w)[8], uint32_t white) {
  const uint32_t K = (0x100u + white - 1u) * 0x00010001u;
  uint32_t g = 0;
#pragma unroll
  for (int d = 0; d < 8; d++) {
    const uint32_t lo = K - (w[d] & 0x00FF00FFu);          // bits 8, 24: bytes 0, 2
    const uint32_t hi = K - ((w[d] >> 8) & 0x00FF00FFu);   // bits 8, 24: bytes 1, 3
    g |= __builtin_amdgcn_perm(hi, lo, 0x07030501u) << d;  // bytes: flags of bytes 0..3
  }
  auto dswap = [](uint32_t x, uint32_t m, int delta) {
    const uint32_t t = ((x >> delta) ^ x) & m;
    return x ^ t ^ (t << delta);
  };
  g = dswap(g, 0x0000F0F0u, 12);
  g = dswap(g, 0x00CC00CCu, 6);
  g = dswap(g, 0x0A0A0A0Au, 3);
  return dswap(g, 0x22222222u, 1);
}

// GRAY8 dark bit-plane: bit b of word w of row y is (pixel 32 w + b < white);
// columns >= W are 0.  One lane per word, two 16-byte loads (rows are
// 256-byte pitched, so a row's last word reads inside the pitch).  The
// classify tiles then read 92-bit region rows as five words each instead of
// re-reading and re-comparing 2x-overlapping byte halos.
__global__ void __launch_bounds__(256) k_noise_bits(PlaneRef img, NoiseGeom g, uint32_t* bits,
                                                    int64_t bstride, int32_t nwr, float rnwr,
                                                    const int32_t* active) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  // t / nwr from the float reciprocal, corrected by one either way
  int32_t y = (int32_t)((float)t * rnwr);
  if (y * nwr > t) y--;
  else if ((y + 1) * nwr <= t) y++;
  if (y >= g.H) return;
  const int32_t wi = t - y * nwr, x0 = 32 * wi;
  const uint4* p = reinterpret_cast<const uint4*>(plane_ptr(img, s) + (int64_t)y * img.P.pitch + x0);
  const uint4 a = p[0], b = p[1];
  uint32_t m = dark_bits32({a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}, g.white);
  if (x0 + 32 > g.W) m &= (1u << (g.W - x0)) - 1u;  // g.W - x0 in [1, 31]
  bits[s * bstride + t] = m;
}

// The decode of a GRAY8 page into its sheet (sheet_stages.c:151-165 with the
// page covering the sheet: a plain copy) fused with the first pass that reads
// the result: the noisefilter's dark bit-plane (k_noise_bits).  A lane per
// 32-pixel word of the whole sheet (rows are ceil(W/32) words, not a multiple
// of 64: a wave per row would leave most lanes of its second pass idle): two
// 16-byte loads, two 16-byte stores (the row's last word in pieces up to W),
// one bit-plane word.
__global__ void __launch_bounds__(256) k_decode_gray(const uint8_t* src, int64_t spitch,
                                                     int64_t sstride, PlaneRef dst, uint8_t white,
                                                     uint32_t* bits, int64_t bstride, int32_t nwr,
                                                     float rnwr, uint32_t* bbits, uint32_t* rm,
                                                     int64_t rm_stride, uint32_t rm_max) {
  const int s = blockIdx.y;
  const Planes& P = dst.P;
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  // t / nwr from the float reciprocal, corrected by one either way
  int32_t y = (int32_t)((float)t * rnwr);
  if (y * nwr > t) y--;
  else if ((y + 1) * nwr <= t) y++;
  if (y >= P.H) return;
  const int32_t wi = t - y * nwr, x0 = 32 * wi;
  const uint8_t* srow = src + s * sstride + (int64_t)y * spitch;
  uint8_t* d = plane_ptr(dst, s) + (int64_t)y * P.pitch + x0;
  // a 16-byte chunk starting before W lies inside the 16-aligned pitch
  const uint4 a = *reinterpret_cast<const uint4*>(srow + x0);
  const uint4 b = x0 + 16 < P.W ? *reinterpret_cast<const uint4*>(srow + x0 + 16)
                                : make_uint4(~0u, ~0u, ~0u, ~0u);
  uint32_t m = dark_bits32({a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}, white);
  // the blurfilter's bits: pixel <= white (byte < white + 1)
  uint32_t mb = bbits ? dark_bits32({a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}, (uint32_t)white + 1u) : 0u;
  // the blackfilter's match plane: pixel <= mask_max
  uint32_t mr = rm ? dark_bits32({a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}, rm_max + 1u) : 0u;
  if (x0 + 32 <= P.W) {
    *reinterpret_cast<uint4*>(d) = a;
    *reinterpret_cast<uint4*>(d + 16) = b;
  } else {
    // the row's last word: n = W - x0 in [1, 31] bytes, as a 16-byte chunk,
    // dwords and the last dword's bytes
    const int32_t n = P.W - x0;
    m &= (1u << n) - 1u;
    mb &= (1u << n) - 1u;
    mr &= (1u << n) - 1u;
    uint4 q = a;
    int32_t j = 0;
    if (n >= 16) {
      *reinterpret_cast<uint4*>(d) = a;
      q = b;
      j = 16;
    }
    const int32_t r = n - j;  // 0..15
    if (r >= 4) *reinterpret_cast<uint32_t*>(d + j) = q.x;
    if (r >= 8) *reinterpret_cast<uint32_t*>(d + j + 4) = q.y;
    if (r >= 12) *reinterpret_cast<uint32_t*>(d + j + 8) = q.z;
    uint32_t last = r < 4 ? q.x : r < 8 ? q.y : r < 12 ? q.z : q.w;
    for (int32_t i = j + (r & ~3); i < n; i++, last >>= 8) d[i] = (uint8_t)last;
  }
  if (bits) bits[s * bstride + t] = m;
  if (bbits) bbits[s * bstride + t] = mb;
  if (rm) {  // rows of (nwr + 1) & ~1 words: an odd row's pad word is 0
    const int32_t rw = (nwr + 1) & ~1;
    uint32_t* r = rm + s * rm_stride + (int64_t)y * rw + wi;
    if (wi + 1 == nwr && (nwr & 1)) *reinterpret_cast<uint2*>(r) = make_uint2(mr, 0u);
    else *r = mr;
  }
}

// The blackfilter's v-stripe row sums (darkness_rect's sums over the stripe's
// columns [vx0, vx1], filters.c:49-104) straight from the GRAY8 pages the
// decode copies unchanged.  A half-wave per row (32 lanes x 16 bytes cover a
// 500-column stripe in one load each), eight rows per wave with all their
// loads in flight, SAD byte sums, then a 32-lane sum per row.
constexpr int kStripeRowsPerWave = 8;
__global__ void __launch_bounds__(256) k_stripe_sums(const uint8_t* src, int64_t spitch,
                                                     int64_t sstride, int32_t H, uint32_t* vsum,
                                                     int64_t vstride, int32_t vx0, int32_t vx1) {
  const int s = blockIdx.y;
  const int lane = threadIdx.x & 63, half = lane >> 5, hl = lane & 31;
  const int32_t yw = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kStripeRowsPerWave;
  if (yw >= H) return;
  const uint8_t* page = src + s * sstride;
  const int32_t xa = vx0 & ~15;
  constexpr int kR = kStripeRowsPerWave / 2;  // rows per half-wave
  uint32_t acc[kR] = {};
  for (int32_t x = xa + 16 * hl; x <= vx1; x += 16 * 32) {  // one pass for stripes <= 512 columns
    uint32_t keep[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t xq = x + 4 * q;
      keep[q] = 0;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (xq + j >= vx0 && xq + j <= vx1) keep[q] |= 0xFFu << (8 * j);
    }
    uint4 v[kR];
#pragma unroll
    for (int r = 0; r < kR; r++) {
      const int32_t y = imin(yw + 2 * r + half, H - 1);
      v[r] = *reinterpret_cast<const uint4*>(page + (int64_t)y * spitch + x);
    }
#pragma unroll
    for (int r = 0; r < kR; r++) {
      acc[r] = __builtin_amdgcn_sad_u8(v[r].x & keep[0], 0u, acc[r]);
      acc[r] = __builtin_amdgcn_sad_u8(v[r].y & keep[1], 0u, acc[r]);
      acc[r] = __builtin_amdgcn_sad_u8(v[r].z & keep[2], 0u, acc[r]);
      acc[r] = __builtin_amdgcn_sad_u8(v[r].w & keep[3], 0u, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kR; r++) {
    uint32_t a = acc[r];
    for (int o = 16; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);  // within the half-wave
    const int32_t y = yw + 2 * r + half;
    if (hl == 0 && y < H) vsum[s * vstride + y] = a;
  }
}

void launch_decode_gray(const uint8_t* src, int64_t spitch, int64_t sstride, const PlaneRef& dst,
                        uint8_t white, uint32_t* bits, int64_t bits_stride, uint32_t* vsum,
                        int64_t vsum_stride, int32_t vx0, int32_t vx1, int count, hipStream_t st,
                        uint32_t* bbits, uint32_t* rm, int64_t rm_stride, uint8_t rm_max) {
  const int32_t nwr = (dst.P.W + 31) >> 5;
  const int64_t words = (int64_t)nwr * dst.P.H;
  UPH_LAUNCH_DIAG(262144, k_decode_gray, dim3((unsigned)((words + 255) / 256), count), dim3(256), 0, st,
                     src, spitch, sstride, dst, white, bits, bits_stride, nwr, 1.0f / (float)nwr,
                     bbits, rm, rm_stride, (uint32_t)rm_max);
  if (vsum && vx0 <= vx1)
    hipLaunchKernelGGL(k_stripe_sums,
                       dim3((unsigned)((dst.P.H + 4 * kStripeRowsPerWave - 1) / (4 * kStripeRowsPerWave)),
                            count),
                       dim3(256), 0, st,
                       src, spitch, sstride, dst.P.H, vsum, vsum_stride, vx0, vx1);
}

// Whether the classification of a small dark pixel (tile coordinates rx, ry)
// must go to the sequential replay, or clears it in parallel (see above).
struct SmallVerdict {
  bool seq, clear;
};
// A small component (<= 4 pixels) as offsets from one of its pixels, packed
// one byte a pixel (dx + 4 | (dy + 4) << 4, 0xFF = none): the restricted
// flood's result, kept from the candidate pass for the verdict pass.
constexpr uint32_t kNotSmall = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t pack_comp(const uint32_t (&comp)[9]) {
  uint32_t rec = kNotSmall;
  int nc = 0;
#pragma unroll
  for (int r = 0; r < 9; r++) {
    uint32_t mm = comp[r];
    while (mm) {
      const int b = __ffs(mm) - 1;
      mm &= mm - 1;
      if (nc < 4) rec = (rec & ~(0xFFu << (8 * nc))) | ((uint32_t)(b | (r << 4)) << (8 * nc));
      nc++;
    }
  }
  return nc <= 4 ? rec : kNotSmall;
}
// The verdict from the component's pixels (offsets cxs, cys from (rx, ry)).
__device__ __forceinline__ SmallVerdict small_verdict_pixels(const uint32_t (*drow)[4],
                                                             const uint32_t (*trow)[4],
                                                             const uint32_t (*srow)[4], int rx,
                                                             int ry, int32_t gx, int32_t gy,
                                                             bool trig, int N, int nc,
                                                             const int (&cxs)[4],
                                                             const int (&cys)[4]) {
  SmallVerdict v{false, false};
  int bx0 = 4, bx1 = -4, by0 = 4, by1 = -4;  // bounding box, offsets from (rx, ry)
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (k < nc) {
      bx0 = imin(bx0, cxs[k]);
      bx1 = imax(bx1, cxs[k]);
      by0 = imin(by0, cys[k]);
      by1 = imax(by1, cys[k]);
    }
  bool eligible = nc <= 4 && gx + bx0 >= kEligible && gy + by0 >= kEligible;
  // no foreign small pixel within Chebyshev 7 of the component: checked on
  // the bounding box dilated by 7 (a superset, so a component rejected here
  // merely takes the exact sequential path).  At most 4 + 14 rows: a fixed,
  // unrolled count, so the row reads are in flight together.
  if (eligible) {
    const int X0 = rx + bx0 - 7, n = bx1 - bx0 + 15;
    const int r0 = ry + by0 - 7, r1 = ry + by1 + 7;
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 18; j++)
      if (r0 + j <= r1) cnt += __popc(row_bits(srow[r0 + j], X0, n));
    eligible = cnt == nc;
  }
  if (!eligible) {
    v.seq = trig;
    return v;
  }
  // cleared iff some trigger of the component passes the ring test on the
  // original image (eligible pixels are >= 40 from the edges, so the
  // reference's unsigned ring-loop skips never apply).  Rings up to N <= 4
  // (larger intensities take the sequential path): the pixel's 9x9 dark
  // window read once, every ring's count from it in registers.
  for (int k = 0; k < nc && k < 4 && !v.clear; k++) {
    const int cx = rx + (k == 0 ? cxs[0] : k == 1 ? cxs[1] : k == 2 ? cxs[2] : cxs[3]);
    const int cy = ry + (k == 0 ? cys[0] : k == 1 ? cys[1] : k == 2 ? cys[2] : cys[3]);
    if (!((trow[cy][cx >> 5] >> (cx & 31)) & 1)) continue;
    uint32_t D[9];  // bit i of D[r]: pixel (cx - 4 + i, cy - 4 + r)
#pragma unroll
    for (int r = 0; r < 9; r++) D[r] = row_bits(drow[cy - 4 + r], cx - 4, 9);
    // noisefilter_count_pixel_neighbors (filters.c:256-300): count 1, then each level's ring until
    // an empty one or past N
    int count = 1;
    bool go = true;
#pragma unroll
    for (int L = 1; L <= 4; L++) {
      if (!go || L > N) break;
      const uint32_t span = ((1u << (2 * L + 1)) - 1u) << (4 - L);
      const uint32_t ends = (1u << (4 - L)) | (1u << (4 + L));
      int lc = __popc(D[4 - L] & span) + __popc(D[4 + L] & span);
#pragma unroll
      for (int r = 4 - L + 1; r <= 4 + L - 1; r++) lc += __popc(D[r] & ends);
      count += lc;
      go = lc != 0;
    }
    v.clear = count <= N;
  }
  return v;
}
__device__ __forceinline__ SmallVerdict small_verdict_rec(const uint32_t (*drow)[4],
                                                          const uint32_t (*trow)[4],
                                                          const uint32_t (*srow)[4], int rx, int ry,
                                                          int32_t gx, int32_t gy, bool trig, int N,
                                                          uint32_t rec) {
  int cxs[4], cys[4], nc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t b = (rec >> (8 * k)) & 0xFFu;
    cxs[k] = (int)(b & 15u) - 4;
    cys[k] = (int)(b >> 4) - 4;
    nc += b != 0xFFu;
  }
  return small_verdict_pixels(drow, trow, srow, rx, ry, gx, gy, trig, N, nc, cxs, cys);
}
__device__ __forceinline__ SmallVerdict small_verdict(const uint32_t (*drow)[4],
                                                      const uint32_t (*trow)[4],
                                                      const uint32_t (*srow)[4], int rx, int ry,
                                                      int32_t gx, int32_t gy, bool trig, int N) {
  uint32_t comp[9];
  flood9(drow, rx, ry, comp);
  const uint32_t rec = pack_comp(comp);
  if (rec == kNotSmall) return SmallVerdict{trig, false};  // more than 4: not eligible
  return small_verdict_rec(drow, trow, srow, rx, ry, gx, gy, trig, N, rec);
}

constexpr int kListCap = 1024;  // LDS work list of one tile (else: row loops)

#ifndef UPH_CLASSIFY_OCC
#define UPH_CLASSIFY_OCC 8
#endif
template <int FMT>
__global__ void __launch_bounds__(256, UPH_CLASSIFY_OCC) k_noise_classify(PlaneRef img, NoiseGeom g, uint8_t* scratch,
                                                        int64_t sstride, const int32_t* active,
                                                        SheetCtl* ctl, const uint32_t* bits,
                                                        int64_t bstride) {
  // XCD-aware tile order: neighbouring tiles' halos are fetched into one L2
  int bxi, byi, s;
  xcd_block(&bxi, &byi, &s);
  if (active && !active[s]) return;
  constexpr int NTX = noise_tile_w<FMT>();  // tile width
  constexpr int RWX = NTX + 2 * kHalo;       // region columns (<= 128)
  static_assert(RWX > 64 && RWX <= 128, "region rows are two 64-bit halves");
  const int32_t tx0 = bxi * NTX, ty0 = byi * kNT;
  const int32_t ox = tx0 - kHalo, oy = ty0 - kHalo;  // region origin
  const uint8_t* base = plane_ptr(img, s);
  NoisePtrs NP = noise_ptrs(g, scratch + s * sstride);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // Everything is kept as 128-bit region rows (bit = region column):
  //   drow dark (lightness < white), trow trigger (max < white; the same
  //   bits for gray planes), srow small (component <= 4 pixels)
  constexpr bool kGray = FMT == F_GRAY8;
  constexpr bool kSplit = FMT == F_RGB24;
  // interior columns [kHalo, kHalo + NTX) of a region row's halves
  constexpr uint64_t kIn0 = ~0ull << kHalo;
  constexpr uint64_t kIn1 = (1ull << (kHalo + NTX - 64)) - 1ull;
  __shared__ uint32_t drow[kRW][4];
  __shared__ uint32_t trow_s[kSplit ? kRW : 1][4];
  __shared__ uint32_t srow[kRW][4];
  __shared__ uint64_t l3[kRW][2], cand[kRW][2];
  __shared__ uint16_t wl[kListCap];
  __shared__ uint32_t crec[kListCap];  // the candidates' components (pack_comp)
  __shared__ int32_t any_dark, nwl;
  uint32_t (*trow)[4] = kSplit ? trow_s : drow;
  constexpr int B = FMT == F_GRAY8 ? 1 : FMT == F_Y400A ? 2 : 3;
  const int64_t pitch = img.P.pitch;
  if (threadIdx.x == 0) {
    any_dark = 0;
    nwl = 0;
  }
  for (int i = threadIdx.x; i < kRW * 4; i += 256) (&srow[0][0])[i] = 0;
  if constexpr (kGray) {
    // Region rows from the dark bit-plane (k_noise_bits): row ry is bits
    // [ox, ox + RWX) of plane row oy + ry, five words realigned by ox mod 32;
    // words outside the row or the image read as 0
    bool dark_here = false;
    if (threadIdx.x < kRW) {
      const int ry = threadIdx.x;
      const int32_t gy = oy + ry;
      const int32_t nwr = (g.W + 31) >> 5;
      const int32_t wb = ox >> 5;  // floor(ox / 32) (arithmetic shift)
      const int sh = ox & 31;
      uint32_t q[5] = {0u, 0u, 0u, 0u, 0u};
      if (gy >= 0 && gy < g.H) {
        const uint32_t* row = bits + s * bstride + (int64_t)gy * nwr;
#pragma unroll
        for (int j = 0; j < 5; j++)
          if (wb + j >= 0 && wb + j < nwr) q[j] = row[wb + j];
      }
      uint32_t d[4];
#pragma unroll
      for (int j = 0; j < 4; j++) d[j] = __builtin_amdgcn_alignbit(q[j + 1], q[j], sh);
      if (RWX < 128) {  // region columns >= RWX
        if (RWX <= 96) {
          d[2] &= RWX > 64 ? (1u << (RWX - 64)) - 1u : 0u;
          d[3] = 0u;
        } else {
          d[3] &= (1u << (RWX - 96)) - 1u;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; j++) drow[ry][j] = d[j];
      const uint64_t lo64 = ((uint64_t)d[1] << 32) | d[0], hi64 = ((uint64_t)d[3] << 32) | d[2];
      dark_here = ry >= kHalo && ry < kHalo + kNT && ((lo64 & kIn0) | (hi64 & kIn1));
    }
    __syncthreads();  // any_dark's reset (thread 0, above) lands first
    if (dark_here) any_dark = 1;
  } else {
    // Stage the region rows into LDS with 16-byte loads, all issued before
    // any is consumed.  Rows start 256-byte aligned, so every vector lies
    // inside its row's pitch; out-of-image pixels are masked below.
    constexpr int NV = (RWX * B + 30) / 16;             // vectors per region row
    constexpr int NLOAD = (kRW * NV + 255) / 256;       // loads per thread
    __shared__ uint4 stage[kRW][NV];
    const int64_t sb = (int64_t)ox * B;
    const int64_t a0 = sb >= 0 ? (sb & ~(int64_t)15) : -((-sb + 15) & ~(int64_t)15);
    uint4 v[NLOAD];
#pragma unroll
    for (int k = 0; k < NLOAD; k++) {
      const int i = threadIdx.x + k * 256;
      const int ry = i / NV, vi = i % NV;
      const int32_t gy = oy + ry;
      const int64_t off = a0 + 16 * vi;
      v[k] = make_uint4(0, 0, 0, 0);
      if (i < kRW * NV && gy >= 0 && gy < g.H && off >= 0 && off < pitch)
        v[k] = *reinterpret_cast<const uint4*>(base + (int64_t)gy * pitch + off);
    }
#pragma unroll
    for (int k = 0; k < NLOAD; k++) {
      const int i = threadIdx.x + k * 256;
      if (i < kRW * NV) stage[i / NV][i % NV] = v[k];
    }
    __syncthreads();
    // dark / trigger bit rows: wave w takes rows w, w+4, ...; lanes own
    // columns lane and 64+lane, each row mask is two ballots
    const int lead = (int)(sb - a0);
    bool colok[2];
    int rxc[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int rx = h * 64 + lane;
      colok[h] = (rx < RWX) & (ox + rx >= 0) & (ox + rx < g.W);
      rxc[h] = rx < RWX ? rx : 0;
    }
    bool tile_dark = false;
    for (int ry = w; ry < kRW; ry += 4) {
      const int32_t gy = oy + ry;
      const bool rowok = (gy >= 0) & (gy < g.H);
      const uint8_t* srow_b = reinterpret_cast<const uint8_t*>(stage[ry]) + lead;
      unsigned long long md[2], mt[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const bool in = colok[h] & rowok;
        if constexpr (kSplit) {
          const Px p = load_px_row<FMT>(srow_b, rxc[h]);
          md[h] = __ballot(in & (light_of(p) < g.white));
          mt[h] = __ballot(in & (dark_of(p) < g.white));
        } else {  // one channel: lightness = darkness = the gray byte
          const uint32_t v = srow_b[rxc[h] * B];
          md[h] = mt[h] = __ballot(in & (v < (uint32_t)g.white));
        }
      }
      if (lane < 4) {
        const unsigned long long q = md[lane >> 1];
        drow[ry][lane] = (uint32_t)(lane & 1 ? q >> 32 : q);
        if (kSplit) {
          const unsigned long long t = mt[lane >> 1];
          trow[ry][lane] = (uint32_t)(lane & 1 ? t >> 32 : t);
        }
      }
      if (ry >= kHalo && ry < kHalo + kNT && ((md[0] & kIn0) | (md[1] & kIn1))) tile_dark = true;
    }
    if (lane == 0 && tile_dark) any_dark = 1;
  }
  __syncthreads();
  if (!any_dark) return;
  if (UPH_DIAG_BITS(g.diag, 3) == 1) return;
  // Pixels provably in a component of >= 5 pixels: L3 = dark pixels with >= 5
  // dark pixels in their 3x3 block (all 8-adjacent to the centre, so one
  // component); large = dark & (L3 | 8-dilation of L3) (8-adjacent to an L3
  // pixel = same component).  Only the remaining dark pixels ("candidates")
  // need the restricted 9x9 flood.  Rows outside the region read as empty,
  // which can only leave pixels undecided, never mislabel them.  One thread
  // per (row, 64-bit half).
  const int hr = threadIdx.x >> 1, hh = threadIdx.x & 1;
  auto dark64 = [&](int r, int h) -> uint64_t {
    return ((uint64_t)drow[r][2 * h + 1] << 32) | drow[r][2 * h];
  };
  if (threadIdx.x < 2 * kRW) {
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int d = -1; d <= 1; d++) {
      const int r = hr + d;
      uint64_t v0 = 0, v1 = 0;
      if (r >= 0 && r < kRW) {
        v0 = dark64(r, 0);
        v1 = dark64(r, 1);
      }
      // left neighbour of column x is bit x-1 (shift up), right is x+1 (down)
      const uint64_t v = hh ? v1 : v0;
      const uint64_t Lw = hh ? (v1 << 1) | (v0 >> 63) : v0 << 1;
      const uint64_t Rw = hh ? v1 >> 1 : (v0 >> 1) | (v1 << 63);
      const uint64_t s0 = v ^ Lw ^ Rw;                          // bit 0
      const uint64_t s1 = (v & Lw) | (v & Rw) | (Lw & Rw);      // bit 1
      // c += s (c: 4 bits, <= 9; s: 2 bits)
      const uint64_t k0 = c0 & s0;
      c0 ^= s0;
      const uint64_t t1 = c1 ^ s1;
      const uint64_t k1 = (c1 & s1) | (t1 & k0);
      c1 = t1 ^ k0;
      const uint64_t k2 = c2 & k1;
      c2 ^= k1;
      c3 |= k2;
    }
    l3[hr][hh] = dark64(hr, hh) & (c3 | (c2 & (c1 | c0)));  // count >= 5: 8 | (4 & (2 | 1))
  }
  __syncthreads();
  // candidates within radius 10 of the tile (region rows [4, kRW - 4),
  // columns [4, RWX - 4)), appended to the tile's work list as
  // (row << 8 | column)
  if (threadIdx.x < 2 * kRW) {
    uint64_t c = 0;
    if (hr >= 4 && hr < kRW - 4) {
      uint64_t dil = 0;
#pragma unroll
      for (int d = -1; d <= 1; d++) {
        const uint64_t a0 = l3[hr + d][0], a1 = l3[hr + d][1];
        dil |= hh ? a1 | (a1 << 1) | (a0 >> 63) | (a1 >> 1) : a0 | (a0 << 1) | (a0 >> 1) | (a1 << 63);
      }
      // bits 4..63 of half 0, 64..RWX-5 of half 1
      c = dark64(hr, hh) & ~dil & (hh ? (1ull << (RWX - 4 - 64)) - 1ull : ~0xFull);
    }
    cand[hr][hh] = c;
    if (c) {
      int k = atomicAdd(&nwl, __popcll(c));
      while (c) {
        const int b = __ffsll((long long)c) - 1;
        c &= c - 1;
        if (k < kListCap) wl[k] = (uint16_t)((hr << 8) | (hh * 64 + b));
        k++;
      }
    }
  }
  __syncthreads();
  if (UPH_DIAG_BITS(g.diag, 3) == 2) return;
  // small bit rows: the restricted flood of every candidate
  const int ncand = nwl;
  if (ncand <= kListCap) {
    for (int i = threadIdx.x; i < ncand; i += 256) {
      const int e = wl[i], ry = e >> 8, rx = e & 0xFF;
      uint32_t comp[9];
      const bool small = flood9(drow, rx, ry, comp) <= 4;
      crec[i] = small ? pack_comp(comp) : kNotSmall;
      if (small) atomicOr(&srow[ry][rx >> 5], 1u << (rx & 31));
    }
  } else {
    for (int ry = w; ry < kRW; ry += 4) {
      unsigned long long m[2] = {0, 0};
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint64_t c = cand[ry][h];
        if (!c) continue;  // uniform
        bool small = false;
        if ((c >> lane) & 1) {
          uint32_t comp[9];
          small = flood9(drow, h * 64 + lane, ry, comp) <= 4;
        }
        m[h] = __ballot(small);
      }
      if (lane < 4) {
        const unsigned long long q = m[lane >> 1];
        srow[ry][lane] = (uint32_t)(lane & 1 ? q >> 32 : q);
      }
    }
  }
  __syncthreads();
  if (UPH_DIAG_BITS(g.diag, 3) == 3) return;
  const int N = g.intensity;
  const bool zone_tile = g.all_seq || tx0 < kZone || ty0 < kZone;  // uniform
  if (zone_tile) {
    // edge zone (and intensity > 4): every trigger there is replayed in
    // order; the tile's rows, one wave per row, lanes on the tile's columns
    for (int t = w; t < kNT; t += 4) {
#pragma unroll 1
      for (int h = 0; h < (NTX + 63) / 64; h++) {
        const int ry = kHalo + t, cx = h * 64 + lane, rx = kHalo + (cx < NTX ? cx : 0);
        const int32_t gy = oy + ry, gx = ox + rx;
        const bool trig = (trow[ry][rx >> 5] >> (rx & 31)) & 1;
        const bool zone = g.all_seq || gx < kZone || gy < kZone;
        const bool dark = (drow[ry][rx >> 5] >> (rx & 31)) & 1;
        // A trigger with >= 5 dark pixels in its 3x3 block, all outside the
        // strip the quirk triggers can bite (x < 2N-1 or y < 2N-2, N <= 4),
        // never clears: that block is connected and larger than N, so no
        // clear ever removes a pixel of it (away from the strip a clear
        // removes whole components of <= N pixels, see above), and its >= 4
        // dark ring-1 pixels keep the trigger's count above N.  Such triggers
        // are left out of the sequence (a dark border's interior).
        const bool noop = !g.all_seq && gx >= 8 && gy >= 7 && ((l3[ry][rx >> 6] >> (rx & 63)) & 1);
        wave_append(cx < NTX && dark & zone & trig & !noop, gx, gy, NP.nseq, NP.seq, g.capacity);
      }
    }
  }
  // small pixels of the tile outside the zone: one lane each, their
  // components kept from the candidate pass (the candidates hold every small
  // pixel: a pixel of a component of <= 4 has < 5 dark pixels in its 3x3 and
  // no large neighbour)
  if (ncand <= kListCap) {
    for (int b0 = 0; b0 < ncand; b0 += 256) {  // uniform trip count
      const int i = b0 + threadIdx.x;
      SmallVerdict v{false, false};
      int32_t gx = 0, gy = 0;
      if (i < ncand) {
        const uint32_t rec = crec[i];
        const int e = wl[i], ry = e >> 8, rx = e & 0xFF;
        gx = ox + rx;
        gy = oy + ry;
        const bool inside = ry >= kHalo && ry < kHalo + kNT && rx >= kHalo && rx < kHalo + NTX;
        if (rec != kNotSmall && inside && !g.all_seq && gx >= kZone && gy >= kZone) {
          const bool trig = (trow[ry][rx >> 5] >> (rx & 31)) & 1;
          v = small_verdict_rec(drow, trow, srow, rx, ry, gx, gy, trig, N, rec);
        }
      }
      wave_append(v.seq, gx, gy, NP.nseq, NP.seq, g.capacity);
      wave_append(v.clear, gx, gy, NP.nclear, NP.clear, g.capacity);
    }
    return;
  }
  // small pixels of the tile outside the zone: one lane each
  if (threadIdx.x == 0) nwl = 0;
  __syncthreads();
  // (row, 32-column chunk) per thread: 2 or 4 chunks a row
  constexpr int kChunks = (NTX + 31) / 32;
  static_assert(kChunks * kNT <= 256, "one thread per chunk");
  if (threadIdx.x < kChunks * kNT) {
    const int ry = kHalo + (threadIdx.x / kChunks), h = threadIdx.x % kChunks;
    uint32_t m = row_bits(srow[ry], kHalo + 32 * h, imin(32, NTX - 32 * h));
    if (m && !g.all_seq && oy + ry >= kZone) {
      const int32_t gx0 = ox + kHalo + 32 * h;  // column of bit 0
      if (gx0 < kZone) m &= kZone - gx0 >= 32 ? 0u : ~((1u << (kZone - gx0)) - 1u);
      if (m) {
        int k = atomicAdd(&nwl, __popc(m));
        while (m) {
          const int b = __ffs(m) - 1;
          m &= m - 1;
          if (k < kListCap) wl[k] = (uint16_t)((ry << 8) | (kHalo + 32 * h + b));
          k++;
        }
      }
    }
  }
  __syncthreads();
  const int nsmall = nwl;
  if (nsmall <= kListCap) {
    for (int b0 = 0; b0 < nsmall; b0 += 256) {  // uniform trip count
      const int i = b0 + threadIdx.x;
      SmallVerdict v{false, false};
      int32_t gx = 0, gy = 0;
      if (i < nsmall) {
        const int e = wl[i], ry = e >> 8, rx = e & 0xFF;
        gx = ox + rx;
        gy = oy + ry;
        const bool trig = (trow[ry][rx >> 5] >> (rx & 31)) & 1;
        v = small_verdict(drow, trow, srow, rx, ry, gx, gy, trig, N);
      }
      wave_append(v.seq, gx, gy, NP.nseq, NP.seq, g.capacity);
      wave_append(v.clear, gx, gy, NP.nclear, NP.clear, g.capacity);
    }
  } else {
    for (int t = w; t < kNT; t += 4) {
      const int ry = kHalo + t;
      uint32_t any = 0;
#pragma unroll
      for (int h = 0; h < kChunks; h++) any |= row_bits(srow[ry], kHalo + 32 * h, imin(32, NTX - 32 * h));
      if (!any) continue;  // uniform
#pragma unroll 1
      for (int h = 0; h < (NTX + 63) / 64; h++) {
        const int cx = h * 64 + lane, rx = kHalo + (cx < NTX ? cx : 0);
        const int32_t gy = oy + ry, gx = ox + rx;
        const bool zone = g.all_seq || gx < kZone || gy < kZone;
        const bool small = cx < NTX && !zone && ((srow[ry][rx >> 5] >> (rx & 31)) & 1);
        SmallVerdict v{false, false};
        if (small) {
          const bool trig = (trow[ry][rx >> 5] >> (rx & 31)) & 1;
          v = small_verdict(drow, trow, srow, rx, ry, gx, gy, trig, N);
        }
        wave_append(v.seq, gx, gy, NP.nseq, NP.seq, g.capacity);
        wave_append(v.clear, gx, gy, NP.nclear, NP.clear, g.capacity);
      }
    }
  }
}

template <int FMT>
__device__ __forceinline__ uint32_t* sheet_bb(const NoiseGeom& g, int s) {
  return FMT == F_GRAY8 && g.bbits ? g.bbits + s * g.bb_stride : nullptr;
}
__device__ __forceinline__ void bb_clear(uint32_t* bb, int32_t W, int32_t x, int32_t y) {
  if (bb) atomicAnd(bb + (int64_t)y * ((W + 31) >> 5) + (x >> 5), ~(1u << (x & 31)));
}

template <int FMT>
__global__ void __launch_bounds__(256) k_noise_apply(PlaneRef img, NoiseGeom g, uint8_t* scratch,
                                                     int64_t sstride, const int32_t* active,
                                                     SheetCtl* ctl) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  NoisePtrs NP = noise_ptrs(g, scratch + s * sstride);
  const uint32_t n = *NP.nclear;
  if (n > (uint32_t)g.capacity) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && ctl) atomicOr(&ctl[s].status, STATUS_NOISE_OVERFLOW);
    return;
  }
  uint8_t* base = plane_ptr(img, s);
  uint32_t* bb = sheet_bb<FMT>(g, s);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t k = NP.clear[i];
    white_px<FMT>(base + (int64_t)(k >> 16) * img.P.pitch, (int32_t)(k & 0xFFFF));
    bb_clear(bb, g.W, (int32_t)(k & 0xFFFF), (int32_t)(k >> 16));
  }
}

// In-LDS / in-global bitonic sort of n uint32 keys by one 256-thread block.
// Bitonic sort of a[0 .. n_pow2) in LDS by the whole block (blockDim.x a
// multiple of 64).  Steps whose partners lie 64 or more apart go through LDS
// with a block barrier each; the steps below 64 of a merge run in registers
// (partners in the same wave: element i belongs to lane i % 64 of one wave),
// with one barrier per merge instead of one per step.
__device__ void block_sort(uint32_t* a, int n_pow2) {
  for (int k = 2; k <= n_pow2; k <<= 1) {
    int j = k >> 1;
    for (; j >= 64; j >>= 1) {
      for (int i = threadIdx.x; i < n_pow2; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint32_t x = a[i], y = a[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __threadfence_block();
      __syncthreads();
    }
    for (int i = threadIdx.x; i < n_pow2; i += blockDim.x) {
      uint32_t x = a[i];
      const bool up = (i & k) == 0;
      for (int jj = j; jj > 0; jj >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)x, jj, 64);
        const bool lower = (i & jj) == 0;  // keeps the smaller one when sorting up
        x = lower == up ? (x < y ? x : y) : (x < y ? y : x);
      }
      a[i] = x;
    }
    __threadfence_block();
    __syncthreads();
  }
}

// Pixel k of the Chebyshev ring L (8L pixels): the two rows dy = -L, +L
// (2L+1 each), then the two columns dx = -L, +L without the corners.
__device__ __forceinline__ bool ring_pos(int L, int k, int* dx, int* dy) {
  const int row = 2 * L + 1, col = 2 * L - 1;
  if (k < row) {
    *dx = k - L;
    *dy = -L;
  } else if (k < 2 * row) {
    *dx = k - row - L;
    *dy = L;
  } else if (k < 2 * row + col) {
    *dx = -L;
    *dy = k - 2 * row - (L - 1);
  } else if (k < 2 * row + 2 * col) {
    *dx = L;
    *dy = k - 2 * row - col - (L - 1);
  } else {
    return false;
  }
  return true;
}

// Whether the reference ring loops visit (x+dx, y+dy) at level L.
__device__ __forceinline__ bool ring_member(int L, int dx, int dy, int32_t x, int32_t y) {
  return iabs(dy) == L ? x >= L : y >= L - 1;
}

// 81-bit position masks of the 9x9 window (bit p = (dy+4)*9 + dx+4): for
// ring L, its two rows (|dy| = L) and its two columns without the corners.
struct Mask81 {
  uint64_t lo;
  uint32_t hi;
};
__device__ __forceinline__ Mask81 ring_part(int L, bool rows) {
  Mask81 m{0, 0};
#pragma unroll
  for (int p = 0; p < 81; p++) {
    const int dx = p % 9 - 4, dy = p / 9 - 4;
    const int adx = iabs(dx), ady = iabs(dy);
    const bool on = rows ? (ady == L && adx <= L) : (adx == L && ady < L);
    if (on) {
      if (p < 64) m.lo |= 1ull << p;
      else m.hi |= 1u << (p - 64);
    }
  }
  return m;
}

// The blurfilter's GRAY8 bit-plane (pixel <= white, NoiseGeom::bbits) follows
// a clear: the sheet's plane `bb` (null: none), bit x of row y.
// One trigger of the raster replay for intensity N <= 4 (filters.c:309-338):
// the 9x9 window read from the frame (dark = lightness < white), rings with
// the reference loops' unsigned comparisons -- rows of ring L counted iff
// x >= L, its columns iff y >= L-1 -- and the clears written straight back.
template <int FMT>
__device__ __forceinline__ void replay_trigger4(int32_t x, int32_t y, int N, const NoiseGeom& g,
                                                uint8_t* base, int64_t pitch,
                                                const Mask81 (&rowp)[5], const Mask81 (&colp)[5],
                                                uint32_t* bb) {
  uint64_t dlo = 0;
  uint32_t dhi = 0;
  bool ctr = false;
  if constexpr (FMT == F_GRAY8) {
    // a box row as three aligned dwords (rows are pitched in whole dwords,
    // so clamped addresses stay inside the row): 27 loads instead of 81
    const int32_t c0 = x - 4;
    const int32_t d0 = c0 >= 0 ? (c0 & ~3) : -(((-c0) + 3) & ~3);  // floor to a multiple of 4
    const int32_t dmax = (int32_t)pitch - 4;
    uint32_t w[9][3];
#pragma unroll
    for (int r = 0; r < 9; r++) {
      const uint8_t* row = base + (int64_t)imin(imax(y + r - 4, 0), g.H - 1) * pitch;
#pragma unroll
      for (int j = 0; j < 3; j++)
        w[r][j] = *reinterpret_cast<const uint32_t*>(row + imin(imax(d0 + 4 * j, 0), dmax));
    }
    const int o = c0 - d0;  // 0 .. 3
#pragma unroll
    for (int p = 0; p < 81; p++) {
      const int r = p / 9, c = p % 9;
      const int32_t qx = c0 + c, qy = y + r - 4;
      const bool in = (qx >= 0) & (qy >= 0) & (qx < g.W) & (qy < g.H);
      const int b = o + c;  // byte of the row's 12
      const uint32_t wd = b < 4 ? w[r][0] : b < 8 ? w[r][1] : w[r][2];
      const uint32_t v = (wd >> (8 * (b & 3))) & 0xFFu;
      const bool dk = in & (v < g.white);
      if (p < 64) dlo |= (uint64_t)dk << p;
      else dhi |= (uint32_t)dk << (p - 64);
      if (p == 40) ctr = v < g.white;
    }
  } else if constexpr (FMT == F_RGB24) {
    // a box row (27 bytes) as eight aligned dwords, realigned to its first
    // byte: 72 loads instead of 243
    const int32_t b0 = 3 * (x - 4);
    const int32_t d0 = b0 >= 0 ? (b0 & ~3) : -(((-b0) + 3) & ~3);
    const int32_t dmax = (int32_t)pitch - 4;
    const int o = b0 - d0;  // 0 .. 3
#pragma unroll
    for (int r = 0; r < 9; r++) {
      const uint8_t* row = base + (int64_t)imin(imax(y + r - 4, 0), g.H - 1) * pitch;
      uint32_t w[8], a[7];
#pragma unroll
      for (int j = 0; j < 8; j++)
        w[j] = *reinterpret_cast<const uint32_t*>(row + imin(imax(d0 + 4 * j, 0), dmax));
#pragma unroll
      for (int j = 0; j < 7; j++) a[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], o);
#pragma unroll
      for (int c = 0; c < 9; c++) {
        const int p = 9 * r + c;
        const int32_t qx = x + c - 4, qy = y + r - 4;
        const bool in = (qx >= 0) & (qy >= 0) & (qx < g.W) & (qy < g.H);
        const int k = 3 * c;  // the pixel's first byte in the realigned row
        const Px q{(uint8_t)(a[k >> 2] >> (8 * (k & 3))), (uint8_t)(a[(k + 1) >> 2] >> (8 * ((k + 1) & 3))),
                   (uint8_t)(a[(k + 2) >> 2] >> (8 * ((k + 2) & 3)))};
        const bool dk = in & (light_of(q) < g.white);
        if (p < 64) dlo |= (uint64_t)dk << p;
        else dhi |= (uint32_t)dk << (p - 64);
        if (p == 40) ctr = dark_of(q) < g.white;
      }
    }
  } else {
#pragma unroll
    for (int p = 0; p < 81; p++) {  // unconditional clamped loads: one round trip
      const int32_t qx = x + p % 9 - 4, qy = y + p / 9 - 4;
      const bool in = (qx >= 0) & (qy >= 0) & (qx < g.W) & (qy < g.H);
      const Px q = load_px_row<FMT>(base + (int64_t)imin(imax(qy, 0), g.H - 1) * pitch,
                                    imin(imax(qx, 0), g.W - 1));
      const bool dk = in & (light_of(q) < g.white);
      if (p < 64) dlo |= (uint64_t)dk << p;
      else dhi |= (uint32_t)dk << (p - 64);
      if (p == 40) ctr = dark_of(q) < g.white;
    }
  }
  if (!ctr) return;  // cleared meanwhile
  Mask81 mem[5];
  int lc[5];
#pragma unroll
  for (int L = 1; L <= 4; L++) {
    mem[L].lo = (x >= L ? rowp[L].lo : 0ull) | (y >= L - 1 ? colp[L].lo : 0ull);
    mem[L].hi = (x >= L ? rowp[L].hi : 0u) | (y >= L - 1 ? colp[L].hi : 0u);
    lc[L] = __popcll(dlo & mem[L].lo) + __popc(dhi & mem[L].hi);
  }
  // do { lc = ring(level); count += lc; level++ } while (lc && level <= N)
  int count = 1, k = N + 1;  // k: first empty ring (N+1: none within N)
  bool open = true;
#pragma unroll
  for (int L = 1; L <= 4; L++) {
    if (open && L <= N) {
      count += lc[L];
      if (lc[L] == 0) {
        k = L;
        open = false;
      }
    }
  }
  if (count > N) return;
  // the centre and rings 1..k-1 are cleared
  white_px<FMT>(base + (int64_t)y * pitch, x);
  bb_clear(bb, g.W, x, y);
#pragma unroll
  for (int Lc = 1; Lc <= 3; Lc++) {
    if (Lc >= k) continue;
    uint64_t clo = dlo & mem[Lc].lo;
    uint32_t chi = dhi & mem[Lc].hi;
    while (clo) {
      const int p = __ffsll((long long)clo) - 1;
      clo &= clo - 1;
      white_px<FMT>(base + (int64_t)(y + p / 9 - 4) * pitch, x + p % 9 - 4);
      bb_clear(bb, g.W, x + p % 9 - 4, y + p / 9 - 4);
    }
    while (chi) {
      const int p = 64 + __ffs(chi) - 1;
      chi &= chi - 1;
      white_px<FMT>(base + (int64_t)(y + p / 9 - 4) * pitch, x + p % 9 - 4);
      bb_clear(bb, g.W, x + p % 9 - 4, y + p / 9 - 4);
    }
  }
}

// Parallel union-find over the trigger indices (parents always point to a
// smaller index, so the CAS links never form a cycle).  GLOBAL: the parents
// live in HBM and are read past the vector L1 (agent-scope atomic loads), so
// a link another wave's CAS made in L2 is seen on the next read.
template <bool GLOBAL = false>
__device__ __forceinline__ uint32_t uf_load(const uint32_t* parent, uint32_t i) {
  if constexpr (GLOBAL)
    return __hip_atomic_load(parent + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    return parent[i];
}
template <bool GLOBAL = false>
__device__ __forceinline__ uint32_t uf_find(const uint32_t* parent, uint32_t i) {
  uint32_t p = uf_load<GLOBAL>(parent, i);
  while (p != i) {
    i = p;
    p = uf_load<GLOBAL>(parent, i);
  }
  return i;
}
template <bool GLOBAL = false>
__device__ __forceinline__ void uf_union(uint32_t* parent, uint32_t a, uint32_t b) {
  for (;;) {
    a = uf_find<GLOBAL>(parent, a);
    b = uf_find<GLOBAL>(parent, b);
    if (a == b) return;
    if (a < b) {
      const uint32_t t = a;
      a = b;
      b = t;
    }
    if (atomicCAS(&parent[a], a, b) == a) return;
  }
}

// k_noise_group is one 256-thread block a sheet with ~49 KiB of LDS: a block
// that needs a whole CU's wave slots and LDS (1024 threads, 147 KiB, round
// 5) waits for a CU to drain while other streams' kernels keep them busy
// (84 ms a launch in the JPEG 2000 runner, behind the code-block decode).
// k_noise_replay blocks per sheet: enough that a lone sheet's components
// spread over the chip (C2/C4 latency: up to 16384 threads a sheet), few
// enough that a 64-sheet batch is not mostly blocks that exit (C3): about one
// block a CU over the launch, clamped to [4, 64].
static int replay_blocks(int count) {
  const int per = (256 + count - 1) / (count > 0 ? count : 1);
  return per < 4 ? 4 : per > 64 ? 64 : per;
}

// The sequential part of the noisefilter (the triggers k_noise_classify could
// not decide in parallel) for intensity N <= 4, in two kernels:
// k_noise_group (a block per sheet) orders the triggers in raster order by a
// counting sort over row buckets (then insertion sort within a bucket; a
// bucket longer than kGroupBucketMax is bitonic-sorted by the whole block in
// LDS), links those within 2N-1 by union-find and writes, per trigger in
// raster order, its key, its component's root (the component's first
// trigger) and, for a root, its component's last trigger; k_noise_replay
// (many blocks per sheet) gives each component to one thread, which replays
// its triggers in raster order.  The replay's scattered box reads then spread
// over the chip instead of one CU's address path.  Where the arrays live is
// the sheet's layout word (word 2 of its list header):
//   kNoiseNothing  nothing left to replay (no trigger, or done in k_noise_group)
//   kNoiseLds      n <= kCompCap: keys / roots / last at [0, C), [C, 2C),
//                  [2C, 3C) of the sort buffer (C = kCompCap); the sort and
//                  the links ran in LDS
//   kNoiseBig      n > kCompCap: keys in the sort buffer, roots in the seq
//                  list (free once its keys are scattered), last in the clear
//                  list (free once k_noise_apply ran); the sort and the links
//                  ran on those global arrays
// Intensity > 4 (every trigger replayed: up to W*H of them) and a bucket of
// more than kCompCap triggers take the literal raster scan by one wave inside
// k_noise_group.  No separate resolver launch: a kernel asking for 128 KiB
// of LDS waits for a nearly idle CU even when all its blocks would exit.
constexpr uint32_t kNoiseNothing = 0, kNoiseLds = 1, kNoiseBig = 2;
constexpr int kNoiseBuckets = 4096;
constexpr int kGroupBucketMax = 256;  // longer buckets: block-wide bitonic sort
constexpr int kLongList = 64;         // long buckets remembered by id (else: all scanned)
// keys, parents, bucket starts, the scan's wave sums + 3 words, the long
// bucket list (all dynamic: allow_dynamic_lds raises the limit to 160 KiB)
constexpr size_t group_lds(int threads) {
  return sizeof(uint32_t) * (2 * (size_t)(kCapPerThread * threads) + kNoiseBuckets + 1 + 16 + 3 + kLongList);
}

__device__ __forceinline__ int noise_bucket_shift(int32_t H) {
  int b = 0;
  while (((H - 1) >> b) >= kNoiseBuckets) b++;
  return b;
}

// The literal raster scan of the sorted triggers by one wave (filters.c:
// 243-348): for intensity > 4 (every trigger queued) and for a sheet whose
// triggers crowd one bucket beyond what the block can sort in LDS.  keys: n
// triggers, pow2 p2 >= n slots (LDS when p2 <= kCompCap, else the sheet's
// global sort buffer).
template <int FMT>
__device__ void noise_raster_replay(uint32_t* keys, int n, int p2, const NoiseGeom& g, const NoisePtrs& NP,
                                    uint8_t* base, int64_t pitch, uint32_t* bb) {
  for (int i = threadIdx.x; i < p2; i += blockDim.x) keys[i] = i < n ? NP.seq[i] : 0xFFFFFFFFu;
  __threadfence_block();
  __syncthreads();
  block_sort(keys, p2);
  if (threadIdx.x >= 64) return;
  const int N = g.intensity;
  const int lane = threadIdx.x;
  if (N <= 4) {
    // small intensity: the whole (2N+1)^2 box of a trigger is read in one
    // round trip (two pixels per lane) and the rings are counted from
    // registers; clears are written straight back
    const int side = 2 * N + 1, area = side * side;
    for (int idx = 0; idx < n; idx++) {
      const uint32_t key = keys[idx];
      const int32_t x = (int32_t)(key & 0xFFFF), y = (int32_t)(key >> 16);
      __threadfence_block();
      int Lv[2];
      bool dk[2], ctr = false;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int pos = h * 64 + lane;
        Lv[h] = -1;
        dk[h] = false;
        if (pos < area) {
          const int dx = pos % side - N, dy = pos / side - N;
          const int L = imax(iabs(dx), iabs(dy));
          const int32_t qx = x + dx, qy = y + dy;
          Lv[h] = L;
          const bool member = L == 0 || ring_member(L, dx, dy, x, y);
          if (member && qx >= 0 && qy >= 0 && qx < g.W && qy < g.H) {
            const Px p = load_px_row<FMT>(base + (int64_t)qy * pitch, qx);
            dk[h] = L > 0 && light_of(p) < g.white;
            if (L == 0) ctr = dark_of(p) < g.white;
          }
        }
      }
      if (!__ballot(ctr)) continue;  // cleared meanwhile
      int count = 1, level = 1, lc;
      do {
        lc = __popcll(__ballot(dk[0] && Lv[0] == level)) +
             __popcll(__ballot(dk[1] && Lv[1] == level));
        count += lc;
        level++;
      } while (lc != 0 && level <= N);
      if (count > N) continue;
      const int k = level - 1;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int pos = h * 64 + lane;
        if (pos >= area || Lv[h] >= k || (Lv[h] > 0 && !dk[h])) continue;
        const int32_t qx = x + pos % side - N, qy = y + pos / side - N;
        white_px<FMT>(base + (int64_t)qy * pitch, qx);
        bb_clear(bb, g.W, qx, qy);
      }
    }
    return;
  }
  for (int idx = 0; idx < n; idx++) {
    const uint32_t key = keys[idx];
    const int32_t x = (int32_t)(key & 0xFFFF), y = (int32_t)(key >> 16);
    __threadfence_block();
    const Px cp = load_px_row<FMT>(base + (int64_t)y * pitch, x);
    if (!(dark_of(cp) < g.white)) continue;  // cleared meanwhile
    // ring counts with the reference loops' unsigned-comparison semantics:
    // rows +-L counted iff x >= L, columns +-L (|dy| < L) counted iff y >= L-1
    // (filters.c:243-302); ring L is walked as its 8L pixels, one per lane
    int count = 1, level = 1, lc;
    do {
      lc = 0;
      for (int b = 0; b < 8 * level; b += 64) {
        int dx, dy;
        const bool in = ring_pos(level, b + lane, &dx, &dy);
        bool dark = false;
        if (in && ring_member(level, dx, dy, x, y)) {
          const int32_t qx = x + dx, qy = y + dy;
          if (qx >= 0 && qy >= 0 && qx < g.W && qy < g.H)
            dark = light_of(load_px_row<FMT>(base + (int64_t)qy * pitch, qx)) < g.white;
        }
        lc += __popcll(__ballot(dark));
      }
      count += lc;
      level++;
    } while (lc != 0 && level <= N);
    if (count > N) continue;
    // centre + rings 1..k-1 (the loop stopped at the first empty ring k)
    const int k = level - 1;
    if (lane == 0) {
      white_px<FMT>(base + (int64_t)y * pitch, x);
      bb_clear(bb, g.W, x, y);
    }
    for (int L = 1; L < k; L++) {
      for (int b = 0; b < 8 * L; b += 64) {
        int dx, dy;
        if (!ring_pos(L, b + lane, &dx, &dy) || !ring_member(L, dx, dy, x, y)) continue;
        const int32_t qx = x + dx, qy = y + dy;
        if (qx < 0 || qy < 0 || qx >= g.W || qy >= g.H) continue;
        uint8_t* row = base + (int64_t)qy * pitch;
        if (light_of(load_px_row<FMT>(row, qx)) < g.white) {
          white_px<FMT>(row, qx);
          bb_clear(bb, g.W, qx, qy);
        }
      }
    }
    __threadfence_block();
  }
}

// UPH_NOISE_CHECK (tuning builds): index checks in k_noise_group that print
// and skip the access instead of faulting; NCHK(...) is `true` otherwise.
#ifdef UPH_NOISE_CHECK
__device__ __forceinline__ bool nchk(bool ok, int tag, long long idx, unsigned n) {
  if (!ok) printf("uphip noise check: sheet %d tag %d idx %lld n %u\n", (int)blockIdx.x, tag, idx, n);
  return ok;
}
#define NCHK(ok, tag, idx) nchk((ok), (tag), (long long)(idx), n)
#else
#define NCHK(ok, tag, idx) true
#endif
// k_noise_group's ordering and linking for one sheet of n (> 0) triggers;
// BIG (n > kCompCap): keys and parents in HBM, else in LDS.  A template
// parameter, so that every pointer below has one address space (LDS through
// ds_*, HBM through global_*): no flat accesses to LDS.
template <int FMT, int T, bool BIG>
__device__ __forceinline__ void noise_group_sheet(const NoiseGeom& g, const NoisePtrs& NP, uint32_t* gk,
                                                  uint32_t* glds, uint8_t* base, int64_t pitch,
                                                  uint32_t* flag, uint32_t n, uint32_t* bb) {
  const int N = g.intensity;
  const int tid = threadIdx.x;
  const bool big = BIG;
  constexpr int kCompCap = kCapPerThread * T;
  constexpr int kGroupThreads = T;
  uint32_t* keys = big ? gk : glds;         // the sorted keys
  uint32_t* cur = glds + kCompCap;          // scatter cursors, then the long-bucket stage
  uint32_t* bc = glds + 2 * kCompCap;       // bucket starts (nb + 1)
  uint32_t* wsum = bc + kNoiseBuckets + 1;
  uint32_t& nlong = wsum[16];
  uint32_t& huge = wsum[17];
  uint32_t* longs = wsum + 19;
  const int b = noise_bucket_shift(g.H);
  const int nb = ((g.H - 1) >> b) + 1;
  const int R = 2 * N - 1;
  if (tid == 0) {
    nlong = 0u;
    huge = 0u;
  }
  for (int i = tid; i <= nb; i += kGroupThreads) bc[i] = 0;
  __syncthreads();
  for (int i = tid; i < (int)n; i += kGroupThreads) {
    if (NCHK(((NP.seq[i] >> 16) >> b) < (uint32_t)nb, 1, NP.seq[i])) atomicAdd(&bc[(NP.seq[i] >> 16) >> b], 1u);
  }
  __syncthreads();
  // exclusive scan of the nb counts: KB consecutive buckets a thread
  {
    constexpr int KB = kNoiseBuckets / kGroupThreads;
    const int b0 = KB * tid;
    uint32_t c[KB], sum = 0;
#pragma unroll
    for (int k = 0; k < KB; k++) {
      c[k] = b0 + k < nb ? bc[b0 + k] : 0u;
      sum += c[k];
      if (c[k] > (uint32_t)kGroupBucketMax) {
        const uint32_t q = atomicAdd(&nlong, 1u);
        if (q < (uint32_t)kLongList) longs[q] = (uint32_t)(b0 + k);
        // staged in LDS, or (BIG) in the clear list: a bucket past that
        // (pow2 slots) takes the literal scan
        int p2 = 1;
        while (p2 < (int)c[k]) p2 <<= 1;
        if (p2 > (BIG ? g.capacity : kCompCap)) huge = 1u;
      }
    }
    // block exclusive scan of `sum`
    uint32_t incl = sum;
    const int lane = tid & 63, wv = tid >> 6;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (int k = 0; k < wv; k++) before += wsum[k];
    uint32_t run = before + incl - sum;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KB; k++) {
      if (b0 + k < nb) {
        bc[b0 + k] = run;
        cur[b0 + k] = run;
      }
      run += c[k];
    }
    if (tid == 0) bc[nb] = n;
  }
  __syncthreads();
  if (huge) {  // one bucket beyond the LDS sort: the literal scan (never on real pages)
    int p2 = 1;
    while (p2 < (int)n) p2 <<= 1;
    if (tid == 0) *flag = kNoiseNothing;
    noise_raster_replay<FMT>(gk, (int)n, p2, g, NP, base, pitch, bb);
    return;
  }
  for (int i = tid; i < (int)n; i += kGroupThreads) {
    const uint32_t key = NP.seq[i];
    const uint32_t dst = atomicAdd(&cur[(key >> 16) >> b], 1u);
    if (NCHK(dst < n, 2, dst)) keys[dst] = key;
  }
  __threadfence_block();
  __syncthreads();
  // raster order inside each bucket: short ones by one thread each
  for (int k = tid; k < nb; k += kGroupThreads) {
    const int lo = (int)bc[k], hi = (int)bc[k + 1];
    if (hi - lo > kGroupBucketMax) continue;
    for (int i = lo + 1; i < hi; i++) {
      const uint32_t v = keys[i];
      int j = i - 1;
      while (j >= lo && keys[j] > v) {
        keys[j + 1] = keys[j];
        j--;
      }
      keys[j + 1] = v;
    }
  }
  // long ones by the whole block, one after another, staged in LDS (BIG: in
  // the clear list when longer than the LDS stage)
  const int nl = (int)nlong;
  for (int q = 0, k = 0; nl > 0 && (nl <= kLongList ? q < nl : k < nb);) {
    const int kb = nl <= kLongList ? (int)longs[q++] : k++;  // uniform
    const int lo = (int)bc[kb], len = (int)bc[kb + 1] - lo;
    if (!NCHK(kb < nb && lo + len <= (int)n, 3, kb)) continue;
    if (len <= kGroupBucketMax) continue;
    int p2 = 1;
    while (p2 < len) p2 <<= 1;
    __threadfence_block();
    __syncthreads();
    if (!BIG || p2 <= kCompCap) {
      for (int i = tid; i < p2; i += kGroupThreads) cur[i] = i < len ? keys[lo + i] : 0xFFFFFFFFu;
      __threadfence_block();
      __syncthreads();
      block_sort(cur, p2);
      for (int i = tid; i < len; i += kGroupThreads) keys[lo + i] = cur[i];
    } else {
      uint32_t* stage = NP.clear;
      for (int i = tid; i < p2; i += kGroupThreads) stage[i] = i < len ? keys[lo + i] : 0xFFFFFFFFu;
      __threadfence_block();
      __syncthreads();
      block_sort(stage, p2);
      for (int i = tid; i < len; i += kGroupThreads) keys[lo + i] = stage[i];
    }
  }
  __threadfence_block();
  __syncthreads();
  // parents: LDS, or (big) the seq list, whose keys are all scattered now
  uint32_t* par = big ? NP.seq : cur;
  for (int i = tid; i < (int)n; i += kGroupThreads) par[i] = (uint32_t)i;
  __threadfence_block();
  __syncthreads();
  // link every trigger to the earlier ones within R (rows y-R .. y)
  for (int i = tid; i < (int)n; i += kGroupThreads) {
    const uint32_t key = keys[i];
    const int32_t x = (int32_t)(key & 0xFFFF), y = (int32_t)(key >> 16);
    if (!NCHK(y < g.H && (imax(y - R, 0) >> b) < nb, 4, key)) continue;
    for (int j = (int)bc[imax(y - R, 0) >> b]; j < i; j++) {
      const uint32_t kj = keys[j];
      const int32_t xj = (int32_t)(kj & 0xFFFF), yj = (int32_t)(kj >> 16);
      if (yj >= y - R && xj >= x - R && xj <= x + R) {
        if (big) uf_union<true>(par, (uint32_t)i, (uint32_t)j);
        else uf_union(par, (uint32_t)i, (uint32_t)j);
      }
    }
  }
  __threadfence_block();
  __syncthreads();
  if (!big) {
    for (int i = tid; i < (int)n; i += kGroupThreads) {
      gk[i] = keys[i];
      gk[kCompCap + i] = uf_find(par, (uint32_t)i);
      (void)NCHK(gk[kCompCap + i] < n, 5, gk[kCompCap + i]);
    }
    __syncthreads();
    for (int i = tid; i < (int)n; i += kGroupThreads) keys[i] = 0u;
    __syncthreads();
    for (int i = tid; i < (int)n; i += kGroupThreads) atomicMax(&keys[gk[kCompCap + i]], (uint32_t)i);
    __syncthreads();
    for (int i = tid; i < (int)n; i += kGroupThreads) gk[2 * kCompCap + i] = keys[i];
    if (tid == 0) *flag = kNoiseLds;
    return;
  }
  // big: roots flattened in place (a concurrent reader sees an old parent or
  // the root, both ancestors), last trigger per root in the clear list
  uint32_t* last = NP.clear;
  for (int i = tid; i < (int)n; i += kGroupThreads) last[i] = 0u;
  for (int i = tid; i < (int)n; i += kGroupThreads) par[i] = uf_find<true>(par, (uint32_t)i);
  __threadfence_block();
  __syncthreads();
  for (int i = tid; i < (int)n; i += kGroupThreads) atomicMax(&last[par[i]], (uint32_t)i);
  __threadfence();
  __syncthreads();
  if (tid == 0) *flag = kNoiseBig;
}

template <int FMT, int T>
__global__ void __launch_bounds__(T) k_noise_group(PlaneRef img, NoiseGeom g, uint8_t* scratch,
                                                               int64_t sstride, const int32_t* active,
                                                               SheetCtl* ctl, uint32_t* sortbuf,
                                                               int64_t sort_stride) {
  constexpr int kCompCap = kCapPerThread * T;
  const int s = blockIdx.x;
  if (active && !active[s]) return;
  NoisePtrs NP = noise_ptrs(g, scratch + s * sstride);
  uint32_t* flag = NP.nclear + 2;
  const uint32_t n = *NP.nseq;
  const int N = g.intensity;
  const int tid = threadIdx.x;
#ifdef UPHIP_DIAG
  if ((g.diag & 8) && tid == 0) printf("uphip noise: sheet %d seq %u clear %u\n", s, n, *NP.nclear);
#endif
  if (n == 0 || n > (uint32_t)g.capacity) {
    if (tid == 0) {
      *flag = kNoiseNothing;
      if (n != 0 && ctl) atomicOr(&ctl[s].status, STATUS_NOISE_OVERFLOW);
    }
    return;
  }
  uint32_t* gk = sortbuf + s * sort_stride;
  extern __shared__ uint32_t glds[];
  uint8_t* base = plane_ptr(img, s);
  const int64_t pitch = img.P.pitch;
  uint32_t* bb = sheet_bb<FMT>(g, s);
  if (N > 4) {  // intensity > 4: every trigger, one wave in raster order
    int p2 = 1;
    while (p2 < (int)n) p2 <<= 1;
    if (tid == 0) *flag = kNoiseNothing;
    if (p2 <= kCompCap) noise_raster_replay<FMT>(glds, (int)n, p2, g, NP, base, pitch, bb);
    else noise_raster_replay<FMT>(gk, (int)n, p2, g, NP, base, pitch, bb);
    return;
  }
  if (n > (uint32_t)kCompCap)
    noise_group_sheet<FMT, T, true>(g, NP, gk, glds, base, pitch, flag, n, bb);
  else
    noise_group_sheet<FMT, T, false>(g, NP, gk, glds, base, pitch, flag, n, bb);
}

#ifndef UPH_REPLAY_WAVES
// > 0: k_noise_replay's register budget in waves a SIMD (A/B: 6 waves 131 ->
// 144 us a C3 launch, C4 noisefilter 0.82 -> 0.88 ms; 8 waves worse: off)
#define UPH_REPLAY_WAVES 0
#endif
#if UPH_REPLAY_WAVES > 0
#define UPH_REPLAY_ATTR __attribute__((amdgpu_waves_per_eu(UPH_REPLAY_WAVES)))
#else
#define UPH_REPLAY_ATTR
#endif
template <int FMT>
__global__ void __launch_bounds__(256) UPH_REPLAY_ATTR k_noise_replay(PlaneRef img, NoiseGeom g, uint8_t* scratch,
                                                      int64_t sstride, const int32_t* active,
                                                      const uint32_t* sortbuf, int64_t sort_stride,
                                                      int kCompCap) {
  const int s = blockIdx.y;
  if (active && !active[s]) return;
  NoisePtrs NP = noise_ptrs(g, scratch + s * sstride);
  const uint32_t n = *NP.nseq;
  const uint32_t layout = NP.nclear[2];
  if (layout == kNoiseNothing || blockIdx.x * blockDim.x >= n) return;
  const uint32_t* keys = sortbuf + s * sort_stride;
  const uint32_t* root = layout == kNoiseLds ? keys + kCompCap : NP.seq;
  const uint32_t* last = layout == kNoiseLds ? keys + 2 * kCompCap : NP.clear;
  Mask81 rowp[5], colp[5];
#pragma unroll
  for (int L = 1; L <= 4; L++) {
    rowp[L] = ring_part(L, true);
    colp[L] = ring_part(L, false);
  }
  uint8_t* base = plane_ptr(img, s);
  uint32_t* bb = sheet_bb<FMT>(g, s);
  // a few blocks per sheet walk its triggers (sheets hold far fewer triggers
  // than kCompCap: a grid sized for the cap was mostly blocks that exit)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < (int)n; i += gridDim.x * blockDim.x) {
    if (root[i] != (uint32_t)i) continue;  // not a component's first trigger
    const int end = (int)last[i];
    for (int j = i; j <= end; j++) {
      if (root[j] != (uint32_t)i) continue;
      const uint32_t key = keys[j];
      __threadfence_block();  // this thread's earlier clears are visible to its loads
      replay_trigger4<FMT>((int32_t)(key & 0xFFFF), (int32_t)(key >> 16), g.intensity, g, base,
                           img.P.pitch, rowp, colp, bb);
    }
  }
}

__global__ void k_noise_zero(uint8_t* scr, int64_t stride, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < count) {
    uint32_t* c = (uint32_t*)(scr + s * stride);
    c[0] = 0;
    c[1] = 0;
  }
}

template <int FMT>
static void launch_noise_t(const PlaneRef& img, const NoiseGeom& g, uint8_t* scr, int64_t ss,
                           const int32_t* active, SheetCtl* ctl, int count, hipStream_t st,
                           uint32_t* sortbuf, int64_t sort_stride, const uint32_t* bits_ready,
                           int64_t bits_stride) {
  constexpr int ntx = noise_tile_w<FMT>();
  dim3 grid((g.W + ntx - 1) / ntx, (g.H + kNT - 1) / kNT, count);
  NoiseGeom gd = g;
  gd.diag = diag_noise();
  uint32_t* bits = nullptr;
  int64_t bstride = 0;
  if (FMT == F_GRAY8 && bits_ready) {
    bits = const_cast<uint32_t*>(bits_ready);
    bstride = bits_stride;
  } else if (FMT == F_GRAY8) {
    // the dark bit-plane in the sort buffer's space (noise_scratch_bytes)
    const int32_t nwr = noise_bit_words(g);
    bits = sortbuf;
    bstride = sort_stride;
    const int64_t words = (int64_t)nwr * g.H;
    hipLaunchKernelGGL(k_noise_bits, dim3((unsigned)((words + 255) / 256), count), dim3(256), 0, st,
                       img, g, bits, bstride, nwr, 1.0f / (float)nwr, active);
  }
  UPH_LAUNCH_DIAG(131072, k_noise_classify<FMT>, grid, dim3(256), 0, st, img, gd, scr, ss, active, ctl,
                     bits, bstride);
  hipLaunchKernelGGL(k_noise_apply<FMT>, dim3(64, count), dim3(256), 0, st, img, g, scr, ss,
                     active, ctl);
  const int gt = group_threads(g.W, g.H);
  if (!(diag_skip() & 2)) {
    if (gt == 1024) {
      allow_dynamic_lds((const void*)k_noise_group<FMT, 1024>, group_lds(1024));
      hipLaunchKernelGGL((k_noise_group<FMT, 1024>), dim3(count), dim3(1024), group_lds(1024), st, img, gd,
                         scr, ss, active, ctl, sortbuf, sort_stride);
    } else {
      allow_dynamic_lds((const void*)k_noise_group<FMT, 256>, group_lds(256));
      hipLaunchKernelGGL((k_noise_group<FMT, 256>), dim3(count), dim3(256), group_lds(256), st, img, gd,
                         scr, ss, active, ctl, sortbuf, sort_stride);
    }
    hipLaunchKernelGGL(k_noise_replay<FMT>, dim3(replay_blocks(count), count), dim3(256), 0, st, img, g,
                       scr, ss, active, sortbuf, sort_stride, kCapPerThread * gt);
  }
}

void launch_noisefilter(const PlaneRef& img, const NoiseGeom& g, void* scratch,
                        int64_t scratch_stride, const int32_t* active, SheetCtl* ctl, int count,
                        hipStream_t st, const uint32_t* bits, int64_t bits_stride) {
  // layout of `scratch` per sheet: [noise lists][sort buffer (capacity pow2)]
  uint8_t* scr = (uint8_t*)scratch;
  const size_t lists = noise_list_bytes(g);
  uint32_t* sortbuf = (uint32_t*)(scr + lists);
  const int64_t sort_stride = scratch_stride / 4;
  hipLaunchKernelGGL(k_noise_zero, dim3((count + 255) / 256), dim3(256), 0, st, scr,
                     scratch_stride, count);
  switch (img.P.fmt) {
    case F_GRAY8:
      launch_noise_t<F_GRAY8>(img, g, scr, scratch_stride, active, ctl, count, st, sortbuf,
                              sort_stride, bits, bits_stride);
      break;
    case F_Y400A:
      launch_noise_t<F_Y400A>(img, g, scr, scratch_stride, active, ctl, count, st, sortbuf,
                              sort_stride, nullptr, 0);
      break;
    default:
      launch_noise_t<F_RGB24>(img, g, scr, scratch_stride, active, ctl, count, st, sortbuf,
                              sort_stride, nullptr, 0);
      break;
  }
}

}  // namespace uph
