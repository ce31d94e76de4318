// filters.h — geometry records and launchers of the filter kernels
// (imageprocess/filters.c) and rotation detection (imageprocess/deskew.c).
#pragma once

#include "scan.h"

namespace uph {

// ---- grayfilter (filters.c:370-402) -------------------------------------
// Tiles of scan_w x scan_h at origins (i*step_x, j*step_y) decompose exactly
// into cells of gcd(step_x, scan_w) x gcd(step_y, scan_h) pixels.
struct GrayGeom {
  int32_t W, H;
  int32_t cw, ch;      // cell size (pixels)
  int32_t ncx, ncy;    // cells covering the image
  int32_t tw, th;      // tile size in cells
  int32_t tsx, tsy;    // tile step in cells
  int32_t ntx, nty;    // tiles per row, tile rows (raster order, x fastest)
  int32_t scan_w, scan_h, step_x, step_y;
  uint8_t black_thr, abs_thr;
};
bool gray_geometry(int32_t W, int32_t H, const UphipGrayfilterParameters& p, uint8_t black_thr,
                   GrayGeom* g);
size_t gray_scratch_bytes(const GrayGeom& g);  // per sheet
// colsum (optional, zeroed by the caller): per-column gray sums over all rows
// of the image the grayfilter leaves, added into colsum[s * colsum_stride + x]
// (gray planes only).  Returns whether colsum was produced.
bool launch_grayfilter(const PlaneRef& img, const GrayGeom& g, void* scratch,
                       int64_t scratch_stride, const int32_t* active, int count, hipStream_t st,
                       uint32_t* colsum = nullptr, int64_t colsum_stride = 0);

// ---- blurfilter (filters.c:149-232) -------------------------------------
struct BlurGeom {
  int32_t W, H;
  int32_t sw, sh, step_y;
  int32_t bpr;       // blocks per row
  int32_t T;         // iterations of the top loop
  int32_t nrect;     // counted rectangles: bpr (row 0) + T*(bpr+1)
  uint8_t white;
  float intensity;
};
bool blur_geometry(int32_t W, int32_t H, const UphipBlurfilterParameters& p, uint8_t white,
                   BlurGeom* g);
size_t blur_scratch_bytes(const BlurGeom& g);
// bbits (optional): the GRAY8 bit-plane of pixels <= white of the image as it
// stands (k_decode_gray made it, the blackfilter and noisefilter kept it
// current), bb_stride words per sheet: the block counts then read it instead
// of the plane (1/8 of the bytes).
void launch_blurfilter(const PlaneRef& img, const BlurGeom& g, void* scratch,
                       int64_t scratch_stride, const int32_t* active, int count, hipStream_t st,
                       const uint32_t* bbits = nullptr, int64_t bb_stride = 0);

// ---- noisefilter (filters.c:238-338) ------------------------------------
struct NoiseGeom {
  int32_t W, H;
  int32_t intensity;   // clamped: > 4 => everything resolved sequentially
  uint8_t white;
  int32_t capacity;    // entries per list per sheet
  int32_t all_seq;
  int32_t diag;        // TEMP timing diagnostics
  // optional: the blurfilter's GRAY8 bit-plane (pixel <= white, k_decode_gray),
  // bb_stride words per sheet; every clear of the filter clears its bit too
  uint32_t* bbits;
  int64_t bb_stride;
};
bool noise_geometry(int32_t W, int32_t H, uint64_t intensity, uint8_t white, NoiseGeom* g);
size_t noise_scratch_bytes(const NoiseGeom& g);
// bits (optional): the GRAY8 dark bit-plane of the image as it stands, one
// u32 per 32 pixels, bits_stride words per sheet (k_decode_gray made it and
// the blackfilter kept it current): k_noise_bits is then skipped.
void launch_noisefilter(const PlaneRef& img, const NoiseGeom& g, void* scratch,
                        int64_t scratch_stride, const int32_t* active, SheetCtl* ctl, int count,
                        hipStream_t st, const uint32_t* bits = nullptr, int64_t bits_stride = 0);
// 32-pixel words per row of the GRAY8 dark bit-plane
inline int32_t noise_bit_words(int32_t W) { return (W + 31) >> 5; }

// ---- blackfilter (filters.c:49-127, fill.c) -----------------------------
struct BlackBar {
  Rect r;          // the bar as scanned (not clipped)
  int32_t dir;     // 0: horizontal-scan stripe, 1: vertical-scan stripe
  int32_t excluded;
};
struct BlackGeom {
  int32_t W, H;
  int32_t nbars;
  int32_t nbars_h;     // first nbars_h bars belong to the horizontal scan
  Rect hregion, vregion;  // clipped sum regions (rows of h-stripe, cols of v-stripe)
  uint8_t abs_threshold;
  uint8_t mask_max;       // image.abs_black_threshold
  uint64_t intensity;
  int32_t stack_capacity; // DFS frames per sheet
  int32_t diag;           // tuning build only: bit 16 prints replay counters
};
// Enumerates the bars exactly as blackfilter_scan's loops visit them.
bool black_geometry(int32_t W, int32_t H, const UphipBlackfilterParameters& p, uint8_t mask_max,
                    BlackGeom* g, BlackBar* bars, int max_bars);
size_t black_scratch_bytes(const BlackGeom& g);
void launch_blackfilter(const PlaneRef& img, const BlackGeom& g, const BlackBar* bars,
                        void* scratch, int64_t scratch_stride, const int32_t* active,
                        SheetCtl* ctl, int count, hipStream_t st);

// ---- rotation detection (deskew.c:48-241) -------------------------------
constexpr int kMaxAngles = 512;
struct RotTable {
  int32_t nangles;
  float angle[kMaxAngles];
  float slope[kMaxAngles];   // tanf(angle) computed on the host (deskew.c:161)
};
struct RotGeom {
  int32_t W, H;
  int32_t nedges;           // enabled edges (<= 4)
  int32_t edge_shift[4][2]; // shift per edge in enable order (left,top,right,bottom)
  int32_t scan_size;        // params.deskewScanSize
  float scan_depth;
  int32_t max_masks;
};
// peaks[(sheet*max_masks + mask)*4 + edge][angle]
void launch_rotation_peaks(const PlaneRef& img, const RotGeom& g, const RotTable* table,
                           const Rect* masks, const int32_t* mask_active, int mask_index,
                           int32_t* peaks, int count, hipStream_t st, int nangles, int max_scan,
                           int32_t* lines, float max_abs_angle);
// Scratch for the scan-line point lists of one launch_rotation_peaks call.
size_t rotation_lines_bytes(int count, int nedges, int nangles, int max_scan);
// Per-line fallback flags inside that scratch (diagnostics).
const int32_t* rotation_line_flags(const int32_t* lines, int nlines, int max_scan);
// Host: the angle sequence of detect_edge_rotation (deskew.c:153-174).
int rotation_angles(const UphipDeskewParameters& p, RotTable* t);
// Host: detect_rotation_cpu's combination of per-edge results (deskew.c:219-240)
float combine_edge_rotations(const float* rot, int count, float deviation_rad);
// vsum_ready: the v-stripe row sums are already in the scratch (k_decode_gray);
// nbits (optional): the noisefilter's dark bit-plane, cleared where fills paint.
void launch_blackfilter_impl(const PlaneRef& img, const BlackGeom& g, const BlackBar* bars,
                             void* scratch, int64_t ss, const int32_t* active, SheetCtl* ctl,
                             int count, hipStream_t st, const AxisArgs* hargs,
                             const AxisArgs* vargs, bool vsum_ready = false,
                             uint32_t* nbits = nullptr, int64_t nbits_stride = 0,
                             uint32_t* bbits = nullptr, int64_t bb_stride = 0,
                             bool rm_ready = false);
// The blackfilter's row-major match plane (RM: bit x of row y = gray <=
// mask_max, 64-bit words, black_wpr words a row) of sheet 0 inside its
// scratch; sheet s at + s * scratch_stride bytes.  k_decode_gray can write it
// (launch_blackfilter_impl's rm_ready).
uint32_t* black_rm_plane(const BlackGeom& g, void* scratch);
// GRAY8 page -> sheet plane (same size), plus on the way: the noisefilter's
// dark bit-plane (pixel < white) and the blackfilter's v-stripe row sums over
// columns [vx0, vx1] (vsum: H entries per sheet after W, vx0 > vx1 = none).
// Pages 16-byte aligned with a 16-multiple pitch.
// bbits (optional): also the blurfilter's plane of pixels <= white, same layout
// rm (optional): also the blackfilter's RM plane (pixel <= rm_max; rows of
// 2 * ceil(W / 64) words, rm_stride words a sheet, black_rm_plane)
void launch_decode_gray(const uint8_t* src, int64_t spitch, int64_t sstride, const PlaneRef& dst,
                        uint8_t white, uint32_t* bits, int64_t bits_stride, uint32_t* vsum,
                        int64_t vsum_stride, int32_t vx0, int32_t vx1, int count, hipStream_t st,
                        uint32_t* bbits = nullptr, uint32_t* rm = nullptr, int64_t rm_stride = 0,
                        uint8_t rm_max = 0);

}  // namespace uph
