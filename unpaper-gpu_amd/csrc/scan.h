// scan.h — argument records and launchers of the reduction / scan kernels.
#pragma once

#include "kernels.h"

namespace uph {

enum Measure : int32_t {
  M_GRAY_SUM = 0,     // (r+g+b)/3              inverse_brightness_rect
  M_DARK_COUNT = 1,   // gray <= thr            count_pixels_within_brightness(0, thr)
  M_DARKINV_SUM = 2,  // max(r,g,b)             darkness_rect
  M_LIGHT_SUM = 3,    // min(r,g,b)             inverse_lightness_rect
};

struct AxisArgs {
  Rect region;   // clipped to the image
  uint8_t thr;
  int32_t active;
};

// One detect_edge scan (masks.c:54-100) over precomputed axis sums.
struct EdgeArgs {
  int32_t active;
  int32_t sums_offset;    // entry offset into the sheet's sums row
  int32_t extent;         // image size along the scan axis (W or H)
  int32_t cross_extent;   // image size across (H or W)
  int32_t c0, c1;         // bar extent across the scan axis (unclipped)
  int32_t b0;             // first bar's low coordinate along the scan axis
  int32_t step;           // signed shift per step
  int32_t size;           // bar size along the scan axis
  float threshold;
};

// One detect_border_edge scan (masks.c:410-449) over per-row/column dark counts.
struct BorderEdgeArgs {
  int32_t active;
  int32_t sums_offset;
  int32_t extent;         // number of valid entries (image rows or columns)
  int32_t lo, hi;         // band 0 span (inclusive, as scanned; lo > hi = empty)
  int32_t step;           // signed shift per iteration
  int32_t max_step;       // result < max_step
  int32_t threshold;
};

void launch_axis_reduce(const PlaneRef& ref, const AxisArgs* args, int axis, int meas,
                        int32_t span_x, int32_t span_y, uint32_t* out, int64_t out_stride,
                        int count, hipStream_t st);
// grid: jobs_per_sheet x count; results[s*jobs + j] = detect_edge count
// max_extent: the largest EdgeArgs/BorderEdgeArgs extent of the launch
void launch_edge_scan(const EdgeArgs* args, int jobs_per_sheet, const uint32_t* sums,
                      int64_t sums_stride, int32_t* results, int count, hipStream_t st,
                      int32_t max_extent);
// Rows [gap0, gap1) of the sums not counted (gap0 >= gap1: none): a sheet
// whose scan reaches them before a hit gets need[s] = 1 and result 0, to be
// scanned again once they are.  only (optional): the sheets to scan.
void launch_border_scan(const BorderEdgeArgs* args, int jobs_per_sheet, const uint32_t* sums,
                        int64_t sums_stride, int32_t* results, int count, hipStream_t st,
                        int32_t max_extent, int32_t gap0 = 0, int32_t gap1 = 0,
                        int32_t* need = nullptr, const int32_t* only = nullptr);

}  // namespace uph
