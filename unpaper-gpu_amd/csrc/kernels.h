// kernels.h — launch interface of the HIP kernels (host side).
//
// Every data kernel processes a batch of frames: grid.z (or the per-sheet
// loop) selects the sheet, per-sheet arguments come from device arrays so the
// same kernels serve the single-image C-ABI ops (count = 1, host-written
// arguments) and the batch pipeline (arguments written by control kernels).
#pragma once

#include "common.h"

namespace uph {

// A plane reference: which of the two ping-pong planes of each sheet to use.
struct PlaneRef {
  Planes P;
  const SheetCtl* ctl;  // may be null: then `which` is the plane index
  int32_t which;        // with ctl: 0 = current plane, 1 = the other one
};

__device__ __forceinline__ uint8_t* plane_ptr(const PlaneRef& R, int s) {
  int k = R.which;
  if (R.ctl) k = R.which ? 1 - R.ctl[s].cur : R.ctl[s].cur;
  return R.P.base[k] + (int64_t)s * R.P.stride;
}

inline PlaneRef cur_ref(const Planes& P, const SheetCtl* ctl) { return PlaneRef{P, ctl, 0}; }
inline PlaneRef other_ref(const Planes& P, const SheetCtl* ctl) { return PlaneRef{P, ctl, 1}; }
inline PlaneRef fixed_ref(const Planes& P, int k) { return PlaneRef{P, nullptr, k}; }

// ---- per-sheet argument records -----------------------------------------
struct FillArgs {
  Rect r;           // already clipped; empty (x1<x0) = no-op
  uint8_t color[3];
  int32_t active;
};

struct CopyArgs {
  Rect a;           // clipped source area
  int32_t tx, ty;   // target coordinates of a's top-left
  int32_t active;
};

struct MaskArgs {  // apply_masks: up to UPHIP_MAX_MASKS rectangles (as given)
  int32_t n;
  uint8_t color[3];
  Rect m[UPHIP_MAX_MASKS];
};

struct MoveArgs {  // center_mask / align_mask as one gather (masks.c:222-300)
  Rect area;         // source area as given (size_of_rectangle(area) = new size)
  int32_t tx, ty;    // target top-left
  uint8_t bg[3];
  int32_t active;    // 0: identity (no pass; plane not flipped)
};

struct RotateArgs {  // deskew (deskew.c:248-286)
  Rect mask;
  float sinval, cosval;
  int32_t active;
};

// ---- launchers (kernels_blit.hip) ---------------------------------------
void launch_fill(const PlaneRef& dst, const FillArgs* args, int count, int rows_hint,
                 hipStream_t st);
void launch_copy(const PlaneRef& src, const PlaneRef& dst, const CopyArgs* args, int count,
                 int rows_hint, hipStream_t st);
void launch_apply_masks(const PlaneRef& dst, const MaskArgs* args, int count, hipStream_t st);
void launch_mirror(const PlaneRef& img, bool horizontal, bool vertical, int count,
                   hipStream_t st);
void launch_rotate90(const PlaneRef& src, const PlaneRef& dst, int direction, int count,
                     hipStream_t st);
void launch_stretch(const PlaneRef& src, const PlaneRef& dst, int interp, int count,
                    hipStream_t st);
void launch_move_rect(const PlaneRef& src, const PlaneRef& dst, const MoveArgs* args,
                      int count, hipStream_t st);
// Work folded into a gray move (k_move_rect_g16), each optional:
//  * masks: apply_masks with masks[s].m[0] (one mask) right before the move
//    (sheet_stages.c:478-488: apply_masks, then align_mask); a sheet whose
//    move is the identity is masked in place;
//  * rows: per row y, the number of pixels <= thr in columns [rx0, rx1] of
//    the sheet's resulting plane (moved, or the current one when the move is
//    the identity) at rows[s * rows_stride + y] -- detect_border's row sums
//    (masks.c:410-449), no other pass over the plane.
//  * dry: count only (rows), write nothing (not with masks); a dry pass may
//    cover only the rows [ya0, ya1) and [yb0, yb1) (empty ranges: all rows),
//    and only the sheets s with only[s] != 0 (only == nullptr: all).
struct MoveExtra {
  const MaskArgs* masks;
  uint32_t* rows;
  int64_t rows_stride;
  int32_t rx0, rx1;
  uint8_t thr;
  bool dry;
  int32_t ya0, ya1, yb0, yb1;
  const int32_t* only;
};
// center_mask (center[s]) then apply_masks (masks[s], one mask) and
// align_mask (align[s]) as one pass from src into dst (every byte of every
// sheet written): what launch_move_rect + launch_move_rect_fused with masks
// produce through an intermediate plane.  False (nothing launched) unless
// the plane is GRAY8 and pitch * H < 2^31.
bool launch_move_chain(const PlaneRef& src, const PlaneRef& dst, const MoveArgs* center,
                       const MaskArgs* masks, const MoveArgs* align, int count, hipStream_t st);
// Returns false (nothing launched) unless the plane is GRAY8.
bool launch_move_rect_fused(const PlaneRef& src, const PlaneRef& dst, const MoveArgs* args,
                            const MoveExtra& x, int count, hipStream_t st);
// max_abs_angle bounds |rotation| of every active sheet (sizes the staged
// source window; tiles whose window does not fit take a slower exact path).
// colsum (optional, zeroed by the caller for the rotated sheets): the
// output's column sums over all rows added into colsum[s * cs_stride + x];
// returns whether they were (GRAY8 cubic, staged window only).
bool launch_rotate_mask(const PlaneRef& src, const PlaneRef& dst, const RotateArgs* args,
                        int interp, int count, hipStream_t st, float max_abs_angle,
                        uint32_t* colsum = nullptr, int64_t cs_stride = 0);
// Bilinear rotation (kernels_rotlin.hip), GRAY8 and RGB24: up to two masks
// per sheet, args[m * mstride + s]; mask m >= 1 only where indep[s] (or
// indep == null).  Sheets with no active mask are left alone (not flipped).
// Returns false (nothing launched) for other formats.
struct LinWindow {
  int32_t cols, rows, stride;  // staged source window bound (floats) per tile
};
bool launch_rotate_linear(const PlaneRef& src, const PlaneRef& dst, const RotateArgs* args,
                          int nmask, int64_t mstride, const int32_t* indep, int count,
                          hipStream_t st, float max_abs_angle);
// Flip `cur` of every sheet whose args[s].active (int at byte offset) is set.
void launch_flip_if_active(SheetCtl* ctl, const int32_t* active, int64_t stride_bytes,
                           int count, hipStream_t st);

}  // namespace uph
