// pipeline.hip — the batch sheet pipeline: src/core/sheet_stages.c:44-696 for
// a whole batch of sheets at once (the MI355X-native peer of lib/batch_worker.c
// running process_sheet, sheet_process.c:134, per job).
//
// Everything that decides SIZES depends only on the options and the input
// geometry, so it is planned on the host once per batch shape (bars of the
// blackfilter, layout points, outside masks, wipe rectangles, plane sizes).
// Everything that depends on PIXELS (masks, rotations, borders, fills) stays
// in HBM: small per-sheet control kernels turn detection results into the
// arguments of the next data kernel, so a batch runs start to finish without
// a host round trip.  One launch per stage covers every sheet (grid.z).
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "filters.h"
#include "jpeg_enc.h"
#include "libm_glibc.h"
#include "runtime.h"

namespace uph {

void launch_fill_thr(const PlaneRef& dst, const FillArgs* args, int count, int rows_hint,
                     uint8_t thr, hipStream_t st);
void launch_copy_thr(const PlaneRef& src, const PlaneRef& dst, const CopyArgs* args, int count,
                     int rows_hint, uint8_t thr, hipStream_t st);
void launch_apply_masks_thr(const PlaneRef& dst, const MaskArgs* args, int count, uint8_t thr,
                            hipStream_t st);
void launch_mirror_oop(const PlaneRef& src, const PlaneRef& dst, bool h, bool v, uint8_t thr,
                       int count, hipStream_t st);
void launch_rotate90_thr(const PlaneRef& src, const PlaneRef& dst, int direction, uint8_t thr,
                         int count, hipStream_t st);
void launch_stretch_thr(const PlaneRef& src, const PlaneRef& dst, int interp, uint8_t thr,
                        int count, hipStream_t st);
void launch_shift(const PlaneRef& src, const PlaneRef& dst, int dx, int dy, const uint8_t bg[3],
                  uint8_t thr, int count, hipStream_t st);

// ---------------------------------------------------------------------------
// control kernels (one thread per sheet)
// ---------------------------------------------------------------------------
__global__ void k_ctl_init(SheetCtl* ctl, int count, int32_t npoints, UphipPoint p0, UphipPoint p1) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  SheetCtl& c = ctl[s];
  c.cur = 0;
  c.status = 0;
  c.point_count = npoints;
  c.mask_count = 0;
  c.points[0] = p0;
  c.points[1] = p1;
  for (int i = 0; i < UPHIP_MAX_PAGES; i++) c.rotation[i] = 0.0f;
}

// Folds every sheet's status into the batch's sticky word at the end of a
// run: k_ctl_init clears the per-sheet words at the start of the next run,
// so without this a failure in an earlier of several runs enqueued before
// one uphip_batch_wait would be lost.
__global__ void k_status_fold(const SheetCtl* ctl, int count, int32_t* sticky) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < count && ctl[s].status) atomicOr(sticky, ctl[s].status);
}

// The encode sources of a batch's output pages: page i = output page i % oc
// of sheet i / oc, in the plane that holds the sheet (jpeg_enc.h)
__global__ void k_jenc_sources(const SheetCtl* ctl, const uint8_t* p0, const uint8_t* p1,
                               int64_t pitch, int64_t stride, int oc, int64_t page_bytes,
                               JencImage* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = i / oc, j = i - s * oc;
  const uint8_t* base = (ctl[s].cur & 1) ? p1 : p0;
  out[i] = JencImage{base + (int64_t)s * stride + (int64_t)j * page_bytes, pitch};
}

__global__ void k_flip_all(SheetCtl* ctl, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < count) ctl[s].cur ^= 1;
}

struct MaskAssembleArgs {
  UphipMaskDetectionParameters p;
  int32_t W, H, npoints, assign;
};

// detect_mask / detect_masks_cpu (masks.c:107-209) from the four edge counts
__global__ void k_mask_assemble(SheetCtl* ctl, const int32_t* edges, MaskAssembleArgs a,
                                int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  SheetCtl& c = ctl[s];
  const UphipMaskDetectionParameters& p = a.p;
  int32_t valid = 0;
  for (int i = 0; i < a.npoints; i++) {
    const int32_t* e = edges + ((int64_t)s * a.npoints + i) * 4;
    const UphipPoint o = c.points[i];
    Rect m;
    if (p.scan_direction.horizontal) {
      m.x0 = o.x - (p.scan_step.horizontal * e[0]) - p.scan_size.width / 2;
      m.x1 = o.x + (p.scan_step.horizontal * e[1]) + p.scan_size.width / 2;
    } else {
      m.x0 = 0;
      m.x1 = a.W - 1;
    }
    if (p.scan_direction.vertical) {
      m.y0 = o.y - (p.scan_step.vertical * e[2]) - p.scan_size.height / 2;
      m.y1 = o.y + (p.scan_step.vertical * e[3]) + p.scan_size.height / 2;
    } else {
      m.y0 = 0;
      m.y1 = a.H - 1;
    }
    const int32_t mw = iabs(m.x0 - m.x1) + 1, mh = iabs(m.y0 - m.y1) + 1;
    if ((p.minimum_width != -1 && mw < p.minimum_width) ||
        (p.maximum_width != -1 && mw > p.maximum_width)) {
      m.x0 = o.x - p.maximum_width / 2;
      m.x1 = o.x + p.maximum_width / 2;
    }
    if ((p.minimum_height != -1 && mh < p.minimum_height) ||
        (p.maximum_height != -1 && mh > p.maximum_height)) {
      m.y0 = o.y - p.maximum_height / 2;
      m.y1 = o.y + p.maximum_height / 2;
    }
    c.masks[i] = from_rect(m);
    if (!(m.x0 == -1 && m.y0 == -1 && m.x1 == -1 && m.y1 == -1)) valid++;
  }
  if (a.assign) c.mask_count = valid;
}

// masks[i] -> a Rect array + active flags for the rotation-peak kernel
// only (may be null): sheets outside it are marked inactive
__global__ void k_mask_pick(const SheetCtl* ctl, int i, Rect* out, int32_t* active, int count,
                            const int32_t* only) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  out[s] = to_rect(ctl[s].masks[i]);
  active[s] = i < ctl[s].mask_count && (!only || only[s]);
}

// Two masks rotated in one launch (the double layout): the reference detects
// and deskews mask 1 after deskewing mask 0 (sheet_stages.c:401-412).  Doing
// both detections first and both rotations from the same image is the same
// thing unless deskew 0 changes a pixel that mask 1's detection or rotation
// reads: detection reads only pixels inside its mask (deskew.c:127-131), and
// the rotation the source window of its mask (a rotated rectangle, bounded
// here by its corners with two taps of margin either side).  dep[s] = 1 for
// the sheets where that may happen: mask 1 is then detected and rotated again
// after mask 0 (second pass); indep[s] = 1 where mask 1 rotates in the first.
__global__ void k_rot_independent(const SheetCtl* ctl, const RotateArgs* args, int64_t mstride,
                                  int32_t* indep, int32_t* dep, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  const SheetCtl& c = ctl[s];
  const RotateArgs a0 = args[s], a1 = args[mstride + s];
  bool d = false;
  if (c.mask_count >= 2 && a0.active) {
    const Rect m0 = normalize(to_rect(c.masks[0])), m1 = normalize(to_rect(c.masks[1]));
    auto meets = [](const Rect& p, const Rect& q) {
      return p.x0 <= q.x1 && q.x0 <= p.x1 && p.y0 <= q.y1 && q.y0 <= p.y1;
    };
    d = meets(m0, m1);
    if (!d && a1.active) {
      // mask 1's source footprint is a rotated rectangle: in source space
      // (deskew.c:264-268) the point of mask pixel (u, v) is C + (u - tcx) e_u
      // + (v - tcy) e_v with e_u = (cos, -sin), e_v = (sin, cos).  It meets
      // mask 0 unless an axis of either separates them (x, y, e_u, e_v);
      // 4 px of margin cover the interpolation taps and float rounding.
      const Rect nm = normalize(a1.mask);
      const int32_t sw = nm.x1 - nm.x0 + 1, sh = nm.y1 - nm.y0 + 1;
      const float scx = nm.x0 + sw / 2.0f, scy = nm.y0 + sh / 2.0f;
      const float tcx = 0 + sw / 2.0f, tcy = 0 + sh / 2.0f;
      const float cs = a1.cosval, sn = a1.sinval, mg = 4.0f;
      float mnx = 3.0e38f, mxx = -3.0e38f, mny = 3.0e38f, mxy = -3.0e38f;
      for (int k = 0; k < 4; k++) {
        const int32_t u = k & 1 ? sw - 1 : 0, v = k & 2 ? sh - 1 : 0;
        const float X = scx + (u - tcx) * cs + (v - tcy) * sn;
        const float Y = scy + (v - tcy) * cs - (u - tcx) * sn;
        mnx = fminf(mnx, X);
        mxx = fmaxf(mxx, X);
        mny = fminf(mny, Y);
        mxy = fmaxf(mxy, Y);
      }
      bool sep = mxx + mg < (float)m0.x0 || mnx - mg > (float)m0.x1 || mxy + mg < (float)m0.y0 ||
                 mny - mg > (float)m0.y1;
      if (!sep) {
        // mask 0's corners on the footprint's own axes
        float au = 3.0e38f, bu = -3.0e38f, av = 3.0e38f, bv = -3.0e38f;
        for (int k = 0; k < 4; k++) {
          const float dx = (float)(k & 1 ? m0.x1 : m0.x0) - scx;
          const float dy = (float)(k & 2 ? m0.y1 : m0.y0) - scy;
          const float pu = dx * cs - dy * sn, pv = dx * sn + dy * cs;
          au = fminf(au, pu);
          bu = fmaxf(bu, pu);
          av = fminf(av, pv);
          bv = fmaxf(bv, pv);
        }
        sep = bu + mg < -tcx || au - mg > (sw - 1) - tcx || bv + mg < -tcy || av - mg > (sh - 1) - tcy;
      }
      d = !sep;
    }
  }
  dep[s] = d;
  indep[s] = !d;
}

// flip every sheet the two-mask launch rotated
// Zero the first n column sums of the sheets whose rotation is active (the
// rotate kernel accumulates theirs; the others keep the previous scan's).
__global__ void k_zero_sums_if_active(const RotateArgs* args, uint32_t* sums, int64_t stride,
                                      int32_t n) {
  const int s = blockIdx.y;
  if (!args[s].active) return;
  for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    sums[s * stride + i] = 0;
}

__global__ void k_flip_rot2(SheetCtl* ctl, const RotateArgs* args, int64_t mstride,
                            const int32_t* indep, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  if (args[s].active || (args[mstride + s].active && indep[s])) ctl[s].cur ^= 1;
}

struct RotCombo {
  float result, sinv, cosv;
};

struct RotSelectArgs {
  int32_t nangles, nedges;
  int32_t negate[4];     // top/bottom edges are negated (deskew.c:197,211)
  int32_t max_masks, mask_index;
  float deviation_rad;
  UphipRectangle dummy;
};

// detect_edge_rotation's argmax + detect_rotation_cpu's combination -> RotateArgs
// for deskew.  <= 2 edges: the host-computed table (host libm); > 2 edges:
// deskew.c:219-240 and :260-261 on the device with glibc's sinf/cosf/powf
// restated bit for bit (libm_glibc.h).  `only`
// only (may be null): other sheets get an inactive RotateArgs and keep their ctl.
// One wave per sheet: the lanes scan the angles in strides, then a wave
// reduction keeps the largest peak and, among equal ones, the first angle --
// the reference loop's `if (peak > max_peak)` from max_peak = 0 (an edge with
// no positive peak keeps angle 0).
__global__ void __launch_bounds__(64) k_rot_select(SheetCtl* ctl, const int32_t* peaks,
                                                   const RotTable* table, const RotCombo* combo,
                                                   RotSelectArgs a, RotateArgs* out, int count,
                                                   const int32_t* only, const uint32_t* pow2,
                                                   int npow2) {
  const int s = blockIdx.x, lane = threadIdx.x;
  if (s >= count) return;
  if (only && !only[s]) {
    if (lane == 0) out[s].active = 0;
    return;
  }
  SheetCtl& c = ctl[s];
  const int i = a.mask_index;
  const bool active = i < c.mask_count;
  int idx[4] = {0, 0, 0, 0};
  for (int e = 0; e < a.nedges; e++) {
    const int32_t* pk = peaks + (((int64_t)s * a.max_masks + i) * 4 + e) * a.nangles;
    int best = 0, bi = 0;
    for (int k = lane; k < a.nangles; k += 64) {
      const int v = pk[k];
      if (v > best) {
        best = v;
        bi = k;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const int ob = __shfl_xor(best, o, 64), oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    idx[e] = best > 0 ? bi : 0;
  }
  if (lane != 0) return;
  RotCombo r;
  if (a.nedges <= 2) {
    int key = 0;
    if (a.nedges >= 1) key = idx[0];
    if (a.nedges == 2) key = idx[0] * a.nangles + idx[1];
    r = combo[key];
  } else {
    // > 2 edges: the reference's float expressions in its order, IEEE division
    // and square root, glibc's powf(d, 2) and sinf/cosf (libm_glibc.h)
    float rot[4], total = 0.0f;
    for (int e = 0; e < a.nedges; e++) {
      const float v = table->angle[idx[e]];
      rot[e] = a.negate[e] ? -v : v;
      total += rot[e];
    }
    const float avg = __fdiv_rn(total, (float)a.nedges);
    float t2 = 0.0f;
    for (int e = 0; e < a.nedges; e++) t2 += glibc::pow2(rot[e] - avg, pow2, npow2);
    r.result = __fsqrt_rn(t2) <= a.deviation_rad ? avg : 0.0f;
    r.sinv = glibc::sinf(-r.result);
    r.cosv = glibc::cosf(-r.result);
  }
  if (i < UPHIP_MAX_PAGES) c.rotation[i] = active ? r.result : 0.0f;
  RotateArgs ra;
  ra.mask = to_rect(c.masks[i]);
  ra.sinval = r.sinv;
  ra.cosval = r.cosv;
  ra.active = active && r.result != 0.0f;
  out[s] = ra;
}

// center_mask (masks.c:222-249) for mask i -> MoveArgs
__global__ void k_center_args(const SheetCtl* ctl, int i, int32_t W, int32_t H, UphipPixel bg,
                              MoveArgs* out, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  const SheetCtl& c = ctl[s];
  MoveArgs m;
  m.area = to_rect(c.masks[i]);
  const int32_t sw = iabs(m.area.x0 - m.area.x1) + 1, sh = iabs(m.area.y0 - m.area.y1) + 1;
  m.tx = c.points[i].x - sw / 2;
  m.ty = c.points[i].y - sh / 2;
  m.bg[0] = bg.r;
  m.bg[1] = bg.g;
  m.bg[2] = bg.b;
  const Rect na = rect_from_size(m.tx, m.ty, sw, sh);
  const Rect img{0, 0, W - 1, H - 1};
  bool active = i < c.mask_count && point_in(na.x0, na.y0, img) && point_in(na.x1, na.y1, img);
  // identity move: area inside the image, normalised, and target == origin
  const Rect n = normalize(m.area);
  const Rect cl = clip(m.area, W, H);
  if (active && n.x0 == m.area.x0 && n.y0 == m.area.y0 && cl.x0 == n.x0 && cl.y0 == n.y0 &&
      cl.x1 == n.x1 && cl.y1 == n.y1 && m.tx == n.x0 && m.ty == n.y0)
    active = false;
  m.active = active;
  out[s] = m;
}

struct BorderAssembleArgs {
  int32_t W, H, nout, cap;
  Rect outside[UPHIP_MAX_PAGES];
  int32_t horizontal, vertical, align;
  UphipMaskAlignmentParameters ap;
  uint8_t mask_color[3];
  uint8_t bg[3];
};

// detect_border + border_to_mask + apply_masks args + align_mask args
// (masks.c:351-488, sheet_stages.c:480-499)
__global__ void k_border_assemble(SheetCtl* ctl, const int32_t* res, BorderAssembleArgs a,
                                  MaskArgs* masks_out, MoveArgs* move_out, int count) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= count) return;
  SheetCtl& c = ctl[s];
  MaskArgs& ma = masks_out[s];
  ma.n = a.nout;
  ma.color[0] = a.mask_color[0];
  ma.color[1] = a.mask_color[1];
  ma.color[2] = a.mask_color[2];
  for (int i = 0; i < a.nout; i++) {
    const Rect o = a.outside[i];
    const int32_t* r = res + ((int64_t)s * a.nout + i) * 4;
    int32_t left = o.x0, top = o.y0, right = a.W - o.x1, bottom = a.H - o.y1;
    if (a.horizontal) {
      left += r[0];
      right += r[1];
    }
    if (a.vertical) {
      top += r[2];
      bottom += r[3];
    }
    const Rect m{left, top, a.W - right - 1, a.H - bottom - 1};
    c.border_masks[i] = from_rect(m);
    ma.m[i] = m;
    // align_mask_cpu target (masks.c:265-290)
    const int32_t iw = iabs(m.x0 - m.x1) + 1, ih = iabs(m.y0 - m.y1) + 1;
    int32_t tx, ty;
    if (a.ap.alignment.left) tx = o.x0 + a.ap.margin.horizontal;
    else if (a.ap.alignment.right) tx = o.x1 - iw - a.ap.margin.horizontal;
    else tx = (o.x0 + o.x1 - iw) / 2;
    if (a.ap.alignment.top) ty = o.y0 + a.ap.margin.vertical;
    else if (a.ap.alignment.bottom) ty = o.y1 - ih - a.ap.margin.vertical;
    else ty = (o.y0 + o.y1 - ih) / 2;
    MoveArgs mv;
    mv.area = m;
    mv.tx = tx;
    mv.ty = ty;
    mv.bg[0] = a.bg[0];
    mv.bg[1] = a.bg[1];
    mv.bg[2] = a.bg[2];
    const Rect n = normalize(m);
    const Rect cl = clip(m, a.W, a.H);
    const bool identity = n.x0 == m.x0 && n.y0 == m.y0 && cl.x0 == n.x0 && cl.y0 == n.y0 &&
                          cl.x1 == n.x1 && cl.y1 == n.y1 && tx == n.x0 && ty == n.y0;
    mv.active = a.align && !identity;
    move_out[(int64_t)i * a.cap + s] = mv;
  }
}

}  // namespace uph

using namespace uph;

// ===========================================================================
// The batch object
// ===========================================================================
struct UphipBatch {
  UphipOptions o;
  UphipBatchGeometry geo;
  int device = 0;
  hipStream_t st = nullptr;
  int cap = 0, n_in = 1;
  size_t dev_bytes = 0;                // device memory this batch allocated
  // geometry (host-planned)
  int32_t rp_w = 0, rp_h = 0;          // page after pre_rotate
  int32_t sheet_w = 0, sheet_h = 0;    // after decode
  int32_t W = 0, H = 0;                // processing size (after pre ops)
  int32_t out_w = 0, out_h = 0;        // after post ops
  int32_t work_fmt = F_GRAY8;
  int32_t out_fmt = F_GRAY8;           // saved format
  int32_t max_w = 0, max_h = 0;
  int64_t in_pitch = 0, in_page_stride = 0;
  int64_t pitch = 0, plane_stride = 0;
  int64_t out_pitch = 0, out_stride = 0;
  uint8_t* inputs = nullptr;
  uint8_t* planes[2] = {nullptr, nullptr};
  uint8_t* out = nullptr;   // only when out_fmt != work_fmt
  SheetCtl* ctl = nullptr;
  // layout
  std::vector<UphipPoint> points;
  std::vector<Rect> outside;
  UphipMaskDetectionParameters mask_params;
  UphipBlackfilterParameters black_params;
  // scratch
  uint8_t* scr = nullptr;
  int64_t scr_stride = 0;
  uint8_t* rot_page = nullptr;   // pre_rotate temp pages
  // device argument arrays (uniform per batch or written by control kernels)
  std::vector<void*> allocs;
  // stage boundary events of every run since the last kernel_times() query
  std::vector<std::vector<std::pair<const char*, hipEvent_t>>> runs;
  std::vector<std::string> time_names;
  bool timing = false;                 // uphip_batch_set_timing
  int32_t* sticky = nullptr;           // OR of every sheet status since the last wait
  // geometry records
  BlackGeom bgeo{};
  BlackBar* dbars = nullptr;
  AxisArgs *black_h = nullptr, *black_v = nullptr;
  NoiseGeom ngeo{};
  BlurGeom blgeo{};
  GrayGeom ggeo{};
  RotTable table{};
  RotTable* dtable = nullptr;
  RotCombo* dcombo = nullptr;
  uint32_t* dpow2 = nullptr;           // > 2 edges: glibc powf(x, 2) exceptions (libm_glibc.h)
  int npow2 = 0;
  int max_scan = 0;
  float max_angle = 0.0f;  // largest |angle| of the scan table (rotation bound)
  int32_t* peaks = nullptr;
  int32_t* rot_lines = nullptr;  // scan-line point lists (k_rot_points)
  Rect* pick_mask = nullptr;
  int32_t* pick_active = nullptr;
  RotateArgs* rot_args = nullptr;      // [UPHIP_MAX_PAGES][cap]
  int32_t* rot_indep = nullptr;        // two-mask launch: mask 1 independent of deskew 0
  int32_t* rot_dep = nullptr;          // ... or redone after it
  uint32_t* nbits = nullptr;           // GRAY8 noisefilter dark bit-plane (k_decode_gray)
  int64_t nbits_stride = 0;            // words per sheet (also bbits')
  uint32_t* bbits = nullptr;           // GRAY8 blurfilter bit-plane, pixel <= white (k_decode_gray)
  MoveArgs* move_args = nullptr;      // cap * MAX_PAGES
  int32_t* border_need = nullptr;     // cap: the chained border scan needs the middle rows
  MaskArgs* border_mask_args = nullptr;
  int32_t* edge_res = nullptr;        // cap * npoints * 4
  int32_t* border_res = nullptr;      // cap * nout * 4
  uint32_t* sums = nullptr;           // cap * sums_stride
  int64_t sums_stride = 0;
  // per-stage prepared uniform args
  struct Prepared;
  std::vector<std::string> names;
  std::vector<float> times;
  int last_count = 0;
  // argument blocks uploaded by the first run and reused (the launch sequence
  // is a pure function of options + geometry, so run k's i-th block equals
  // run 0's i-th block)
  std::vector<void*> cache;
  size_t cache_pos = 0;
  // GPU JPEG output branch (uphip_batch_encode_jpeg_async)
  JencContext* jenc = nullptr;
  int jenc_pages = 0;
};

namespace {

template <class T>
T* dalloc(UphipBatch* b, size_t n) {
  void* p = nullptr;
  if (!UPH_HIP(hipMalloc(&p, sizeof(T) * (n ? n : 1)))) return nullptr;
  b->allocs.push_back(p);
  b->dev_bytes += sizeof(T) * (n ? n : 1);
  return (T*)p;
}

// upload a host block once (first run) and hand out the same device copy on
// every later run at the same point of the launch sequence
void* upload_cached(UphipBatch* b, const void* host, size_t bytes) {
  if (b->cache_pos < b->cache.size()) return b->cache[b->cache_pos++];
  void* d = nullptr;
  if (!UPH_HIP(hipMalloc(&d, bytes ? bytes : 1))) return nullptr;
  b->allocs.push_back(d);
  b->dev_bytes += bytes ? bytes : 1;
  if (host) UPH_HIP(hipMemcpy(d, host, bytes, hipMemcpyHostToDevice));
  b->cache.push_back(d);
  b->cache_pos++;
  return d;
}

// replicate one argument record for every sheet of the batch
template <class T>
T* replicate(UphipBatch* b, const T& v) {
  std::vector<T> h((size_t)b->cap, v);
  return (T*)upload_cached(b, h.data(), sizeof(T) * h.size());
}

bool is_gray_px(UphipPixel p) { return p.r == p.g && p.g == p.b; }

int compare_sizes_h(int32_t aw, int32_t ah, int32_t bw, int32_t bh) {
  if (ah == bh && aw == bw) return 0;
  return imin(ah, aw) < imin(bh, bw) ? -1 : 1;
}

Planes planes_of(UphipBatch* b, int32_t w, int32_t h) {
  Planes P;
  P.base[0] = b->planes[0];
  P.base[1] = b->planes[1];
  P.pitch = b->pitch;
  P.stride = b->plane_stride;
  P.W = w;
  P.H = h;
  P.fmt = b->work_fmt;
  P.count = b->cap;
  return P;
}

void mark(UphipBatch* b, const char* name) {
  if (!b->timing) return;
  if (b->runs.empty()) return;
  hipEvent_t e;
  hipEventCreate(&e);
  hipEventRecord(e, b->st);
  b->runs.back().push_back({name, e});
}

void flip_all(UphipBatch* b, int count) {
  hipLaunchKernelGGL(k_flip_all, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl, count);
}

}  // namespace

// ---------------------------------------------------------------------------
// Planning
// ---------------------------------------------------------------------------
static bool plan(UphipBatch* b) {
  const UphipOptions& o = b->o;
  const int n = b->n_in;
  b->rp_w = b->geo.page_width;
  b->rp_h = b->geo.page_height;
  if (o.pre_rotate != 0) std::swap(b->rp_w, b->rp_h);
  // decode: input_size = coerce(sheet_size, (page_w * n, page_h))
  b->sheet_w = o.sheet_size.width == -1 ? b->rp_w * n : o.sheet_size.width;
  b->sheet_h = o.sheet_size.height == -1 ? b->rp_h : o.sheet_size.height;
  // working plane: GRAY8 is exact when every colour written is gray
  const bool gray_in = b->geo.page_format != UPHIP_FMT_RGB24;
  b->work_fmt = (gray_in && is_gray_px(o.sheet_background) && is_gray_px(o.mask_color)) ? F_GRAY8
                                                                                       : F_RGB24;
  // pre ops sizes
  int32_t w = b->sheet_w, h = b->sheet_h;
  b->max_w = w;
  b->max_h = h;
  {
    int32_t sw = o.stretch_size.width == -1 ? w : o.stretch_size.width;
    int32_t sh = o.stretch_size.height == -1 ? h : o.stretch_size.height;
    sw *= o.pre_zoom_factor;
    sh *= o.pre_zoom_factor;
    if (compare_sizes_h(w, h, sw, sh) != 0) {
      w = sw;
      h = sh;
    }
    b->max_w = imax(b->max_w, w);
    b->max_h = imax(b->max_h, h);
    if (o.page_size.width != -1 || o.page_size.height != -1) {
      const int32_t pw = o.page_size.width == -1 ? w : o.page_size.width;
      const int32_t ph = o.page_size.height == -1 ? h : o.page_size.height;
      if (compare_sizes_h(w, h, pw, ph) != 0) {
        const float hr = (float)pw / (float)w, vr = (float)ph / (float)h;
        int32_t ssw, ssh;
        if (hr < vr) {
          ssw = pw;
          ssh = (int32_t)(h * hr);
        } else if (vr < hr) {
          ssw = (int32_t)(w * vr);
          ssh = ph;
        } else {
          ssw = pw;
          ssh = ph;
        }
        b->max_w = imax(b->max_w, ssw);
        b->max_h = imax(b->max_h, ssh);
        w = pw;
        h = ph;
      }
    }
  }
  b->W = w;
  b->H = h;
  b->max_w = imax(b->max_w, w);
  b->max_h = imax(b->max_h, h);
  // post ops sizes
  int32_t ow = w, oh = h;
  if (o.post_rotate != 0) std::swap(ow, oh);
  b->max_w = imax(b->max_w, ow);
  b->max_h = imax(b->max_h, oh);
  {
    int32_t sw = o.post_stretch_size.width == -1 ? ow : o.post_stretch_size.width;
    int32_t sh = o.post_stretch_size.height == -1 ? oh : o.post_stretch_size.height;
    sw *= o.post_zoom_factor;
    sh *= o.post_zoom_factor;
    if (compare_sizes_h(ow, oh, sw, sh) != 0) {
      ow = sw;
      oh = sh;
    }
    b->max_w = imax(b->max_w, ow);
    b->max_h = imax(b->max_h, oh);
    if (o.post_page_size.width != -1 || o.post_page_size.height != -1) {
      const int32_t pw = o.post_page_size.width == -1 ? ow : o.post_page_size.width;
      const int32_t ph = o.post_page_size.height == -1 ? oh : o.post_page_size.height;
      if (compare_sizes_h(ow, oh, pw, ph) != 0) {
        const float hr = (float)pw / (float)ow, vr = (float)ph / (float)oh;
        int32_t ssw, ssh;
        if (hr < vr) {
          ssw = pw;
          ssh = (int32_t)(oh * hr);
        } else if (vr < hr) {
          ssw = (int32_t)(ow * vr);
          ssh = ph;
        } else {
          ssw = pw;
          ssh = ph;
        }
        b->max_w = imax(b->max_w, ssw);
        b->max_h = imax(b->max_h, ssh);
        ow = pw;
        oh = ph;
      }
    }
  }
  b->out_w = ow;
  b->out_h = oh;
  b->max_w = imax(b->max_w, ow);
  b->max_h = imax(b->max_h, oh);
  if (b->W <= 0 || b->H <= 0 || b->out_w <= 0 || b->out_h <= 0) return fail("batch: empty sheet");
  // output format (sheet_stages.c:536-552 + saveImage mapping, file.c:193-200)
  int32_t of = o.output_pixel_format == UPHIP_FMT_NONE ? b->geo.page_format : o.output_pixel_format;
  if (of == UPHIP_FMT_Y400A) of = UPHIP_FMT_GRAY8;
  if (of == UPHIP_FMT_MONOBLACK) of = UPHIP_FMT_MONOWHITE;
  b->out_fmt = of;
  // layout defaults (sheet_stages.c:232-279) on the processing size
  const int32_t W = b->W, H = b->H;
  b->points.assign(o.points, o.points + o.point_count);
  int32_t mmw = o.mask_detection_parameters.maximum_width;
  int32_t mmh = o.mask_detection_parameters.maximum_height;
  if (o.layout == UPHIP_LAYOUT_SINGLE) {
    if (b->points.empty()) b->points.push_back(UphipPoint{W / 2, H / 2});
    if (mmw == -1) mmw = W;
    if (mmh == -1) mmh = H;
    b->outside.push_back(Rect{0, 0, W - 1, H - 1});
  } else if (o.layout == UPHIP_LAYOUT_DOUBLE) {
    if (b->points.empty()) {
      b->points.push_back(UphipPoint{W / 4, H / 2});
      b->points.push_back(UphipPoint{W - W / 4, H / 2});
    }
    if (mmw == -1) mmw = W / 2;
    if (mmh == -1) mmh = H;
    b->outside.push_back(Rect{0, 0, W / 2, H - 1});
    b->outside.push_back(Rect{W / 2, 0, W - 1, H - 1});
  }
  if (mmw == -1) mmw = W;
  if (mmh == -1) mmh = H;
  if (b->points.size() > UPHIP_MAX_PAGES)
    return fail("batch: at most %d mask points are supported (got %zu)", UPHIP_MAX_PAGES,
                b->points.size());
  b->mask_params = o.mask_detection_parameters;
  b->mask_params.maximum_width = mmw;
  b->mask_params.maximum_height = mmh;
  b->black_params = o.blackfilter_parameters;
  if (b->black_params.exclusions_count == 0 && o.layout != UPHIP_LAYOUT_NONE) {
    UphipBlackfilterParameters& bp = b->black_params;
    if (o.layout == UPHIP_LAYOUT_SINGLE) {
      bp.exclusions[bp.exclusions_count++] = from_rect(rect_from_size(W / 4, H / 4, W / 2, H / 2));
    } else {
      const int32_t fw = W / 4, fh = H / 2;
      bp.exclusions[bp.exclusions_count++] = from_rect(rect_from_size(W / 8, H / 4, fw, fh));
      bp.exclusions[bp.exclusions_count++] =
          from_rect(rect_from_size(W / 8 + W / 2, H / 4, fw, fh));
    }
  }
  return true;
}

static bool allocate(UphipBatch* b) {
  const int cap = b->cap;
  const UphipOptions& o = b->o;
  b->in_pitch = round_pitch(row_bytes(b->geo.page_width, b->geo.page_format));
  b->in_page_stride = b->in_pitch * b->geo.page_height;
  b->inputs = dalloc<uint8_t>(b, (size_t)b->in_page_stride * cap * b->n_in);
  const int bpp = b->work_fmt == F_GRAY8 ? 1 : 3;
  b->pitch = round_pitch((int64_t)b->max_w * bpp);
  b->plane_stride = b->pitch * b->max_h;
  b->planes[0] = dalloc<uint8_t>(b, (size_t)b->plane_stride * cap);
  b->planes[1] = dalloc<uint8_t>(b, (size_t)b->plane_stride * cap);
  if (b->out_fmt != b->work_fmt) {
    b->out_pitch = round_pitch(row_bytes(b->out_w, b->out_fmt));
    b->out_stride = b->out_pitch * b->out_h;
    b->out = dalloc<uint8_t>(b, (size_t)b->out_stride * cap);
    if (b->out) UPH_HIP(hipMemset(b->out, 0, (size_t)b->out_stride * cap));
  }
  if (o.pre_rotate != 0) {
    const int64_t rp = round_pitch(row_bytes(b->rp_w, b->geo.page_format));
    b->rot_page = dalloc<uint8_t>(b, (size_t)rp * b->rp_h * cap);
  }
  b->ctl = dalloc<SheetCtl>(b, cap);
  b->sticky = dalloc<int32_t>(b, 1);
  if (!b->inputs || !b->planes[0] || !b->planes[1] || !b->ctl || !b->sticky) return false;
  if (!UPH_HIP(hipMemset(b->sticky, 0, sizeof(int32_t)))) return false;
  // filter geometry + scratch (one region per sheet, reused stage after stage)
  const int32_t W = b->W, H = b->H;
  size_t need = 0;
  std::vector<BlackBar> bars(2 * (size_t)(W + H) + 16);
  if (!(o.disable & UPHIP_NO_BLACKFILTER)) {
    if (b->work_fmt == F_GRAY8 && o.abs_black_threshold == 255)
      return fail("batch: abs_black_threshold 255 makes the reference flood fill recurse forever");
    if (!black_geometry(W, H, b->black_params, o.abs_black_threshold, &b->bgeo, bars.data(),
                        (int)bars.size()))
      return fail("batch: invalid blackfilter parameters");
    need = std::max(need, black_scratch_bytes(b->bgeo));
    if (b->bgeo.nbars) {
      b->dbars = dalloc<BlackBar>(b, b->bgeo.nbars);
      UPH_HIP(hipMemcpy(b->dbars, bars.data(), sizeof(BlackBar) * b->bgeo.nbars,
                        hipMemcpyHostToDevice));
    }
    std::vector<AxisArgs> hv((size_t)cap, AxisArgs{b->bgeo.hregion, 0, 1});
    b->black_h = dalloc<AxisArgs>(b, cap);
    UPH_HIP(hipMemcpy(b->black_h, hv.data(), sizeof(AxisArgs) * cap, hipMemcpyHostToDevice));
    hv.assign((size_t)cap, AxisArgs{b->bgeo.vregion, 0, 1});
    b->black_v = dalloc<AxisArgs>(b, cap);
    UPH_HIP(hipMemcpy(b->black_v, hv.data(), sizeof(AxisArgs) * cap, hipMemcpyHostToDevice));
  }
  if (!(o.disable & UPHIP_NO_NOISEFILTER)) {
    noise_geometry(W, H, o.noisefilter_intensity, o.abs_white_threshold, &b->ngeo);
    need = std::max(need, noise_scratch_bytes(b->ngeo));
    if (b->work_fmt == F_GRAY8) {
      b->nbits_stride = ((int64_t)noise_bit_words(W) * H + 63) & ~(int64_t)63;
      b->nbits = dalloc<uint32_t>(b, (size_t)b->nbits_stride * cap);
      if (!b->nbits) return false;
    }
  }
  if (!(o.disable & UPHIP_NO_BLURFILTER)) {
    if (!blur_geometry(W, H, o.blurfilter_parameters, o.abs_white_threshold, &b->blgeo))
      return fail("batch: invalid blurfilter parameters");
    need = std::max(need, blur_scratch_bytes(b->blgeo));
    // the bit-plane stays exact only while every clear makes a pixel > white
    if (b->work_fmt == F_GRAY8 && o.abs_white_threshold < 255 && b->blgeo.nrect > 0 &&
        b->blgeo.sw >= 32) {
      b->nbits_stride = ((int64_t)noise_bit_words(W) * H + 63) & ~(int64_t)63;
      b->bbits = dalloc<uint32_t>(b, (size_t)b->nbits_stride * cap);
      if (!b->bbits) return false;
    }
  }
  if (!(o.disable & UPHIP_NO_GRAYFILTER)) {
    if (!gray_geometry(W, H, o.grayfilter_parameters, o.abs_black_threshold, &b->ggeo))
      return fail("batch: invalid grayfilter parameters");
    need = std::max(need, gray_scratch_bytes(b->ggeo));
  }
  need = (need + 255) & ~(size_t)255;
  b->scr_stride = (int64_t)need;
  if (need) {
    b->scr = dalloc<uint8_t>(b, need * cap);
    if (!b->scr) return false;
  }
  // detection buffers
  const int np = (int)b->points.size();
  const int nout = (int)b->outside.size();
  b->sums_stride = (int64_t)imax(b->max_w, b->max_h) * 2 * imax(np, nout) + 64;
  b->sums = dalloc<uint32_t>(b, (size_t)b->sums_stride * cap);
  b->edge_res = dalloc<int32_t>(b, (size_t)cap * imax(np, 1) * 4);
  b->border_res = dalloc<int32_t>(b, (size_t)cap * imax(nout, 1) * 4);
  b->move_args = dalloc<MoveArgs>(b, (size_t)cap * UPHIP_MAX_PAGES);
  b->border_need = dalloc<int32_t>(b, cap);
  b->border_mask_args = dalloc<MaskArgs>(b, cap);
  b->rot_args = dalloc<RotateArgs>(b, (size_t)cap * UPHIP_MAX_PAGES);
  b->rot_indep = dalloc<int32_t>(b, cap);
  b->rot_dep = dalloc<int32_t>(b, cap);
  b->pick_mask = dalloc<Rect>(b, cap);
  b->pick_active = dalloc<int32_t>(b, cap);
  // rotation tables
  if (!(o.disable & UPHIP_NO_DESKEW)) {
    if (rotation_angles(o.deskew_parameters, &b->table) < 0)
      return fail("batch: too many deskew angles");
    const int na = b->table.nangles;
    for (int i = 0; i < na; i++) b->max_angle = fmaxf(b->max_angle, fabsf(b->table.angle[i]));
    b->dtable = dalloc<RotTable>(b, 1);
    UPH_HIP(hipMemcpy(b->dtable, &b->table, sizeof(RotTable), hipMemcpyHostToDevice));
    int nedges = 0;
    int kinds[4];
    const UphipEdges& E = o.deskew_parameters.scan_edges;
    const bool on[4] = {E.left, E.top, E.right, E.bottom};
    for (int k = 0; k < 4; k++)
      if (on[k]) kinds[nedges++] = k;
    // exact combination table for <= 2 edges (host libm, like deskew.c)
    size_t ncombo = nedges == 2 ? (size_t)na * na : (size_t)na;
    std::vector<RotCombo> combo(ncombo);
    for (size_t key = 0; key < ncombo; key++) {
      float rot[2];
      int idx[2] = {(int)(nedges == 2 ? key / na : key), (int)(key % na)};
      for (int e = 0; e < nedges && e < 2; e++) {
        const float v = b->table.angle[idx[e]];
        rot[e] = (kinds[e] == 1 || kinds[e] == 3) ? -v : v;
      }
      RotCombo c;
      c.result = combine_edge_rotations(rot, nedges > 2 ? 2 : nedges,
                                        o.deskew_parameters.deskewScanDeviationRad);
      c.sinv = sinf(-c.result);
      c.cosv = cosf(-c.result);
      combo[key] = c;
    }
    b->dcombo = dalloc<RotCombo>(b, ncombo);
    UPH_HIP(hipMemcpy(b->dcombo, combo.data(), sizeof(RotCombo) * ncombo, hipMemcpyHostToDevice));
    if (nedges > 2) {
      const uint32_t* t = glibc_pow2_table(&b->npow2);
      if (!t) return fail("batch: this libm's powf(x, 2) is not reproducible on the device");
      b->dpow2 = dalloc<uint32_t>(b, imax(b->npow2, 1));
      UPH_HIP(hipMemcpy(b->dpow2, t, sizeof(uint32_t) * b->npow2, hipMemcpyHostToDevice));
    }
    b->peaks = dalloc<int32_t>(b, (size_t)cap * UPHIP_MAX_PAGES * 4 * (na > 0 ? na : 1));
    int ms = o.deskew_parameters.deskewScanSize;
    if (ms == -1 || ms > 10000) ms = 10000;
    b->max_scan = imin(ms, imax(W, H));
    b->rot_lines = (int32_t*)dalloc<uint8_t>(b, rotation_lines_bytes(cap, nedges, na, b->max_scan));
    if (!b->rot_lines) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------
// Stage helpers
// ---------------------------------------------------------------------------
static void fill_uniform(UphipBatch* b, const Planes& P, int which, Rect clipped, UphipPixel c,
                         int count) {
  if (clipped.x1 < clipped.x0 || clipped.y1 < clipped.y0) return;
  FillArgs fa{clipped, {c.r, c.g, c.b}, 1};
  FillArgs* d = replicate(b, fa);
  launch_fill_thr(PlaneRef{P, b->ctl, which}, d, count, clipped.y1 - clipped.y0 + 1,
                  b->o.abs_black_threshold, b->st);
}

static void masks_uniform(UphipBatch* b, const Planes& P, const Rect* m, int n, UphipPixel c,
                          int count) {
  if (n <= 0) return;
  MaskArgs ma;
  memset(&ma, 0, sizeof(ma));
  ma.n = n;
  ma.color[0] = c.r;
  ma.color[1] = c.g;
  ma.color[2] = c.b;
  for (int i = 0; i < n; i++) ma.m[i] = m[i];
  MaskArgs* d = replicate(b, ma);
  launch_apply_masks_thr(cur_ref(P, b->ctl), d, count, b->o.abs_black_threshold, b->st);
}

static void wipes_uniform(UphipBatch* b, const Planes& P, const UphipWipes& w, int count) {
  // apply_wipes_cpu (masks.c:333-345): as-given rectangles, set_pixel clips
  for (size_t i = 0; i < w.count && i < UPHIP_MAX_MASKS; i++) {
    const Rect r = to_rect(w.areas[i]);
    if (r.x0 > r.x1 || r.y0 > r.y1) continue;
    fill_uniform(b, P, 0, clip(r, P.W, P.H), b->o.mask_color, count);
  }
}

static void border_uniform(UphipBatch* b, const Planes& P, const UphipBorder& br, int count) {
  if (br.left == 0 && br.top == 0 && br.right == 0 && br.bottom == 0) return;
  const Rect m{br.left, br.top, P.W - br.right - 1, P.H - br.bottom - 1};
  masks_uniform(b, P, &m, 1, b->o.mask_color, count);
}

// stretch_and_replace / resize_and_replace on every sheet (blit.c:231-282)
static void stretch_all(UphipBatch* b, int32_t& w, int32_t& h, int32_t nw, int32_t nh,
                        int count) {
  if (compare_sizes_h(w, h, nw, nh) == 0) return;
  const Planes S = planes_of(b, w, h), D = planes_of(b, nw, nh);
  launch_stretch_thr(cur_ref(S, b->ctl), other_ref(D, b->ctl), b->o.interpolate_type,
                     b->o.abs_black_threshold, count, b->st);
  flip_all(b, count);
  w = nw;
  h = nh;
}

static void resize_all(UphipBatch* b, int32_t& w, int32_t& h, int32_t pw, int32_t ph,
                       int count) {
  if (compare_sizes_h(w, h, pw, ph) == 0) return;
  const float hr = (float)pw / (float)w, vr = (float)ph / (float)h;
  int32_t sw, sh;
  if (hr < vr) {
    sw = pw;
    sh = (int32_t)(h * hr);
  } else if (vr < hr) {
    sw = (int32_t)(w * vr);
    sh = ph;
  } else {
    sw = pw;
    sh = ph;
  }
  stretch_all(b, w, h, sw, sh, count);
  if (pw == sw && ph == sh) return;
  // resized = bg-filled (pw x ph); center_image(stretched, resized, origin, size)
  const Planes D = planes_of(b, pw, ph);
  fill_uniform(b, D, 1, Rect{0, 0, pw - 1, ph - 1}, b->o.sheet_background, count);
  int32_t sox = 0, soy = 0, tox = 0, toy = 0, ssw = w, ssh = h;
  if (ssw <= pw) tox += (pw - ssw) / 2;
  else {
    sox += (ssw - pw) / 2;
    ssw = pw;
  }
  if (ssh <= ph) toy += (ph - ssh) / 2;
  else {
    soy += (ssh - ph) / 2;
    ssh = ph;
  }
  CopyArgs ca{clip(rect_from_size(sox, soy, ssw, ssh), w, h), tox, toy, 1};
  CopyArgs* d = replicate(b, ca);
  launch_copy_thr(cur_ref(planes_of(b, w, h), b->ctl), other_ref(D, b->ctl), d, count, ssh,
                  b->o.abs_black_threshold, b->st);
  flip_all(b, count);
  w = pw;
  h = ph;
}

// The first mask scan (sheet_stages.c:393-399) runs on the image the
// grayfilter leaves; with one point, a horizontal-only scan over every row
// and a gray plane, its column sums come out of the grayfilter's cell pass
// (plus its wipes' changes) instead of a pass of their own.
// One point, a horizontal-only scan over every row, a gray plane: the scan's
// sums are plain column sums of the whole image.
static bool mask_scan_all_rows(const UphipBatch* b) {
  const UphipMaskDetectionParameters& p = b->mask_params;
  if (b->points.size() != 1 || !p.scan_direction.horizontal || p.scan_direction.vertical) return false;
  if (b->work_fmt != F_GRAY8) return false;
  const int32_t depth = p.scan_depth.horizontal == -1 ? b->H : p.scan_depth.horizontal;
  const int32_t c0 = b->points[0].y - depth / 2, c1 = c0 + depth - 1;
  return c0 <= 0 && c1 >= b->H - 1;
}
static bool mask_sums_from_gray(const UphipBatch* b) {
  const UphipOptions& o = b->o;
  if (o.disable & (UPHIP_NO_DESKEW | UPHIP_NO_MASK_SCAN | UPHIP_NO_GRAYFILTER)) return false;
  return mask_scan_all_rows(b);
}
// The second mask scan (sheet_stages.c:415-421) runs on the deskewed image:
// its column sums are the rotate kernel's output sums for the rotated sheets
// and, for the others (unchanged since), the first scan's, still in b->sums.
static bool mask_sums_from_rotate(const UphipBatch* b) {
  const UphipOptions& o = b->o;
  if (o.disable & (UPHIP_NO_DESKEW | UPHIP_NO_MASK_SCAN | UPHIP_NO_MASK_CENTER)) return false;
  return mask_scan_all_rows(b);
}

// detect_masks on every sheet -> ctl.masks / ctl.mask_count (masks.c:54-209).
// sums_ready: point 0's horizontal column sums are already in b->sums
// (mask_sums_from_gray).
static void detect_masks_all(UphipBatch* b, int assign, int count, bool sums_ready = false) {
  const UphipMaskDetectionParameters& p = b->mask_params;
  if (!p.scan_direction.horizontal && !p.scan_direction.vertical) return;
  const int np = (int)b->points.size();
  const int32_t W = b->W, H = b->H;
  const Planes P = planes_of(b, W, H);
  if (!sums_ready)
    UPH_HIP(hipMemsetAsync(b->sums, 0, sizeof(uint32_t) * b->sums_stride * count, b->st));
  std::vector<EdgeArgs> ea((size_t)np * 4);
  for (int i = 0; i < np; i++) {
    const UphipPoint o = b->points[i];
    for (int k = 0; k < 4; k++) ea[i * 4 + k].active = 0;
    if (p.scan_direction.horizontal) {
      const int32_t depth = p.scan_depth.horizontal == -1 ? H : p.scan_depth.horizontal;
      const int32_t c0 = o.y - depth / 2, c1 = c0 + depth - 1;
      const Rect reg = clip(Rect{0, c0, W - 1, c1}, W, H);
      const int32_t off = (2 * i) * imax(W, H);
      if (reg.y1 >= reg.y0 && !(sums_ready && i == 0)) {
        AxisArgs* aa = replicate(b, AxisArgs{reg, 0, 1});
        launch_axis_reduce(cur_ref(P, b->ctl), aa, 0, M_GRAY_SUM, W, H, b->sums + off,
                           b->sums_stride, count, b->st);
      }
      for (int k = 0; k < 2; k++) {
        EdgeArgs& e = ea[i * 4 + k];
        e = EdgeArgs{1, off, W, H, c0, c1, o.x - p.scan_size.width / 2,
                     (k == 0 ? -1 : 1) * p.scan_step.horizontal, p.scan_size.width,
                     p.scan_threshold.horizontal};
      }
    }
    if (p.scan_direction.vertical) {
      const int32_t depth = p.scan_depth.vertical == -1 ? W : p.scan_depth.vertical;
      const int32_t c0 = o.x - depth / 2, c1 = c0 + depth - 1;
      const Rect reg = clip(Rect{c0, 0, c1, H - 1}, W, H);
      const int32_t off = (2 * i + 1) * imax(W, H);
      if (reg.x1 >= reg.x0) {
        AxisArgs* aa = replicate(b, AxisArgs{reg, 0, 1});
        launch_axis_reduce(cur_ref(P, b->ctl), aa, 1, M_GRAY_SUM, W, H, b->sums + off,
                           b->sums_stride, count, b->st);
      }
      for (int k = 2; k < 4; k++) {
        EdgeArgs& e = ea[i * 4 + k];
        e = EdgeArgs{1, off, H, W, c0, c1, o.y - p.scan_size.height / 2,
                     (k == 2 ? -1 : 1) * p.scan_step.vertical, p.scan_size.height,
                     p.scan_threshold.vertical};
      }
    }
  }
  // replicate the 4*np jobs for every sheet
  std::vector<EdgeArgs> all((size_t)b->cap * np * 4);
  for (int s = 0; s < b->cap; s++)
    for (int j = 0; j < np * 4; j++) all[(size_t)s * np * 4 + j] = ea[j];
  EdgeArgs* de = (EdgeArgs*)upload_cached(b, all.data(), sizeof(EdgeArgs) * all.size());
  launch_edge_scan(de, np * 4, b->sums, b->sums_stride, b->edge_res, count, b->st, imax(W, H));
  MaskAssembleArgs ma{p, W, H, np, assign};
  hipLaunchKernelGGL(k_mask_assemble, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl,
                     b->edge_res, ma, count);
}

// The border scan's row sums can come out of the last mask-centering move
// (k_move_rect_g16 counts the dark pixels of every row it writes): one
// outside rectangle, a vertical scan only, a gray plane, and nothing between
// the centering and the border scan that writes the sheet (sheet_stages.c:
// 425-473: explicit wipes, the middle wipe, the explicit border).
static bool border_rows_from_center(const UphipBatch* b) {
  const UphipOptions& o = b->o;
  const uint32_t dis = o.disable;
  const UphipBorderScanParameters& p = o.border_scan_parameters;
  if ((dis & UPHIP_NO_MASK_CENTER) || b->points.empty()) return false;
  if ((dis & UPHIP_NO_BORDER_SCAN) || b->outside.size() != 1) return false;
  if (p.scan_direction.horizontal || !p.scan_direction.vertical) return false;
  if (b->work_fmt != F_GRAY8) return false;
  if (b->outside[0].x0 > b->outside[0].x1) return false;
  if (!(dis & UPHIP_NO_WIPE)) {
    if (o.wipes.count > 0) return false;
    if (o.layout == UPHIP_LAYOUT_DOUBLE && (o.middle_wipe[0] > 0 || o.middle_wipe[1] > 0)) return false;
  }
  if (!(dis & UPHIP_NO_BORDER) &&
      (o.border.left || o.border.top || o.border.right || o.border.bottom))
    return false;
  return true;
}

// The centring move, the border scan and the masked align move chained
// (launch_move_chain): the centring only counts (a dry pass, C is never
// written) and the align move gathers straight from the uncentred plane.
// Needs border_rows_from_center, one page (one centring move), the align move
// on, and 32-bit plane offsets.
#ifndef UPH_CHAIN_MOVES
#define UPH_CHAIN_MOVES 1  // 0: the two moves as separate passes (A/B builds)
#endif
static bool chain_center_align(const UphipBatch* b) {
  if (!UPH_CHAIN_MOVES || !border_rows_from_center(b) || b->points.size() != 1) return false;
  if (b->o.disable & UPHIP_NO_BORDER_ALIGN) return false;
  return b->pitch * (int64_t)b->H < (1ll << 31) && UPHIP_MAX_PAGES >= 2;
}

// The chained border scan first counts only the rows within
// kBorderEdgeRows of the top and bottom (the scan from each edge stops at the
// first dark band, normally within the margin); sheets whose scan reaches
// the middle rows get them counted and are scanned again.
constexpr int32_t kBorderEdgeRows = 320;  // a multiple of the move's block rows
static bool border_edge_rows_only(const UphipBatch* b) { return b->H > 2 * kBorderEdgeRows + 64; }
// The centring move's counting pass (border_rows_from_center): C's dark
// pixels per row over outside rect 0's columns into border_all's row sums.
static MoveExtra center_count_args(const UphipBatch* b) {
  const Rect oc = clip(b->outside[0], b->W, b->H);
  MoveExtra x{};
  x.rows = b->sums + imax(b->W, b->H);  // border_all's vertical offset, outside rect 0
  x.rows_stride = b->sums_stride;
  x.rx0 = oc.x0;
  x.rx1 = oc.x1;
  x.thr = b->o.abs_black_threshold;
  return x;
}

// rows_ready: the vertical scan's row sums are already in b->sums
// (border_rows_from_center).  center: the chained centring move's arguments
// (chain_center_align), whose plane was never written.
static void border_all(UphipBatch* b, int count, bool rows_ready,
                       const MoveArgs* center = nullptr) {
  const UphipBorderScanParameters& p = b->o.border_scan_parameters;
  const int nout = (int)b->outside.size();
  const int32_t W = b->W, H = b->H;
  const Planes P = planes_of(b, W, H);
  if (!rows_ready)
    UPH_HIP(hipMemsetAsync(b->sums, 0, sizeof(uint32_t) * b->sums_stride * count, b->st));
  std::vector<BorderEdgeArgs> ea((size_t)nout * 4);
  memset(ea.data(), 0, sizeof(BorderEdgeArgs) * ea.size());
  for (int i = 0; i < nout; i++) {
    const Rect o = b->outside[i];
    const int32_t mw = iabs(o.x0 - o.x1) + 1, mh = iabs(o.y0 - o.y1) + 1;
    if (p.scan_direction.horizontal) {
      const int32_t off = (2 * i) * imax(W, H);
      AxisArgs a{clip(Rect{0, o.y0, W - 1, o.y1}, W, H), b->o.abs_black_threshold,
                 o.y0 <= o.y1 ? 1 : 0};
      if (a.active && a.region.y1 >= a.region.y0)
        launch_axis_reduce(cur_ref(P, b->ctl), replicate(b, a), 0, M_DARK_COUNT, W, H,
                           b->sums + off, b->sums_stride, count, b->st);
      const int32_t sz = p.scan_size.width, stp = p.scan_step.horizontal;
      ea[i * 4 + 0] = BorderEdgeArgs{1, off, W, o.x0, o.x0 + sz, stp, mw, p.scan_threshold.horizontal};
      ea[i * 4 + 1] = BorderEdgeArgs{1, off, W, o.x1 - sz, o.x1, -stp, mw, p.scan_threshold.horizontal};
    }
    if (p.scan_direction.vertical) {
      const int32_t off = (2 * i + 1) * imax(W, H);
      AxisArgs a{clip(Rect{o.x0, 0, o.x1, H - 1}, W, H), b->o.abs_black_threshold,
                 o.x0 <= o.x1 ? 1 : 0};
      if (a.active && a.region.x1 >= a.region.x0 && !rows_ready)
        launch_axis_reduce(cur_ref(P, b->ctl), replicate(b, a), 1, M_DARK_COUNT, W, H,
                           b->sums + off, b->sums_stride, count, b->st);
      const int32_t sz = p.scan_size.height, stp = p.scan_step.vertical;
      ea[i * 4 + 2] = BorderEdgeArgs{1, off, H, o.y0, o.y0 + sz, stp, mh, p.scan_threshold.vertical};
      ea[i * 4 + 3] = BorderEdgeArgs{1, off, H, o.y1 - sz, o.y1, -stp, mh, p.scan_threshold.vertical};
    }
  }
  std::vector<BorderEdgeArgs> all((size_t)b->cap * nout * 4);
  for (int s = 0; s < b->cap; s++)
    for (int j = 0; j < nout * 4; j++) all[(size_t)s * nout * 4 + j] = ea[j];
  BorderEdgeArgs* de =
      (BorderEdgeArgs*)upload_cached(b, all.data(), sizeof(BorderEdgeArgs) * all.size());
  UPH_HIP(hipMemsetAsync(b->border_res, 0, sizeof(int32_t) * count * nout * 4, b->st));
  if (center && border_edge_rows_only(b)) {
    // rows [kBorderEdgeRows, H - kBorderEdgeRows) not counted yet: scan, count
    // them for the sheets that reach them, scan those again
    UPH_HIP(hipMemsetAsync(b->border_need, 0, sizeof(int32_t) * count, b->st));
    launch_border_scan(de, nout * 4, b->sums, b->sums_stride, b->border_res, count, b->st,
                       imax(W, H), kBorderEdgeRows, H - kBorderEdgeRows, b->border_need);
    MoveExtra x = center_count_args(b);
    x.dry = true;
    x.ya0 = kBorderEdgeRows;
    x.ya1 = H - kBorderEdgeRows;
    x.only = b->border_need;
    launch_move_rect_fused(cur_ref(P, b->ctl), other_ref(P, b->ctl), center, x, count, b->st);
    launch_border_scan(de, nout * 4, b->sums, b->sums_stride, b->border_res, count, b->st,
                       imax(W, H), 0, 0, nullptr, b->border_need);
  } else {
    launch_border_scan(de, nout * 4, b->sums, b->sums_stride, b->border_res, count, b->st,
                       imax(W, H));
  }
  BorderAssembleArgs ba;
  memset(&ba, 0, sizeof(ba));
  ba.W = W;
  ba.H = H;
  ba.nout = nout;
  ba.cap = b->cap;
  for (int i = 0; i < nout; i++) ba.outside[i] = b->outside[i];
  ba.horizontal = p.scan_direction.horizontal;
  ba.vertical = p.scan_direction.vertical;
  ba.align = !(b->o.disable & UPHIP_NO_BORDER_ALIGN);
  ba.ap = b->o.mask_alignment_parameters;
  ba.mask_color[0] = b->o.mask_color.r;
  ba.mask_color[1] = b->o.mask_color.g;
  ba.mask_color[2] = b->o.mask_color.b;
  ba.bg[0] = b->o.sheet_background.r;
  ba.bg[1] = b->o.sheet_background.g;
  ba.bg[2] = b->o.sheet_background.b;
  hipLaunchKernelGGL(k_border_assemble, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl,
                     b->border_res, ba, b->border_mask_args, b->move_args, count);
  // apply_masks then align_mask (sheet_stages.c:478-488): with one outside
  // rectangle on a gray plane, one pass -- the move writes the mask colour
  // outside the border mask (and masks in place where the move is the
  // identity)
  const bool align = !(b->o.disable & UPHIP_NO_BORDER_ALIGN);
  const bool fold = align && nout == 1 && P.fmt == F_GRAY8;
  if (center) {
    // every sheet's output written to the other plane: flip them all
    launch_move_chain(cur_ref(P, b->ctl), other_ref(P, b->ctl), center, b->border_mask_args,
                      b->move_args, count, b->st);
    flip_all(b, count);
    return;
  }
  if (!fold)
    launch_apply_masks_thr(cur_ref(P, b->ctl), b->border_mask_args, count,
                           b->o.abs_black_threshold, b->st);
  for (int i = 0; i < nout && align; i++) {
    MoveArgs* mv = b->move_args + (int64_t)i * b->cap;
    if (fold) {
      MoveExtra x{};
      x.masks = b->border_mask_args;
      launch_move_rect_fused(cur_ref(P, b->ctl), other_ref(P, b->ctl), mv, x, count, b->st);
    } else {
      launch_move_rect(cur_ref(P, b->ctl), other_ref(P, b->ctl), mv, count, b->st);
    }
    launch_flip_if_active(b->ctl, &mv->active, sizeof(MoveArgs), count, b->st);
  }
}

// ---------------------------------------------------------------------------
// run
// ---------------------------------------------------------------------------
// The decode may also produce the noisefilter's dark bit-plane and the
// blackfilter's v-stripe row sums (k_decode_gray) when a GRAY8 page becomes
// the sheet unchanged and nothing writes the sheet between the decode and
// the filters (sheet_stages.c:187-325: pre-mirror, -shift, -masks,
// -stretch/size, -wipes, -border all off).
static bool decode_fused(const UphipBatch* b, const uint8_t* src, int64_t spitch,
                         int64_t sstride) {
  const UphipOptions& o = b->o;
  const uint32_t dis = o.disable;
  if (b->work_fmt != F_GRAY8 || b->geo.page_format != F_GRAY8 || b->n_in != 1) return false;
  if (b->rp_w != b->sheet_w || b->rp_h != b->sheet_h || o.pre_rotate != 0) return false;
  if (b->sheet_w != b->W || b->sheet_h != b->H) return false;  // stretch / page size
  // 16-byte vector loads at src + s*sstride + y*spitch (a row's last vector
  // may read up to 15 bytes past the row within its pitch)
  if (((uintptr_t)src & 15) || (spitch & 15) || (sstride & 15)) return false;
  if (o.pre_mirror.horizontal || o.pre_mirror.vertical) return false;
  if (o.pre_shift.horizontal != 0 || o.pre_shift.vertical != 0 || o.pre_mask_count > 0) return false;
  if (!(dis & UPHIP_NO_WIPE) && o.pre_wipes.count > 0) return false;
  if (!(dis & UPHIP_NO_BORDER) &&
      (o.pre_border.left || o.pre_border.top || o.pre_border.right || o.pre_border.bottom))
    return false;
  return true;
}

static bool run_batch(UphipBatch* b, int count, const uint8_t* src, int64_t spitch,
                      int64_t sstride) {
  const UphipOptions& o = b->o;
  const uint32_t dis = o.disable;
  if (b->timing) b->runs.emplace_back();
  b->cache_pos = 0;
  mark(b, "start");
  const UphipPoint p0 = b->points.size() > 0 ? b->points[0] : UphipPoint{0, 0};
  const UphipPoint p1 = b->points.size() > 1 ? b->points[1] : UphipPoint{0, 0};
  hipLaunchKernelGGL(k_ctl_init, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl, count,
                     (int32_t)b->points.size(), p0, p1);
  // ---- decode: pages -> working sheet (sheet_stages.c:44-185) ----------
  const int n = b->n_in;
  int32_t w = b->sheet_w, h = b->sheet_h;
  Planes S0 = planes_of(b, w, h);
  const bool covered = n == 1 && b->rp_w == w && b->rp_h == h;
  const bool fused = decode_fused(b, src, spitch, sstride);
  // what the fused decode hands on
  const bool black_on = !(dis & UPHIP_NO_BLACKFILTER) && b->bgeo.nbars > 0;
  const bool vsum_ready = fused && black_on && b->bgeo.vregion.x1 >= b->bgeo.vregion.x0;
#ifndef UPH_NO_DECODE_RM
  const bool rm_ready = fused && black_on;  // the blackfilter's match plane from the decode
#else
  const bool rm_ready = false;
#endif
  uint32_t* bits_ready = fused && !(dis & UPHIP_NO_NOISEFILTER) ? b->nbits : nullptr;
  // the blurfilter's plane: made by the decode, kept by the black/noise clears
#ifndef UPH_NO_BLUR_BITS
  uint32_t* bb_ready = fused && !(dis & UPHIP_NO_BLURFILTER) ? b->bbits : nullptr;
#else  // tuning A/B: the blur counts read the plane
  uint32_t* bb_ready = nullptr;
#endif
  if (fused) {
    launch_decode_gray(src, spitch, sstride, cur_ref(S0, b->ctl), o.abs_white_threshold, bits_ready,
                       b->nbits_stride, vsum_ready ? (uint32_t*)b->scr + b->bgeo.W : nullptr,
                       b->scr_stride / 4, b->bgeo.vregion.x0, b->bgeo.vregion.x1, count, b->st,
                       bb_ready, rm_ready ? black_rm_plane(b->bgeo, b->scr) : nullptr,
                       b->scr_stride / 4, b->bgeo.mask_max);
  }
  if (!covered) fill_uniform(b, S0, 0, Rect{0, 0, w - 1, h - 1}, o.sheet_background, count);
  for (int j = 0; j < n && !fused; j++) {
    Planes pg;
    pg.base[0] = pg.base[1] = const_cast<uint8_t*>(src) + j * sstride;
    pg.pitch = spitch;
    pg.stride = sstride * n;
    pg.W = b->geo.page_width;
    pg.H = b->geo.page_height;
    pg.fmt = b->geo.page_format;
    pg.count = count;
    if (o.pre_rotate != 0) {
      Planes rp;
      rp.base[0] = rp.base[1] = b->rot_page;
      rp.pitch = round_pitch(row_bytes(b->rp_w, pg.fmt));
      rp.stride = rp.pitch * b->rp_h;
      rp.W = b->rp_w;
      rp.H = b->rp_h;
      rp.fmt = pg.fmt;
      rp.count = count;
      launch_rotate90_thr(fixed_ref(pg, 0), fixed_ref(rp, 0), o.pre_rotate / 90,
                          o.abs_black_threshold, count, b->st);
      pg = rp;
    }
    // center_image(page, sheet, (w*j/n, 0), (w/n, h))  (blit.c:175-202)
    int32_t tox = w * j / n, toy = 0, tw = w / n, th = h;
    int32_t sox = 0, soy = 0, ssw = pg.W, ssh = pg.H;
    if ((ssw < tw || ssh < th) && covered == false) {
      // target rectangle already holds the background (whole-sheet fill)
    }
    if (ssw <= tw) tox += (tw - ssw) / 2;
    else {
      sox += (ssw - tw) / 2;
      ssw = tw;
    }
    if (ssh <= th) toy += (th - ssh) / 2;
    else {
      soy += (ssh - th) / 2;
      ssh = th;
    }
    CopyArgs ca{clip(rect_from_size(sox, soy, ssw, ssh), pg.W, pg.H), tox, toy, 1};
    launch_copy_thr(fixed_ref(pg, 0), cur_ref(S0, b->ctl), replicate(b, ca), count, ssh,
                    o.abs_black_threshold, b->st);
  }
  mark(b, "decode");
  // ---- pre (sheet_stages.c:187-325) -----------------------------------
  if (o.pre_mirror.horizontal || o.pre_mirror.vertical) {
    const Planes P = planes_of(b, w, h);
    launch_mirror_oop(cur_ref(P, b->ctl), other_ref(P, b->ctl), o.pre_mirror.horizontal,
                      o.pre_mirror.vertical, o.abs_black_threshold, count, b->st);
    flip_all(b, count);
  }
  if (o.pre_shift.horizontal != 0 || o.pre_shift.vertical != 0) {
    const Planes P = planes_of(b, w, h);
    const uint8_t bg[3] = {o.sheet_background.r, o.sheet_background.g, o.sheet_background.b};
    launch_shift(cur_ref(P, b->ctl), other_ref(P, b->ctl), o.pre_shift.horizontal,
                 o.pre_shift.vertical, bg, o.abs_black_threshold, count, b->st);
    flip_all(b, count);
  }
  if (o.pre_mask_count > 0) {
    std::vector<Rect> pm(o.pre_mask_count);
    for (size_t i = 0; i < o.pre_mask_count; i++) pm[i] = to_rect(o.pre_masks[i]);
    masks_uniform(b, planes_of(b, w, h), pm.data(), (int)pm.size(), o.mask_color, count);
  }
  {
    int32_t sw = o.stretch_size.width == -1 ? w : o.stretch_size.width;
    int32_t sh = o.stretch_size.height == -1 ? h : o.stretch_size.height;
    sw *= o.pre_zoom_factor;
    sh *= o.pre_zoom_factor;
    stretch_all(b, w, h, sw, sh, count);
    if (o.page_size.width != -1 || o.page_size.height != -1)
      resize_all(b, w, h, o.page_size.width == -1 ? w : o.page_size.width,
                 o.page_size.height == -1 ? h : o.page_size.height, count);
  }
  const Planes P = planes_of(b, b->W, b->H);
  if (!(dis & UPHIP_NO_WIPE)) wipes_uniform(b, P, o.pre_wipes, count);
  if (!(dis & UPHIP_NO_BORDER)) border_uniform(b, P, o.pre_border, count);
  mark(b, "pre");
  // ---- filters (sheet_stages.c:327-357) ---------------------------------
  if (!(dis & UPHIP_NO_BLACKFILTER) && b->bgeo.nbars > 0) {
    launch_blackfilter_impl(cur_ref(P, b->ctl), b->bgeo, b->dbars, b->scr, b->scr_stride, nullptr,
                            b->ctl, count, b->st, b->black_h, b->black_v, vsum_ready, bits_ready,
                            b->nbits_stride, bb_ready, b->nbits_stride, rm_ready);
    mark(b, "blackfilter");
  }
  if (!(dis & UPHIP_NO_NOISEFILTER)) {
    NoiseGeom ng = b->ngeo;
    ng.bbits = bb_ready;
    ng.bb_stride = b->nbits_stride;
    launch_noisefilter(cur_ref(P, b->ctl), ng, b->scr, b->scr_stride, nullptr, b->ctl, count,
                       b->st, bits_ready, b->nbits_stride);
    mark(b, "noisefilter");
  }
  if (!(dis & UPHIP_NO_BLURFILTER)) {
    launch_blurfilter(cur_ref(P, b->ctl), b->blgeo, b->scr, b->scr_stride, nullptr, count, b->st,
                      bb_ready, b->nbits_stride);
    mark(b, "blurfilter");
  }
  bool mask_sums_ready = false;
  bool center_sums_ready = false;  // the second scan's sums came with the rotation
  // ---- masks (sheet_stages.c:359-386): the first detection is dead for a
  // fresh job (its count is discarded and its masks are overwritten before
  // any read), so it is skipped; mask_count is 0 -> no apply_masks.
  if (!(dis & UPHIP_NO_GRAYFILTER)) {
    uint32_t* cs = nullptr;
    if (mask_sums_from_gray(b)) {
      UPH_HIP(hipMemsetAsync(b->sums, 0, sizeof(uint32_t) * b->sums_stride * count, b->st));
      cs = b->sums;  // point 0, horizontal: offset 0
    }
    mask_sums_ready = launch_grayfilter(cur_ref(P, b->ctl), b->ggeo, b->scr, b->scr_stride, nullptr,
                                        count, b->st, cs, b->sums_stride);
    mark(b, "grayfilter");
  }
  // ---- deskew (sheet_stages.c:388-413) ---------------------------------
  if (!(dis & UPHIP_NO_DESKEW)) {
    if (!(dis & UPHIP_NO_MASK_SCAN)) {
      detect_masks_all(b, 1, count, mask_sums_ready);
      mark(b, "masks_deskew");
    }
    const UphipEdges& E = o.deskew_parameters.scan_edges;
    RotGeom rg;
    memset(&rg, 0, sizeof(rg));
    rg.W = b->W;
    rg.H = b->H;
    const int shifts[4][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};
    const bool on[4] = {E.left, E.top, E.right, E.bottom};
    RotSelectArgs ra;
    memset(&ra, 0, sizeof(ra));
    for (int k = 0; k < 4; k++)
      if (on[k]) {
        rg.edge_shift[rg.nedges][0] = shifts[k][0];
        rg.edge_shift[rg.nedges][1] = shifts[k][1];
        ra.negate[rg.nedges] = (k == 1 || k == 3);
        rg.nedges++;
      }
    rg.scan_size = o.deskew_parameters.deskewScanSize;
    rg.scan_depth = o.deskew_parameters.deskewScanDepth;
    rg.max_masks = UPHIP_MAX_PAGES;
    ra.nangles = b->table.nangles;
    ra.nedges = rg.nedges;
    ra.max_masks = UPHIP_MAX_PAGES;
    ra.deviation_rad = o.deskew_parameters.deskewScanDeviationRad;
    // detection of mask i (mask_pick, peaks, select) into rot_args[i]
    auto detect = [&](int i, const int32_t* only) {
      hipLaunchKernelGGL(k_mask_pick, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl, i,
                         b->pick_mask, b->pick_active, count, only);
      launch_rotation_peaks(cur_ref(P, b->ctl), rg, b->dtable, b->pick_mask, b->pick_active, i,
                            b->peaks, count, b->st, b->table.nangles, b->max_scan, b->rot_lines,
                            b->max_angle);
#ifdef UPHIP_DIAG
      if (getenv("UPHIP_DIAG_ROTATION")) {  // tuning build only: lines left to the direct walk
        const int nl = count * rg.nedges * b->table.nangles;
        std::vector<int32_t> fl((size_t)nl);
        UPH_HIP(hipMemcpyAsync(fl.data(), rotation_line_flags(b->rot_lines, nl, b->max_scan),
                               sizeof(int32_t) * nl, hipMemcpyDeviceToHost, b->st));
        UPH_HIP(hipStreamSynchronize(b->st));
        int nf = 0;
        for (int t = 0; t < nl; t++) nf += fl[t] != 0;
        fprintf(stderr, "uphip: batch rotation %d of %d lines walked directly\n", nf, nl);
      }
#endif
      ra.mask_index = i;
      hipLaunchKernelGGL(k_rot_select, dim3(count), dim3(64), 0, b->st, b->ctl,
                         b->peaks, b->dtable, b->dcombo, ra, b->rot_args + (int64_t)i * b->cap,
                         count, only, b->dpow2, b->npow2);
    };
    const bool linear = o.interpolate_type == UPHIP_INTERP_LINEAR &&
                        (P.fmt == F_GRAY8 || P.fmt == F_RGB24);
    // rotations are angles of the scan table, |angle| <= scan range
    auto rotate = [&](const RotateArgs* args, int nmask, const int32_t* indep,
                      uint32_t* colsum = nullptr) {
      if (linear && launch_rotate_linear(cur_ref(P, b->ctl), other_ref(P, b->ctl), args, nmask,
                                         b->cap, indep, count, b->st, b->max_angle))
        return false;
      return launch_rotate_mask(cur_ref(P, b->ctl), other_ref(P, b->ctl), args,
                                o.interpolate_type, count, b->st, b->max_angle, colsum,
                                b->sums_stride);
    };
    if (linear && b->points.size() == 2) {
      // both masks detected on the same image, rotated in one launch where
      // independent (k_rot_independent); mask 1 again after mask 0 elsewhere
      detect(0, nullptr);
      detect(1, nullptr);
      hipLaunchKernelGGL(k_rot_independent, dim3((count + 255) / 256), dim3(256), 0, b->st,
                         b->ctl, b->rot_args, (int64_t)b->cap, b->rot_indep, b->rot_dep, count);
      mark(b, "deskew_detect");
      rotate(b->rot_args, 2, b->rot_indep);
      mark(b, "deskew_rotate");  // brackets exactly the rotation kernel
      hipLaunchKernelGGL(k_flip_rot2, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl,
                         b->rot_args, (int64_t)b->cap, b->rot_indep, count);
      RotateArgs* a1 = b->rot_args + b->cap;
      detect(1, b->rot_dep);
      mark(b, "deskew_detect");
      rotate(a1, 1, nullptr);
      mark(b, "deskew_rotate");
      launch_flip_if_active(b->ctl, &a1->active, sizeof(RotateArgs), count, b->st);
    } else {
      for (size_t i = 0; i < b->points.size(); i++) {
        detect((int)i, nullptr);
        RotateArgs* ai = b->rot_args + (int64_t)i * b->cap;
        const bool fuse = mask_sums_from_rotate(b);
        if (fuse)
          hipLaunchKernelGGL(k_zero_sums_if_active, dim3(4, count), dim3(256), 0, b->st, ai,
                             b->sums, b->sums_stride, b->W);
        mark(b, "deskew_detect");
        center_sums_ready = rotate(ai, 1, nullptr, fuse ? b->sums : nullptr);
        mark(b, "deskew_rotate");  // brackets exactly the rotation kernel
        launch_flip_if_active(b->ctl, &ai->active, sizeof(RotateArgs), count, b->st);
      }
    }
  }
  // ---- post (sheet_stages.c:415-534) -------------------------------------
  const bool rows_fused = border_rows_from_center(b);
  const bool chain = chain_center_align(b);
  MoveArgs* const center_mv = chain ? b->move_args + b->cap : nullptr;  // align uses [0, cap)
  if (!(dis & UPHIP_NO_MASK_CENTER)) {
    if (!(dis & UPHIP_NO_MASK_SCAN)) {
      detect_masks_all(b, 1, count, center_sums_ready);
      mark(b, "masks_center");
    }
    for (size_t i = 0; i < b->points.size(); i++) {
      MoveArgs* mv = chain ? center_mv : b->move_args;  // reuse the first cap entries
      hipLaunchKernelGGL(k_center_args, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl,
                         (int)i, b->W, b->H, o.sheet_background, mv, count);
      if (rows_fused && i + 1 == b->points.size()) {
        // the last move also counts the border scan's dark pixels per row
        MoveExtra x = center_count_args(b);
        x.dry = chain;  // chained: count C's rows from R, write nothing
        if (chain && border_edge_rows_only(b)) {  // the rows near the edges first
          x.ya0 = 0;
          x.ya1 = kBorderEdgeRows;
          x.yb0 = b->H - kBorderEdgeRows;
          x.yb1 = b->H;
        }
        launch_move_rect_fused(cur_ref(P, b->ctl), other_ref(P, b->ctl), mv, x, count, b->st);
      } else {
        launch_move_rect(cur_ref(P, b->ctl), other_ref(P, b->ctl), mv, count, b->st);
      }
      if (!chain) launch_flip_if_active(b->ctl, &mv->active, sizeof(MoveArgs), count, b->st);
    }
    mark(b, "center");
  }
  if (!(dis & UPHIP_NO_WIPE)) {
    UphipWipes wp = o.wipes;
    if (o.layout == UPHIP_LAYOUT_DOUBLE && (o.middle_wipe[0] > 0 || o.middle_wipe[1] > 0) &&
        wp.count < UPHIP_MAX_MASKS) {
      wp.areas[wp.count++] = from_rect(Rect{b->W / 2 - o.middle_wipe[0], 0,
                                            b->W / 2 + o.middle_wipe[1], b->H - 1});
    }
    wipes_uniform(b, P, wp, count);
  }
  if (!(dis & UPHIP_NO_BORDER)) border_uniform(b, P, o.border, count);
  if (!(dis & UPHIP_NO_BORDER_SCAN) && !b->outside.empty()) {
    border_all(b, count, rows_fused, center_mv);
    mark(b, "border");
  }
  if (!(dis & UPHIP_NO_WIPE)) wipes_uniform(b, P, o.post_wipes, count);
  if (!(dis & UPHIP_NO_BORDER)) border_uniform(b, P, o.post_border, count);
  w = b->W;
  h = b->H;
  if (o.post_mirror.horizontal || o.post_mirror.vertical) {
    const Planes Q = planes_of(b, w, h);
    launch_mirror_oop(cur_ref(Q, b->ctl), other_ref(Q, b->ctl), o.post_mirror.horizontal,
                      o.post_mirror.vertical, o.abs_black_threshold, count, b->st);
    flip_all(b, count);
  }
  if (o.post_shift.horizontal != 0 || o.post_shift.vertical != 0) {
    const Planes Q = planes_of(b, w, h);
    const uint8_t bg[3] = {o.sheet_background.r, o.sheet_background.g, o.sheet_background.b};
    launch_shift(cur_ref(Q, b->ctl), other_ref(Q, b->ctl), o.post_shift.horizontal,
                 o.post_shift.vertical, bg, o.abs_black_threshold, count, b->st);
    flip_all(b, count);
  }
  if (o.post_rotate != 0) {
    const Planes S = planes_of(b, w, h), D = planes_of(b, h, w);
    launch_rotate90_thr(cur_ref(S, b->ctl), other_ref(D, b->ctl), o.post_rotate / 90,
                        o.abs_black_threshold, count, b->st);
    flip_all(b, count);
    std::swap(w, h);
  }
  {
    int32_t sw = o.post_stretch_size.width == -1 ? w : o.post_stretch_size.width;
    int32_t sh = o.post_stretch_size.height == -1 ? h : o.post_stretch_size.height;
    sw *= o.post_zoom_factor;
    sh *= o.post_zoom_factor;
    stretch_all(b, w, h, sw, sh, count);
    if (o.post_page_size.width != -1 || o.post_page_size.height != -1)
      resize_all(b, w, h, o.post_page_size.width == -1 ? w : o.post_page_size.width,
                 o.post_page_size.height == -1 ? h : o.post_page_size.height, count);
  }
  // ---- output (sheet_stages.c:536-631, saveImage file.c:187-259) --------
  if (b->out) {
    Planes Q = planes_of(b, w, h);
    Planes O;
    O.base[0] = O.base[1] = b->out;
    O.pitch = b->out_pitch;
    O.stride = b->out_stride;
    O.W = w;
    O.H = h;
    O.fmt = b->out_fmt;
    O.count = count;
    CopyArgs ca{Rect{0, 0, w - 1, h - 1}, 0, 0, 1};
    launch_copy_thr(cur_ref(Q, b->ctl), fixed_ref(O, 0), replicate(b, ca), count, h,
                    o.abs_black_threshold, b->st);
  }
  mark(b, "output");
  hipLaunchKernelGGL(k_status_fold, dim3((count + 255) / 256), dim3(256), 0, b->st, b->ctl, count,
                     b->sticky);
  b->last_count = count;
  return uphip_last_error() == nullptr;
}

extern "C" {

UphipBatch* uphip_batch_create(const UphipOptions* options, const UphipBatchGeometry* geometry) {
  if (!options || !geometry) return fail("batch_create: null argument"), nullptr;
  if (!runtime_ready()) return fail("batch_create: no HIP device"), nullptr;
  if (geometry->capacity <= 0 || geometry->page_width <= 0 || geometry->page_height <= 0)
    return fail("batch_create: invalid geometry"), nullptr;
  if (options->input_count < 1 || options->input_count > UPHIP_MAX_PAGES)
    return fail("batch_create: input_count must be 1 or 2"), nullptr;
  if (geometry->page_format < UPHIP_FMT_GRAY8 || geometry->page_format > UPHIP_FMT_MONOBLACK)
    return fail("batch_create: invalid page format"), nullptr;
  UphipBatch* b = new UphipBatch();
  b->o = *options;
  b->geo = *geometry;
  b->cap = geometry->capacity;
  b->n_in = options->input_count;
  b->device = current_device();
  hipSetDevice(b->device);
  if (!UPH_HIP(hipStreamCreateWithFlags(&b->st, hipStreamNonBlocking)) || !plan(b) ||
      !allocate(b)) {
    uphip_batch_destroy(b);
    return nullptr;
  }
  return b;
}

void uphip_batch_destroy(UphipBatch* b) {
  if (!b) return;
  hipSetDevice(b->device);
  if (b->st) hipStreamSynchronize(b->st);
  for (auto& r : b->runs)
    for (auto& m : r) hipEventDestroy(m.second);
  for (void* p : b->allocs) hipFree(p);
  delete b->jenc;
  if (b->st) hipStreamDestroy(b->st);
  delete b;
}

int uphip_batch_output_info(UphipBatch* b, int32_t* width, int32_t* height, int32_t* format,
                            int64_t* bytes_per_sheet) {
  if (!b) return -1;
  if (width) *width = b->out_w;
  if (height) *height = b->out_h;
  if (format) *format = b->out_fmt;
  if (bytes_per_sheet) *bytes_per_sheet = row_bytes(b->out_w, b->out_fmt) * b->out_h;
  return 0;
}

int uphip_batch_device_bytes(UphipBatch* b, int64_t* bytes) {
  if (!b || !bytes) return fail("batch_device_bytes: null argument"), -1;
  *bytes = (int64_t)b->dev_bytes;
  return 0;
}

void* uphip_batch_input_ptr(UphipBatch* b, int32_t slot, int64_t* pitch) {
  if (!b || slot < 0 || slot >= b->cap * b->n_in) return nullptr;
  if (pitch) *pitch = b->in_pitch;
  return b->inputs + (int64_t)slot * b->in_page_stride;
}

int uphip_batch_set_input(UphipBatch* b, int32_t slot, const void* host, int64_t linesize) {
  if (!b || slot < 0 || slot >= b->cap * b->n_in) return fail("batch_set_input: bad slot"), -1;
  hipSetDevice(b->device);
  const int64_t rb = row_bytes(b->geo.page_width, b->geo.page_format);
  return UPH_HIP(hipMemcpy2DAsync(b->inputs + (int64_t)slot * b->in_page_stride, b->in_pitch, host,
                                  linesize, rb, b->geo.page_height, hipMemcpyHostToDevice, b->st))
             ? 0
             : -1;
}

int uphip_batch_run(UphipBatch* b, int32_t count) {
  if (!b || count <= 0 || count > b->cap) return fail("batch_run: bad count"), -1;
  hipSetDevice(b->device);
  return run_batch(b, count, b->inputs, b->in_pitch, b->in_page_stride) ? 0 : -1;
}

int uphip_batch_run_device(UphipBatch* b, int32_t count, const void* pages, int64_t pitch,
                           int64_t page_stride) {
  if (!b || count <= 0 || count > b->cap || !pages)
    return fail("batch_run_device: bad arguments"), -1;
  if (pitch < row_bytes(b->geo.page_width, b->geo.page_format))
    return fail("batch_run_device: pitch too small"), -1;
  hipSetDevice(b->device);
  return run_batch(b, count, (const uint8_t*)pages, pitch, page_stride) ? 0 : -1;
}

int uphip_batch_wait(UphipBatch* b) {
  if (!b) return -1;
  hipSetDevice(b->device);
  if (!UPH_HIP(hipStreamSynchronize(b->st))) return -1;
  // surface device-side failures (overflowing candidate lists / DFS stack) of
  // every run since the previous wait, then re-arm the sticky word
  int32_t any = 0;
  if (!UPH_HIP(hipMemcpy(&any, b->sticky, sizeof(any), hipMemcpyDeviceToHost))) return -1;
  if (!any) return 0;
  UPH_HIP(hipMemset(b->sticky, 0, sizeof(int32_t)));
  std::vector<SheetCtl> c(b->last_count > 0 ? b->last_count : 1);
  if (b->last_count > 0) {
    UPH_HIP(hipMemcpy(c.data(), b->ctl, sizeof(SheetCtl) * b->last_count,
                      hipMemcpyDeviceToHost));
    for (int s = 0; s < b->last_count; s++)
      if (c[s].status)
        return fail("batch: sheet %d failed on the device (status 0x%x)", s, c[s].status), -1;
  }
  return fail("batch: a sheet of an earlier run since the last wait failed on the device "
              "(status 0x%x)", any), -1;
}

void* uphip_batch_output_ptr(UphipBatch* b, int32_t sheet, int64_t* pitch) {
  if (!b || sheet < 0 || sheet >= b->cap) return nullptr;
  // the pointer is handed out only once the batch's kernels have finished
  // writing it (the caller may read it from any stream or the host)
  hipSetDevice(b->device);
  if (!UPH_HIP(hipStreamSynchronize(b->st))) return nullptr;
  if (b->out) {
    if (pitch) *pitch = b->out_pitch;
    return b->out + (int64_t)sheet * b->out_stride;
  }
  int32_t cur = 0;
  hipMemcpy(&cur, &b->ctl[sheet].cur, 4, hipMemcpyDeviceToHost);
  if (pitch) *pitch = b->pitch;
  return b->planes[cur] + (int64_t)sheet * b->plane_stride;
}

int uphip_batch_get_output(UphipBatch* b, int32_t sheet, void* host, int64_t linesize) {
  int64_t pitch = 0;
  void* p = uphip_batch_output_ptr(b, sheet, &pitch);
  if (!p) return fail("batch_get_output: bad sheet"), -1;
  const int64_t rb = row_bytes(b->out_w, b->out_fmt);
  if (linesize < rb) return fail("batch_get_output: linesize too small"), -1;
  if (!UPH_HIP(hipMemcpy2DAsync(host, linesize, p, pitch, rb, b->out_h, hipMemcpyDeviceToHost,
                                b->st)))
    return -1;
  return UPH_HIP(hipStreamSynchronize(b->st)) ? 0 : -1;
}

int uphip_batch_get_report(UphipBatch* b, int32_t sheet, UphipSheetReport* r) {
  if (!b || !r || sheet < 0 || sheet >= b->cap) return -1;
  SheetCtl c;
  hipSetDevice(b->device);
  hipStreamSynchronize(b->st);
  if (!UPH_HIP(hipMemcpy(&c, &b->ctl[sheet], sizeof(c), hipMemcpyDeviceToHost))) return -1;
  memset(r, 0, sizeof(*r));
  r->mask_count = c.mask_count;
  for (int i = 0; i < UPHIP_MAX_PAGES; i++) {
    r->masks[i] = c.masks[i];
    r->rotation[i] = c.rotation[i];
    r->border_masks[i] = c.border_masks[i];
  }
  r->width = b->out_w;
  r->height = b->out_h;
  r->flags = (uint32_t)c.status;
  return 0;
}

void* uphip_batch_stream(UphipBatch* b) { return b ? (void*)b->st : nullptr; }

int uphip_batch_output_pitch(UphipBatch* b, int64_t* pitch) {
  if (!b || !pitch) return -1;
  *pitch = b->out ? b->out_pitch : b->pitch;
  return 0;
}

int uphip_batch_query(UphipBatch* b) {
  if (!b) return -1;
  hipSetDevice(b->device);
  const hipError_t e = hipStreamQuery(b->st);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return check_hip(e, "hipStreamQuery"), -1;
}

int uphip_batch_upload_async(UphipBatch* b, int32_t count, const void* host, int64_t linesize,
                             int64_t page_stride) {
  if (!b || !host || count <= 0 || count > b->cap)
    return fail("batch_upload_async: bad arguments"), -1;
  const int64_t rb = row_bytes(b->geo.page_width, b->geo.page_format);
  if (linesize < rb) return fail("batch_upload_async: linesize too small"), -1;
  hipSetDevice(b->device);
  const int64_t n = (int64_t)count * b->n_in;
  const uint8_t* h = (const uint8_t*)host;
  if (linesize == b->in_pitch && page_stride == b->in_page_stride)  // staging laid out like the slots
    return UPH_HIP(hipMemcpyAsync(b->inputs, h, (size_t)(n * page_stride), hipMemcpyHostToDevice,
                                  b->st))
               ? 0
               : -1;
  for (int64_t i = 0; i < n; i++)
    if (!UPH_HIP(hipMemcpy2DAsync(b->inputs + i * b->in_page_stride, b->in_pitch,
                                  h + i * page_stride, linesize, rb, b->geo.page_height,
                                  hipMemcpyHostToDevice, b->st)))
      return -1;
  return 0;
}

int uphip_batch_download_async(UphipBatch* b, void* host, int64_t linesize, int64_t sheet_stride) {
  if (!b || !host || b->last_count <= 0) return fail("batch_download_async: nothing to download"), -1;
  const int64_t rb = row_bytes(b->out_w, b->out_fmt);
  if (linesize < rb) return fail("batch_download_async: linesize too small"), -1;
  hipSetDevice(b->device);
  const hipError_t q = hipStreamQuery(b->st);
  if (q == hipErrorNotReady) return fail("batch_download_async: the run has not finished"), -1;
  if (!check_hip(q, "hipStreamQuery")) return -1;
  const int n = b->last_count;
  // which plane holds each sheet (ctl[s].cur; the stream is idle)
  std::vector<int32_t> cur((size_t)n, 0);
  if (!b->out &&
      !UPH_HIP(hipMemcpy2D(cur.data(), sizeof(int32_t), &b->ctl[0].cur, sizeof(SheetCtl),
                           sizeof(int32_t), n, hipMemcpyDeviceToHost)))
    return -1;
  uint8_t* h = (uint8_t*)host;
  const int64_t sp = b->out ? b->out_pitch : b->pitch;
  const int64_t ss = b->out ? b->out_stride : b->plane_stride;
  auto src_of = [&](int s) -> const uint8_t* {
    return b->out ? b->out + (int64_t)s * ss : b->planes[cur[s] & 1] + (int64_t)s * ss;
  };
  if (linesize == sp && sheet_stride == sp * b->out_h && ss == sheet_stride) {
    // host staging laid out like the planes: runs of sheets in the same plane
    // go as one linear DMA copy (2D copies run far below the link rate); the
    // last sheet of a run ends at its last row, so a caller's buffer need not
    // pad its final sheet to a whole stride
    const int64_t extent = (int64_t)(b->out_h - 1) * sp + rb;
    for (int s = 0; s < n;) {
      int e = s + 1;
      while (e < n && (b->out || (cur[e] & 1) == (cur[s] & 1))) e++;
      if (!UPH_HIP(hipMemcpyAsync(h + s * sheet_stride, src_of(s), (size_t)((e - s - 1) * ss + extent),
                                  hipMemcpyDeviceToHost, b->st)))
        return -1;
      s = e;
    }
    return 0;
  }
  for (int s = 0; s < n; s++)
    if (!UPH_HIP(hipMemcpy2DAsync(h + s * sheet_stride, linesize, src_of(s), sp, rb, b->out_h,
                                  hipMemcpyDeviceToHost, b->st)))
      return -1;
  return 0;
}

// ---- GPU JPEG output branch (sheet_stages.c:554-581) -----------------------
int uphip_batch_encode_jpeg_async(UphipBatch* b, int32_t quality, int32_t sampling) {
  if (!b || b->last_count <= 0) return fail("batch_encode_jpeg: nothing to encode"), -1;
  if (quality == 0) quality = UPHIP_JPEG_DEFAULT_QUALITY;
  hipSetDevice(b->device);
  const int oc = b->o.output_count < 1 ? 1 : b->o.output_count;
  const int n = b->last_count * oc;
  const int bpp = b->work_fmt == F_GRAY8 ? 1 : 3;
  const int32_t pw = b->out_w / oc;
  // bit stream per page: the page's pixel bytes (+64 KiB); pages that do not
  // fit (noise at high quality) come back as -1 for a single re-encode
  const int64_t page = (int64_t)pw * b->out_h * bpp + (64 << 10);
  if (!b->jenc) b->jenc = new JencContext();
  JencContext& c = *b->jenc;
  if (!c.setup(pw, b->out_h, b->work_fmt == F_GRAY8 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24, sampling,
               quality, n, page / 4, page * n, b->st))
    return -1;
  hipLaunchKernelGGL(k_jenc_sources, dim3((n + 255) / 256), dim3(256), 0, b->st, b->ctl,
                     b->planes[0], b->planes[1], b->pitch, b->plane_stride, oc,
                     (int64_t)pw * bpp, c.B.images, n);
  if (!c.encode_async(b->st)) return -1;
  b->jenc_pages = n;
  return 0;
}

int64_t uphip_batch_jpeg_sizes(UphipBatch* b, int64_t* sizes, int32_t max_pages) {
  if (!b || !b->jenc || b->jenc_pages <= 0) return fail("batch_jpeg_sizes: no encode"), -1;
  if (uphip_batch_query(b) != 1) return fail("batch_jpeg_sizes: the encode has not finished"), -1;
  int64_t total = 0;
  for (int i = 0; i < b->jenc_pages; i++) {
    const int64_t s = b->jenc->host_sizes[i];
    if (sizes && i < max_pages) sizes[i] = s < 0 ? -1 : s;
    if (s > 0) total += s;
  }
  return total;
}

int uphip_batch_jpeg_download_async(UphipBatch* b, void* host, int64_t capacity) {
  const int64_t total = uphip_batch_jpeg_sizes(b, nullptr, 0);
  if (total < 0) return -1;
  if (!host || capacity < total) return fail("batch_jpeg_download: buffer too small"), -1;
  if (total == 0) return 0;
  hipSetDevice(b->device);
  return UPH_HIP(hipMemcpyAsync(host, b->jenc->out, (size_t)total, hipMemcpyDeviceToHost, b->st))
             ? 0
             : -1;
}

int uphip_batch_jpeg_page(UphipBatch* b, int32_t page, const void** device_src, int64_t* pitch,
                          int32_t* width, int32_t* height, int32_t* format) {
  const int oc = b && b->o.output_count > 1 ? b->o.output_count : 1;
  if (!b || page < 0 || page >= b->last_count * oc) return fail("batch_jpeg_page: bad page"), -1;
  hipSetDevice(b->device);
  if (!UPH_HIP(hipStreamSynchronize(b->st))) return -1;
  const int s = page / oc, j = page % oc;
  int32_t cur = 0;
  if (!UPH_HIP(hipMemcpy(&cur, &b->ctl[s].cur, 4, hipMemcpyDeviceToHost))) return -1;
  const int bpp = b->work_fmt == F_GRAY8 ? 1 : 3;
  const int32_t pw = b->out_w / oc;
  if (device_src)
    *device_src = b->planes[cur & 1] + (int64_t)s * b->plane_stride + (int64_t)j * pw * bpp;
  if (pitch) *pitch = b->pitch;
  if (width) *width = pw;
  if (height) *height = b->out_h;
  if (format) *format = b->work_fmt == F_GRAY8 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24;
  return 0;
}

int uphip_batch_set_timing(UphipBatch* b, int32_t enable) {
  if (!b) return -1;
  b->timing = enable != 0;
  return 0;
}

int uphip_batch_kernel_times(UphipBatch* b, const char** names, float* ms, int max_entries) {
  // per-stage totals over every run since the previous query (the events
  // bracket each stage on the batch stream); the record is then cleared
  if (!b) return -1;
  hipSetDevice(b->device);
  if (!UPH_HIP(hipStreamSynchronize(b->st))) return -1;
  std::vector<std::string> order;
  std::vector<double> tot;
  for (auto& r : b->runs) {
    for (size_t i = 1; i < r.size(); i++) {
      float t = 0.0f;
      hipEventElapsedTime(&t, r[i - 1].second, r[i].second);
      size_t k = 0;
      while (k < order.size() && order[k] != r[i].first) k++;
      if (k == order.size()) {
        order.push_back(r[i].first);
        tot.push_back(0.0);
      }
      tot[k] += t;
    }
    for (auto& m : r) hipEventDestroy(m.second);
  }
  b->runs.clear();
  b->time_names = order;
  int k = 0;
  for (; k < (int)order.size() && k < max_entries; k++) {
    if (names) names[k] = b->time_names[k].c_str();
    if (ms) ms[k] = (float)tot[k];
  }
  return k;
}

}  // extern "C"
