// ops_filters.hip — filter and rotation-detection ops of the C ABI
// (imageprocess/filters.c, deskew.c peers) for single device frames.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "filters.h"
#include "mono_proxy.h"
#include "runtime.h"

using namespace uph;

static bool ready(const UphipImage& im, const char* op) {
  if (!im.frame) return fail("%s: image has no frame", op);
  if (!runtime_ready()) return fail("%s: no HIP device", op);
  hipSetDevice(im.frame->device);
  return true;
}

static PlaneRef ref1(const UphipFrame* f) { return fixed_ref(frame_planes(f), 0); }

// The peaks of every enabled edge (left, top, right, bottom) x angle
// (detect_edge_rotation_peak, deskew.c:48-146, for each angle of
// detect_edge_rotation's loop, deskew.c:153-174) into hp[edge * na + angle].
static bool rotation_peaks(const UphipImage& image, UphipRectangle mask,
                           const UphipDeskewParameters& params, RotTable& table, bool (&on)[4],
                           std::vector<int32_t>& hp) {
  if (rotation_angles(params, &table) < 0)
    return fail("detect_rotation: more than %d angles", kMaxAngles);
  const int na = table.nangles;
  RotGeom g;
  g.W = image.frame->width;
  g.H = image.frame->height;
  g.nedges = 0;
  const UphipEdges& E = params.scan_edges;
  const int shifts[4][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};  // left, top, right, bottom
  on[0] = E.left;
  on[1] = E.top;
  on[2] = E.right;
  on[3] = E.bottom;
  for (int k = 0; k < 4; k++)
    if (on[k]) {
      g.edge_shift[g.nedges][0] = shifts[k][0];
      g.edge_shift[g.nedges][1] = shifts[k][1];
      g.nedges++;
    }
  g.scan_size = params.deskewScanSize;
  g.scan_depth = params.deskewScanDepth;
  g.max_masks = 1;
  hipStream_t st = current_stream();
  RotTable* dt = (RotTable*)scratch(4, sizeof(RotTable));
  Rect* dm = (Rect*)scratch(5, sizeof(Rect));
  int32_t* peaks = (int32_t*)scratch(6, sizeof(int32_t) * 4 * (size_t)(na > 0 ? na : 1));
  if (!dt || !dm || !peaks) return false;
  Rect m = to_rect(mask);
  UPH_HIP(hipMemcpyAsync(dt, &table, sizeof(RotTable), hipMemcpyHostToDevice, st));
  UPH_HIP(hipMemcpyAsync(dm, &m, sizeof(Rect), hipMemcpyHostToDevice, st));
  const int32_t mw = iabs(m.x0 - m.x1) + 1, mh = iabs(m.y0 - m.y1) + 1;
  int max_scan = params.deskewScanSize == -1 ? imax(mw, mh) : params.deskewScanSize;
  max_scan = imin(imin(max_scan, 10000), imax(mw, mh));
  int32_t* lines = (int32_t*)scratch(7, rotation_lines_bytes(1, g.nedges, na, max_scan));
  if (!lines) return false;
  float max_angle = 0.0f;
  for (int i = 0; i < na; i++) max_angle = fmaxf(max_angle, fabsf(table.angle[i]));
  launch_rotation_peaks(ref1(image.frame), g, dt, dm, nullptr, 0, peaks, 1, st, na, max_scan,
                        lines, max_angle);
  hp.assign(4 * (size_t)(na > 0 ? na : 1), 0);
  UPH_HIP(hipMemcpyAsync(hp.data(), peaks, sizeof(int32_t) * g.nedges * na,
                         hipMemcpyDeviceToHost, st));
#ifdef UPHIP_DIAG
  if (getenv("UPHIP_DIAG_ROTATION")) {  // tuning build only: lines left to the direct walk
    std::vector<int32_t> fl((size_t)g.nedges * na);
    UPH_HIP(hipMemcpyAsync(fl.data(), rotation_line_flags(lines, g.nedges * na, max_scan),
                           sizeof(int32_t) * fl.size(), hipMemcpyDeviceToHost, st));
    UPH_HIP(hipStreamSynchronize(st));
    int nf = 0;
    for (int32_t f : fl) nf += f != 0;
    fprintf(stderr, "uphip: detect_rotation %d of %d lines walked directly\n", nf, (int)fl.size());
  }
#endif
  return UPH_HIP(hipStreamSynchronize(st));
}

extern "C" {

void uphip_grayfilter(UphipImage image0, UphipGrayfilterParameters params) {
  // grayfilter_cpu, filters.c:370-402
  if (!ready(image0, "grayfilter")) return;
  MonoProxy mp(image0, true, "grayfilter");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return;
  const UphipImage image = mp.image();
  GrayGeom g;
  if (!gray_geometry(image.frame->width, image.frame->height, params, image.abs_black_threshold,
                     &g))
    return (void)fail("grayfilter: invalid scan size/step");
  hipStream_t st = current_stream();
  void* scr = scratch(2, gray_scratch_bytes(g));
  if (!scr) return;
  launch_grayfilter(ref1(image.frame), g, scr, 0, nullptr, 1, st);
  mp.finish();
}

void uphip_blurfilter(UphipImage image0, UphipBlurfilterParameters params,
                      uint8_t abs_white_threshold) {
  // blurfilter_cpu, filters.c:149-232
  if (!ready(image0, "blurfilter")) return;
  MonoProxy mp(image0, true, "blurfilter");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return;
  const UphipImage image = mp.image();
  BlurGeom g;
  if (!blur_geometry(image.frame->width, image.frame->height, params, abs_white_threshold, &g))
    return (void)fail("blurfilter: invalid scan size");
  void* scr = scratch(2, blur_scratch_bytes(g));
  if (!scr) return;
  launch_blurfilter(ref1(image.frame), g, scr, 0, nullptr, 1, current_stream());
  mp.finish();
}

void uphip_noisefilter(UphipImage image0, uint64_t intensity, uint8_t min_white_level) {
  // noisefilter_cpu, filters.c:309-338
  if (!ready(image0, "noisefilter")) return;
  MonoProxy mp(image0, true, "noisefilter");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return;
  const UphipImage image = mp.image();
  NoiseGeom g;
  noise_geometry(image.frame->width, image.frame->height, intensity, min_white_level, &g);
  if (intensity > 64) return (void)fail("noisefilter: intensity > 64 unsupported");
  const size_t bytes = noise_scratch_bytes(g);
  void* scr = scratch(2, bytes);
  SheetCtl* ctl = (SheetCtl*)scratch(3, sizeof(SheetCtl));
  if (!scr || !ctl) return;
  hipStream_t st = current_stream();
  UPH_HIP(hipMemsetAsync(ctl, 0, sizeof(SheetCtl), st));
  launch_noisefilter(ref1(image.frame), g, scr, (int64_t)bytes, nullptr, ctl, 1, st);
  int32_t status = 0;
  UPH_HIP(hipMemcpyAsync(&status, &ctl->status, 4, hipMemcpyDeviceToHost, st));
  UPH_HIP(hipStreamSynchronize(st));
  if (status) return (void)fail("noisefilter: candidate list overflow (status %d)", status);
  mp.finish();
}

void uphip_blackfilter(UphipImage image0, UphipBlackfilterParameters params) {
  // blackfilter_cpu, filters.c:111-127
  if (!ready(image0, "blackfilter")) return;
  MonoProxy mp(image0, true, "blackfilter");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return;
  const UphipImage image = mp.image();
  const int32_t W = image.frame->width, H = image.frame->height;
  if (image.abs_black_threshold == 255)
    return (void)fail("blackfilter: abs_black_threshold 255 makes the reference fill recurse "
                      "forever");
  std::vector<BlackBar> bars(2 * (size_t)(W + H) + 16);
  BlackGeom g;
  if (!black_geometry(W, H, params, image.abs_black_threshold, &g, bars.data(), (int)bars.size()))
    return (void)fail("blackfilter: invalid scan parameters");
  if (g.nbars == 0) return;
  hipStream_t st = current_stream();
  const size_t bytes = black_scratch_bytes(g);
  void* scr = scratch(2, bytes);
  BlackBar* dbars = (BlackBar*)scratch(4, sizeof(BlackBar) * g.nbars);
  SheetCtl* ctl = (SheetCtl*)scratch(3, sizeof(SheetCtl));
  if (!scr || !dbars || !ctl) return;
  UPH_HIP(hipMemcpyAsync(dbars, bars.data(), sizeof(BlackBar) * g.nbars, hipMemcpyHostToDevice,
                         st));
  UPH_HIP(hipMemsetAsync(ctl, 0, sizeof(SheetCtl), st));
  AxisArgs ah{g.hregion, 0, 1}, av{g.vregion, 0, 1};
  AxisArgs* dah = stage_args(&ah, 1, st);
  AxisArgs* dav = stage_args(&av, 1, st);
  if (!dah || !dav) return;
  launch_blackfilter_impl(ref1(image.frame), g, dbars, scr, (int64_t)bytes, nullptr, ctl, 1, st,
                          dah, dav);
  arg_fence(st);
  int32_t status = 0;
  UPH_HIP(hipMemcpyAsync(&status, &ctl->status, 4, hipMemcpyDeviceToHost, st));
  UPH_HIP(hipStreamSynchronize(st));
  if (status) return (void)fail("blackfilter: flood-fill stack overflow (status %d)", status);
  mp.finish();
}

float uphip_detect_rotation(UphipImage image0, UphipRectangle mask,
                            const UphipDeskewParameters params) {
  // detect_rotation_cpu, deskew.c:181-241: peaks on the GPU, the per-edge
  // argmax and the mean/deviation on the host exactly as the reference does
  if (!ready(image0, "detect_rotation")) return 0.0f;
  MonoProxy mp(image0, false, "detect_rotation");  // 1-bit frames: GRAY8 proxy (mono_proxy.h)
  if (!mp.ok()) return 0.0f;
  static thread_local RotTable table;
  bool on[4];
  std::vector<int32_t> hp;
  if (!rotation_peaks(mp.image(), mask, params, table, on, hp)) return 0.0f;
  const int na = table.nangles;
  float rot[4];
  int count = 0, e = 0;
  for (int k = 0; k < 4; k++) {
    if (!on[k]) continue;
    // detect_edge_rotation, deskew.c:153-174: first strictly larger peak
    int max_peak = 0;
    float detected = 0.0;
    for (int a = 0; a < na; a++) {
      const int peak = hp[(size_t)e * na + a];
      if (peak > max_peak) {
        detected = table.angle[a];
        max_peak = peak;
      }
    }
    rot[count++] = (k == 1 || k == 3) ? -detected : detected;
    e++;
  }
  return combine_edge_rotations(rot, count, params.deskewScanDeviationRad);
}

int32_t uphip_detect_rotation_peaks(UphipImage image0, UphipRectangle mask,
                                    const UphipDeskewParameters params, int32_t* peaks,
                                    int32_t capacity) {
  // the per-line peaks behind uphip_detect_rotation (deskew.c:48-146)
  if (!peaks || capacity < 0) return fail("detect_rotation_peaks: bad arguments"), -1;
  if (!ready(image0, "detect_rotation_peaks")) return -1;
  MonoProxy mp(image0, false, "detect_rotation_peaks");
  if (!mp.ok()) return -1;
  static thread_local RotTable table;
  bool on[4];
  std::vector<int32_t> hp;
  if (!rotation_peaks(mp.image(), mask, params, table, on, hp)) return -1;
  const int n = (on[0] + on[1] + on[2] + on[3]) * table.nangles;
  if (n > capacity) return fail("detect_rotation_peaks: %d peaks, capacity %d", n, capacity), -1;
  for (int i = 0; i < n; i++) peaks[i] = hp[(size_t)i];
  return n;
}

}  // extern "C"

