/* synth.h — deterministic synthetic scanned pages (BASELINE.md §3 workload).
 *
 * Integer-only and stateless per pixel, so the HIP kernel (bench inputs
 * generated straight into HBM) and the host function (CPU baseline, tests)
 * produce identical bytes.  A page: white paper, a skewed text block with
 * >= 150 px white margins (detect_edge terminates), ~2000 salt
 * specks (noisefilter), light-gray blotches (grayfilter), and on every 4th
 * page a dark 40 px band at the left edge (blackfilter flood fill).
 */
#ifndef UNPAPER_HIP_SYNTH_H
#define UNPAPER_HIP_SYNTH_H

#include <stdint.h>

#ifdef __HIPCC__
#define SYNTH_FN __host__ __device__ static inline
#else
#define SYNTH_FN static inline
#endif

#define SYNTH_SEED 0x756E7061706572ull /* "unpaper" */

SYNTH_FN uint64_t synth_mix(uint64_t z) { /* splitmix64 finaliser */
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

SYNTH_FN uint64_t synth_h(uint64_t page, uint64_t a, uint64_t b, uint64_t c) {
  return synth_mix((SYNTH_SEED ^ page) + synth_mix(a * 0x100000001B3ull + synth_mix(b + (c << 32))));
}

/* arithmetic (floor) shift for signed values, identical on host and device */
SYNTH_FN int64_t synth_asr(int64_t v, int s) { return v >= 0 ? v >> s : -((-v + (1ll << s) - 1) >> s); }

SYNTH_FN uint8_t synth_pixel(uint32_t page, int32_t W, int32_t H, int32_t x, int32_t y) {
  const uint64_t ph = synth_h(page, 1, 0, 0);
  /* skew: +-[0.3, 2.0] degrees as a Q16 shear slope (tan 0.3deg*65536 = 343) */
  int64_t slope = 343 + (int64_t)(ph % 1946);
  if ((ph >> 20) & 1) slope = -slope;
  const int32_t cx = W / 2, cy = H / 2;
  /* un-skewed coordinates (shear approximation of the rotation) */
  const int64_t dx = x - cx, dy = y - cy;
  const int64_t u = dx + synth_asr(dy * slope, 16) + cx;
  const int64_t v = dy - synth_asr(dx * slope, 16) + cy;
  uint8_t val = 255;
  /* text block */
  const int32_t mx = 150 + (int32_t)(ph >> 24) % 60, my = 170 + (int32_t)(ph >> 32) % 60;
  if (u >= mx && u < W - mx && v >= my && v < H - my) {
    const int64_t lv = v - my;
    const int64_t line = lv / 48, r = lv % 48;
    const uint64_t lh = synth_h(page, 2, (uint64_t)line, 0);
    const int32_t gh = 20 + (int32_t)(lh % 9);
    /* justified lines; one in six ends a paragraph short */
    const int64_t full = W - 2 * mx;
    const int64_t len = (lh >> 8) % 6 == 0 ? full - (int64_t)((lh >> 11) % (uint64_t)(full / 2 + 1))
                                          : full;
    if (r < gh && (u - mx) < len && (lh >> 40) % 23 != 0) {
      const int64_t word = (u - mx) / 40, wu = (u - mx) % 40;
      const uint64_t wh = synth_h(page, 3, (uint64_t)line, (uint64_t)word);
      if (wu < 28 + (int64_t)(wh % 10)) {
        const uint64_t gl = synth_h(page, 4, (uint64_t)(line * 4096 + (u - mx) / 3),
                                    (uint64_t)(r / 3));
        if (gl % 5 < 2) val = (uint8_t)(gl >> 16) % 41;
      }
    }
  }
  /* light-gray blotches (4..8 of 60x60) */
  const int nb = 4 + (int)(ph >> 40) % 5;
  for (int i = 0; i < nb; i++) {
    const uint64_t bh = synth_h(page, 5, (uint64_t)i, 0);
    const int32_t bx = 200 + (int32_t)(bh % (uint64_t)(W > 500 ? W - 400 : 1));
    const int32_t by = 200 + (int32_t)((bh >> 24) % (uint64_t)(H > 500 ? H - 400 : 1));
    if (x >= bx && x < bx + 60 && y >= by && y < by + 60 && val == 255)
      val = (uint8_t)(185 + synth_h(page, 6, (uint64_t)x, (uint64_t)y) % 31);
  }
  /* salt specks: ~6% of 16x16 cells carry one 1..3 px speck */
  {
    const int32_t bx = x >> 4, by = y >> 4;
    const uint64_t sh = synth_h(page, 7, (uint64_t)bx, (uint64_t)by);
    if (sh % 1000 < 58) {
      const int32_t sx = (bx << 4) + (int32_t)((sh >> 10) % 14), sy = (by << 4) + (int32_t)((sh >> 14) % 14);
      const int32_t sw = 1 + (int32_t)((sh >> 18) % 3), shh = 1 + (int32_t)((sh >> 20) % 2);
      if (x >= sx && x < sx + sw && y >= sy && y < sy + shh) val = (uint8_t)((sh >> 24) % 61);
    }
  }
  /* every 4th page: dark band at the left edge */
  if ((page & 3) == 3 && x < 40) val = (uint8_t)(synth_h(page, 8, (uint64_t)x, (uint64_t)y) % 11);
  return val;
}

/* BASELINE configs[3] (C4): a 600 dpi RGB24 double-page scan, W x H = two
 * pages of W/2 x H side by side (pages 2*sheet and 2*sheet + 1), each channel
 * darkened by a per-page tint of 0..8 levels. */
SYNTH_FN uint8_t synth_rgb_channel(uint32_t sheet, int32_t W, int32_t H, int32_t x, int32_t y,
                                   int ch) {
  const int32_t half = W / 2;
  const int right = x >= half;
  const uint32_t pg = 2u * sheet + (uint32_t)right;
  const uint8_t v = synth_pixel(pg, half, H, x - (right ? half : 0), y);
  const uint8_t t = (uint8_t)(synth_h(pg, 9, (uint64_t)ch, 0) % 9);
  return v >= t ? (uint8_t)(v - t) : 0;
}

#endif
