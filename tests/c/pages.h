/* pages.h — the synthetic page the C callers test with (TEST
 * INFRASTRUCTURE: builds an oracle image). */
#pragma once

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/unpaper_hip.h"
#include "../../oracle/oracle.h"

/* A page-like image in format `fmt` (synth.h page, colour tint, alpha ramp). */
static inline OImage host_page(int fmt, int w, int h, uint32_t seed) {
  OImage im = o_create_image((UphipRectangleSize){w, h}, fmt, false, (UphipPixel){255, 255, 255},
                             170);
  uint8_t *g = malloc((size_t)w * h);
  uphip_synth_page_host(g, w, w, h, seed);
  for (int y = 0; y < h; y++) {
    uint8_t *row = im.data + (int64_t)y * im.linesize;
    if (fmt == UPHIP_FMT_MONOWHITE || fmt == UPHIP_FMT_MONOBLACK) memset(row, 0, (size_t)im.linesize);
    for (int x = 0; x < w; x++) {
      const uint8_t v = g[(size_t)y * w + x];
      switch (fmt) {
        case UPHIP_FMT_GRAY8: row[x] = v; break;
        case UPHIP_FMT_Y400A: row[2 * x] = v; row[2 * x + 1] = (uint8_t)(x * 7 + y * 3); break;
        case UPHIP_FMT_RGB24: {
          const int t = (int)((x / 64 + y / 97 + seed) % 23) - 11;
          const int gg = v + t < 0 ? 0 : v + t > 255 ? 255 : v + t;
          row[3 * x] = v;
          row[3 * x + 1] = (uint8_t)gg;
          row[3 * x + 2] = (uint8_t)(v > 20 ? v - 20 * ((x / 150) & 1) : v);
          break;
        }
        case UPHIP_FMT_MONOWHITE:
          if (v < 128) row[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
          break;
        default:
          if (v >= 128) row[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
      }
    }
  }
  free(g);
  return im;
}

