/* jbig2_hip.c — lib/jbig2_decode.c for unpaper-gpu without jbig2dec: the
 * reference's JBIG2 API (lib/jbig2_decode.h, as it is) on libunpaper_hip's
 * decoder (uphip_jbig2_decode; csrc/jbig2.h).  Link it instead of
 * lib/jbig2_decode.c and jbig2dec.
 * Compiles against the reference headers where they lie
 * (`cc -I<reference> -I<repo>/include -c integration/jbig2_hip.c`). */
#include <stdarg.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lib/jbig2_decode.h"
#include "unpaper_hip.h"

_Static_assert(sizeof(Jbig2DecodedImage) == sizeof(UphipJbig2Image), "Jbig2DecodedImage");

static __thread char last_error[512];

const char *jbig2_get_last_error(void) { return last_error; }

bool jbig2_is_available(void) { return true; }

bool jbig2_decode(const uint8_t *data, size_t size, const uint8_t *globals, size_t globals_size,
                  Jbig2DecodedImage *out) {
  if (!data || !size || !out) {
    snprintf(last_error, sizeof(last_error), "Invalid arguments");
    return false;
  }
  UphipJbig2Image u;
  if (uphip_jbig2_decode(data, size, globals, globals_size, &u) != 0) {
    const char *e = uphip_last_error();
    snprintf(last_error, sizeof(last_error), "%s", e ? e : "JBIG2 decode failed");
    uphip_clear_error();
    return false;
  }
  out->data = u.data;  /* malloc'd: jbig2_free_image frees it */
  out->width = u.width;
  out->height = u.height;
  out->stride = u.stride;
  return true;
}

void jbig2_free_image(Jbig2DecodedImage *image) {
  if (!image) return;
  free(image->data);
  memset(image, 0, sizeof(*image));
}

/* lib/jbig2_decode.c:136-170: 1 (black) -> 0, 0 -> 255; invert swaps them */
bool jbig2_expand_to_gray8(const Jbig2DecodedImage *jbig2, uint8_t *gray_out, size_t gray_stride, bool invert) {
  if (!jbig2 || !jbig2->data || !gray_out || gray_stride < jbig2->width) {
    snprintf(last_error, sizeof(last_error), "Invalid arguments");
    return false;
  }
  const uint8_t white = invert ? 0 : 255, black = invert ? 255 : 0;
  for (uint32_t y = 0; y < jbig2->height; y++) {
    const uint8_t *s = jbig2->data + (size_t)y * jbig2->stride;
    uint8_t *d = gray_out + (size_t)y * gray_stride;
    for (uint32_t x = 0; x < jbig2->width; x++) d[x] = (s[x >> 3] >> (7 - (x & 7)) & 1) ? black : white;
  }
  return true;
}
