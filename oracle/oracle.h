/*
 * oracle.h — CPU restatement of the reference CPU path (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle for the HIP backend.  It restates, function by
 * function, the CPU semantics of ErrorTzy/unpaper-gpu's --device=cpu path
 * (imageprocess/{pixel,primitives,image,blit,fill,filters,masks,deskew,
 * interpolate}.c and src/core/sheet_stages.c).  It is NOT part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The reference itself is not buildable here (it needs FFmpeg's libavutil
 * headers, which the image lacks), so the oracle is
 * pinned against the reference's own golden images (tests/golden_images) and
 * the scenarios of its C unit tests.
 */
#ifndef UNPAPER_ORACLE_H
#define UNPAPER_ORACLE_H

#include "../include/unpaper_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Host image: AVFrame data[0]/linesize[0]/width/height/format + Image fields
 * (image.h:11-15). */
typedef struct {
  uint8_t *data;
  int64_t linesize;
  int32_t width, height;
  int32_t format; /* UphipPixelFormat */
  UphipPixel background;
  uint8_t abs_black_threshold;
} OImage;

OImage o_create_image(UphipRectangleSize size, int32_t format, bool fill,
                      UphipPixel background, uint8_t abs_black_threshold);
void o_free_image(OImage *image);
int64_t o_min_linesize(int32_t width, int32_t format);

/* pixel.c */
UphipPixel o_get_pixel(OImage image, UphipPoint p);
void o_set_pixel(OImage image, UphipPoint p, UphipPixel px);

/* the 20 backend ops (backend.c:11-48), CPU semantics */
void o_wipe_rectangle(OImage image, UphipRectangle area, UphipPixel color);
void o_copy_rectangle(OImage source, OImage target, UphipRectangle source_area,
                      UphipPoint target_coords);
void o_center_image(OImage source, OImage target, UphipPoint target_origin,
                    UphipRectangleSize target_size);
void o_stretch_and_replace(OImage *pImage, UphipRectangleSize size, int32_t interp);
void o_resize_and_replace(OImage *pImage, UphipRectangleSize size, int32_t interp);
void o_flip_rotate_90(OImage *pImage, int32_t direction);
void o_mirror(OImage image, UphipDirection direction);
void o_shift_image(OImage *pImage, UphipDelta d);
void o_apply_masks(OImage image, const UphipRectangle *masks, size_t count,
                   UphipPixel color);
void o_apply_wipes(OImage image, const UphipWipes *wipes, UphipPixel color);
void o_apply_border(OImage image, UphipBorder border, UphipPixel color);
size_t o_detect_masks(OImage image, const UphipMaskDetectionParameters *params,
                      const UphipPoint *points, size_t points_count,
                      UphipRectangle *masks);
void o_align_mask(OImage image, UphipRectangle inside_area,
                  UphipRectangle outside, UphipMaskAlignmentParameters params);
UphipBorder o_detect_border(OImage image, UphipBorderScanParameters params,
                            UphipRectangle outside_mask);
void o_blackfilter(OImage image, const UphipBlackfilterParameters *params);
void o_blurfilter(OImage image, UphipBlurfilterParameters params,
                  uint8_t abs_white_threshold);
void o_noisefilter(OImage image, uint64_t intensity, uint8_t min_white_level);
void o_grayfilter(OImage image, UphipGrayfilterParameters params);
/* the per-(edge, angle) peaks o_detect_rotation chooses from; -1 past capacity */
int o_rotation_peaks(OImage image, UphipRectangle mask, const UphipDeskewParameters *params,
                     int32_t *out, int capacity);
float o_detect_rotation(OImage image, UphipRectangle mask,
                        const UphipDeskewParameters *params);
void o_deskew(OImage source, UphipRectangle mask, float radians, int32_t interp);
void o_center_mask(OImage image, UphipPoint center, UphipRectangle area);

/* Sheet pipeline (sheet_stages.c:44-696 for a fresh batch job).  `pages` are
 * the sheet's input pages (count = options->input_count; a page with
 * data == NULL is blank).  On success *sheet_out holds the processed sheet in
 * the reference's working format (RGB24) and *out_format the output pixel
 * format the reference would save with; returns 0. */
typedef struct {
  int32_t mask_count;
  UphipRectangle masks[UPHIP_MAX_PAGES];
  float rotation[UPHIP_MAX_PAGES];
  UphipRectangle border_masks[UPHIP_MAX_PAGES];
  int32_t width, height;
  uint32_t flags;
} OReport;

int o_process_sheet(const UphipOptions *options, const OImage *pages,
                    OImage *sheet_out, int32_t *out_format, OReport *report);

/* saveImage conversion (file.c:187-259): convert a sheet to `format`
 * (Y400A→GRAY8, MONOBLACK→MONOWHITE as the reference does). */
OImage o_convert_for_save(OImage sheet, int32_t format);

/* Deterministic counters for instrumentation of the sequential parts. */
typedef struct {
  uint64_t flood_fill_calls, flood_fill_matches, flood_fill_max_depth;
  uint64_t noise_clusters;
  uint64_t blackfilter_fills;
} OStats;
void o_stats_get(OStats *out);
void o_stats_reset(void);

/* options_init defaults (lib/options.c:23-173 + cli_options.c thresholds) */
void o_options_init(UphipOptions *o);

/* jpeg_enc.c — the JPEG encode of the GPU output branch (nvimgcodec.c:
 * 1007-1212), restated as libjpeg-turbo's baseline encoder (pinned to PIL's
 * libjpeg-turbo; nvImageCodec itself is unpinned).  fmt GRAY8 -> 1 component,
 * RGB24 -> YCbCr with sampling 0 = 4:4:4, 1 = 4:2:2, 2 = 4:2:0. */
int64_t o_jpeg_encode(const uint8_t *src, int64_t linesize, int w, int h, int fmt,
                      int quality, int sampling, uint8_t *out, int64_t cap);
int64_t o_jpeg_header(int w, int h, int ncomp, int sampling, int quality, uint8_t *out,
                      int64_t cap);
void o_jpeg_quant_tables(int quality, uint16_t qtab[2][64]);
size_t oracle_abi_sizeof(const char *name);

#ifdef __cplusplus
}
#endif

#endif
