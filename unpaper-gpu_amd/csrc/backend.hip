// backend.hip — the UphipBackend vtable (imageprocess/backend.h:19-57 peer)
// and options defaults (lib/options.c:23-173 + cli_options.c thresholds).
#include <cmath>
#include <cstring>

#include "runtime.h"

extern "C" {

static const UphipBackend g_backend_hip = {
    "hip",
    uphip_wipe_rectangle,
    uphip_copy_rectangle,
    uphip_center_image,
    uphip_stretch_and_replace,
    uphip_resize_and_replace,
    uphip_flip_rotate_90,
    uphip_mirror,
    uphip_shift_image,
    uphip_apply_masks,
    uphip_apply_wipes,
    uphip_apply_border,
    uphip_detect_masks,
    uphip_align_mask,
    uphip_detect_border,
    uphip_blackfilter,
    uphip_blurfilter,
    uphip_noisefilter,
    uphip_grayfilter,
    uphip_detect_rotation,
    uphip_deskew,
};

const UphipBackend* uphip_backend(void) { return &g_backend_hip; }

// degreesToRadians (deskew.c:20): float d promoted to double, result float
static float deg2rad(float d) { return d * M_PI / 180.0; }

void uphip_options_init(UphipOptions* o) {
  memset(o, 0, sizeof(*o));
  o->layout = UPHIP_LAYOUT_SINGLE;
  o->input_count = 1;
  o->output_count = 1;
  o->output_pixel_format = UPHIP_FMT_NONE;
  o->sheet_size = o->page_size = o->post_page_size = UphipRectangleSize{-1, -1};
  o->stretch_size = o->post_stretch_size = UphipRectangleSize{-1, -1};
  o->pre_zoom_factor = 1.0f;
  o->post_zoom_factor = 1.0f;
  o->sheet_background = UphipPixel{255, 255, 255};
  o->mask_color = UphipPixel{255, 255, 255};
  // cli_options.c:229-230,1108-1109: WHITE * (1.0 - 0.33f), WHITE * 0.9f
  const float black_threshold = 0.33f, white_threshold = 0.9f;
  o->abs_black_threshold = (uint8_t)(0xFF * (1.0 - black_threshold));
  o->abs_white_threshold = (uint8_t)(0xFF * (white_threshold));
  o->interpolate_type = UPHIP_INTERP_CUBIC;
  o->noisefilter_intensity = 4;

  UphipBlackfilterParameters* bf = &o->blackfilter_parameters;
  bf->scan_size = UphipRectangleSize{20, 20};
  bf->scan_step = UphipDelta{5, 5};
  bf->scan_depth.horizontal = 500;
  bf->scan_depth.vertical = 500;
  bf->scan_direction = UphipDirection{true, true};
  bf->abs_threshold = (uint8_t)(UINT8_MAX * 0.95f);
  bf->intensity = 20;
  o->blurfilter_parameters = UphipBlurfilterParameters{{100, 100}, {50, 50}, 0.01f};
  o->grayfilter_parameters.scan_size = UphipRectangleSize{50, 50};
  o->grayfilter_parameters.scan_step = UphipDelta{20, 20};
  o->grayfilter_parameters.abs_threshold = (uint8_t)(UINT8_MAX * 0.5f);

  UphipDeskewParameters* dp = &o->deskew_parameters;
  dp->deskewScanRangeRad = deg2rad(5.0f);
  dp->deskewScanStepRad = deg2rad(0.1f);
  dp->deskewScanDeviationRad = deg2rad(1.0f);
  dp->deskewScanSize = 1500;
  dp->deskewScanDepth = 0.5f;
  dp->scan_edges = UphipEdges{true, false, true, false};

  UphipMaskDetectionParameters* mp = &o->mask_detection_parameters;
  mp->scan_size = UphipRectangleSize{50, 50};
  mp->scan_step = UphipDelta{5, 5};
  mp->scan_depth.horizontal = -1;
  mp->scan_depth.vertical = -1;
  mp->scan_direction = UphipDirection{true, false};
  mp->scan_threshold.horizontal = 0.1f;
  mp->scan_threshold.vertical = 0.1f;
  mp->minimum_width = 100;
  mp->minimum_height = 100;
  mp->maximum_width = -1;
  mp->maximum_height = -1;

  UphipBorderScanParameters* bs = &o->border_scan_parameters;
  bs->scan_size = UphipRectangleSize{5, 5};
  bs->scan_step = UphipDelta{5, 5};
  bs->scan_threshold.horizontal = 5;
  bs->scan_threshold.vertical = 5;
  bs->scan_direction = UphipDirection{false, true};
}

}  // extern "C"
