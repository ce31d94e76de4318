/* backend_hip.h — the HIP ImageBackend adapter for unpaper-gpu: the 20 ops
 * with the exact signatures of imageprocess/backend.h:22-56, plus the
 * residency hooks image_cuda.c provides for CUDA.  The vtable instance
 * (`backend_hip`) is in backend_hip_av.c next to the libavutil hooks, since
 * backend.h pulls in lib/options.h and with it libavutil/pixfmt.h. */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "imageprocess/blit.h"
#include "imageprocess/deskew.h"
#include "imageprocess/filters.h"
#include "imageprocess/image.h"
#include "imageprocess/interpolate.h"
#include "imageprocess/masks.h"
#include "imageprocess/primitives.h"

#include "hip_frame.h"

void wipe_rectangle_hip(Image image, Rectangle input_area, Pixel color);
void copy_rectangle_hip(Image source, Image target, Rectangle source_area, Point target_coords);
void center_image_hip(Image source, Image target, Point target_origin, RectangleSize target_size);
void stretch_and_replace_hip(Image *pImage, RectangleSize size, Interpolation interpolate_type);
void resize_and_replace_hip(Image *pImage, RectangleSize size, Interpolation interpolate_type);
void flip_rotate_90_hip(Image *pImage, RotationDirection direction);
void mirror_hip(Image image, Direction direction);
void shift_image_hip(Image *pImage, Delta d);
void apply_masks_hip(Image image, const Rectangle masks[], size_t masks_count, Pixel color);
void apply_wipes_hip(Image image, Wipes wipes, Pixel color);
void apply_border_hip(Image image, const Border border, Pixel color);
size_t detect_masks_hip(Image image, MaskDetectionParameters params, const Point points[],
                        size_t points_count, Rectangle masks[]);
void align_mask_hip(Image image, const Rectangle inside_area, const Rectangle outside,
                    MaskAlignmentParameters params);
Border detect_border_hip(Image image, BorderScanParameters params, const Rectangle outside_mask);
void blackfilter_hip(Image image, BlackfilterParameters params);
void blurfilter_hip(Image image, BlurfilterParameters params, uint8_t abs_white_threshold);
void noisefilter_hip(Image image, uint64_t intensity, uint8_t min_white_level);
void grayfilter_hip(Image image, GrayfilterParameters params);
float detect_rotation_hip(Image image, Rectangle mask, const DeskewParameters params);
void deskew_hip(Image source, Rectangle mask, float radians, Interpolation interpolate_type);

/* image_ensure_cpu / image_mark_cpu_dirty / image_mark_cuda_dirty
 * (image.h:32-38, image_cuda.c:109-305) when the HIP backend is selected. */
void backend_hip_ensure_cpu(Image *image);
void backend_hip_mark_cpu_dirty(Image *image);
void backend_hip_mark_gpu_dirty(Image *image);
/* Free the device copy a frame's state owns (from the state's free). */
void backend_hip_release(HipState *st);
/* nvimgcodec_encode_to_file's peer for the GPU output branch (JPEG). */
bool backend_hip_encode_to_file(Image *image, int quality, const char *filename);
