/* backend_hip_av.c — the libavutil half of the HIP adapter and the vtable
 * instance, for imageprocess/ in unpaper-gpu.
 *
 * It needs the FFmpeg development headers (lib/options.h includes
 * libavutil/pixfmt.h), which this image does not carry, so it is not
 * compiled here; tests/c/adapter_main.c implements the same three hooks over
 * a plain struct and runs backend_hip.c through them on the GPU.
 *
 * Where it plugs in:
 *   - imageprocess/backend.c:79-97 (image_backend_select): a
 *     UNPAPER_DEVICE_HIP case that returns &backend_hip;
 *   - imageprocess/image.h:32-38: image_ensure_cpu / image_mark_cpu_dirty /
 *     image_mark_cuda_dirty call the backend_hip_* hooks when that device is
 *     selected; free_image needs nothing, the state is freed with the frame's
 *     opaque_ref (the same place image_cuda.c:40-107 keeps ImageCudaState).
 */
#include <libavutil/buffer.h>
#include <libavutil/frame.h>
#include <libavutil/mem.h>
#include <libavutil/pixfmt.h>

#include "imageprocess/backend.h"
#include "lib/logging.h"

#include "backend_hip.h"

static void state_free(void *opaque, uint8_t *data) {
  (void)opaque;
  backend_hip_release((HipState *)data);
  av_free(data);
}

HipState *hip_state(AVFrame *frame) {
  if (!frame->opaque_ref) {
    HipState *st = av_mallocz(sizeof *st);
    if (!st) errOutput("HIP backend: out of memory");
    st->host_newer = true;
    frame->opaque_ref = av_buffer_create((uint8_t *)st, sizeof *st, state_free, NULL, 0);
    if (!frame->opaque_ref) errOutput("HIP backend: out of memory");
  }
  return (HipState *)frame->opaque_ref->data;
}

/* the formats sheet_stages.c:75-92 keeps native */
static UphipPixelFormat format_of(int av) {
  switch (av) {
    case AV_PIX_FMT_GRAY8: return UPHIP_FMT_GRAY8;
    case AV_PIX_FMT_Y400A: return UPHIP_FMT_Y400A;
    case AV_PIX_FMT_RGB24: return UPHIP_FMT_RGB24;
    case AV_PIX_FMT_MONOWHITE: return UPHIP_FMT_MONOWHITE;
    case AV_PIX_FMT_MONOBLACK: return UPHIP_FMT_MONOBLACK;
    default: errOutput("HIP backend: unsupported pixel format %d", av);
  }
  return UPHIP_FMT_NONE;
}

HipFrameView hip_frame_view(AVFrame *frame) {
  return (HipFrameView){frame->width, frame->height, format_of(frame->format), frame->data[0],
                        frame->linesize[0]};
}

void hip_adopt(Image *pImage, UphipImage d) {
  const UphipRectangleSize s = uphip_size_of_image(d);
  /* host buffer of the new size; its bytes stay stale until ensure_cpu */
  Image n = create_image((RectangleSize){s.width, s.height}, pImage->frame->format, false,
                         pImage->background, pImage->abs_black_threshold);
  HipState *st = hip_state(n.frame);
  st->img = d;
  st->host_newer = false;
  st->device_newer = true;
  replace_image(pImage, &n); /* frees the old frame and, with it, its state */
}

const ImageBackend backend_hip = {
    .name = "hip",
    .wipe_rectangle = wipe_rectangle_hip,
    .copy_rectangle = copy_rectangle_hip,
    .center_image = center_image_hip,
    .stretch_and_replace = stretch_and_replace_hip,
    .resize_and_replace = resize_and_replace_hip,
    .flip_rotate_90 = flip_rotate_90_hip,
    .mirror = mirror_hip,
    .shift_image = shift_image_hip,
    .apply_masks = apply_masks_hip,
    .apply_wipes = apply_wipes_hip,
    .apply_border = apply_border_hip,
    .detect_masks = detect_masks_hip,
    .align_mask = align_mask_hip,
    .detect_border = detect_border_hip,
    .blackfilter = blackfilter_hip,
    .blurfilter = blurfilter_hip,
    .noisefilter = noisefilter_hip,
    .grayfilter = grayfilter_hip,
    .detect_rotation = detect_rotation_hip,
    .deskew = deskew_hip,
};
