/* hip_frame.h — the three frame hooks the HIP vtable adapter needs from the
 * host side of unpaper-gpu.  They are the only place where `AVFrame` fields
 * are touched, so the adapter itself (backend_hip.c) compiles against the
 * reference's value-type headers alone.
 *
 * Production implementation: backend_hip_av.c (libavutil; keeps the state in
 * `frame->opaque_ref` exactly where image_cuda.c:40-107 keeps its
 * ImageCudaState).  Test implementation: tests/c/adapter_main.c (a plain
 * struct standing in for the frame, so the adapter runs without FFmpeg).
 */
#pragma once

#include <stdbool.h>
#include <stdint.h>

#include "imageprocess/image.h"
#include "unpaper_hip.h"

/* Residency of one frame, the peer of ImageCudaState (image_cuda.c:22-30):
 * `host_newer` is its cpu_dirty, `device_newer` its cuda_dirty. */
typedef struct {
  UphipImage img;    /* device copy; img.frame == NULL until first GPU use */
  bool host_newer;   /* frame bytes changed since the last upload */
  bool device_newer; /* a GPU op changed the device copy since the last download */
} HipState;

/* Host view of a frame: geometry, pixel format (already mapped from
 * AVPixelFormat, sheet_stages.c:75-92) and the bytes of plane 0. */
typedef struct {
  int32_t width, height;
  UphipPixelFormat format;
  uint8_t *data;
  int64_t linesize;
} HipFrameView;

/* The frame's state, created on first use with host_newer = true. */
HipState *hip_state(AVFrame *frame);
HipFrameView hip_frame_view(AVFrame *frame);
/* Give *pImage a new frame of d's size and format whose state owns `d`
 * (device_newer = true), then release the old frame and its state the way
 * replace_image (image.c:46-50) does. */
void hip_adopt(Image *pImage, UphipImage d);
