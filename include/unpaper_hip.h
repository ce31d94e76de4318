/*
 * unpaper_hip.h — C ABI of the MI355X-native (gfx950) page-cleanup backend.
 *
 * This header is the drop-in boundary: it is what a `backend_hip.c` inside the
 * reference tree binds.  Every declaration cites the
 * reference interface it replaces (paths relative to ErrorTzy/unpaper-gpu).
 *
 *  - value types           <- imageprocess/primitives.h:13-108, masks.h:14-101,
 *                             filters.h:12-70, deskew.h:13-20, interpolate.h:10-15
 *  - UphipImage            <- imageprocess/image.h:11-15 (Image{AVFrame*,...});
 *                             the device copy that the reference hangs off
 *                             AVFrame.opaque_ref (backend_cuda_internal.h:18-27)
 *                             is the UphipFrame itself here.
 *  - UphipBackend / ops    <- imageprocess/backend.h:19-57 (ImageBackend vtable)
 *  - uphip_try_init        <- imageprocess/cuda_runtime.h (unpaper_cuda_try_init)
 *  - stream pool / TLS     <- imageprocess/cuda_stream_pool.h, cuda_runtime.c:70
 *  - UphipOptions          <- lib/options.h:32-127 (Options) + SheetProcessConfig
 *                             (sheet_process.h:22-37)
 *  - uphip_batch_*         <- sheet_process.c:134 process_sheet driven by
 *                             lib/batch_worker.c:79 batch_process_job
 *
 * No torch or HIP types appear in any signature: plain pointers, sizes, PODs.
 * All structs are layout-identical to their reference counterparts (checked by
 * static asserts in INTEGRATION.md's adapter) so the adapter can cast.
 */
#ifndef UNPAPER_HIP_H
#define UNPAPER_HIP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UPHIP_ABI_VERSION 1

/* constants.h:8-12 */
#define UPHIP_MAX_MASKS 100
#define UPHIP_MAX_POINTS 100
#define UPHIP_MAX_PAGES 2

/* ---------------------------------------------------------------------------
 * Value types — imageprocess/primitives.h:13-108
 * ------------------------------------------------------------------------- */
typedef struct { int32_t x, y; } UphipPoint;                  /* primitives.h:13-16 */
typedef struct { int32_t horizontal, vertical; } UphipDelta;  /* primitives.h:23-26 */
typedef struct { bool horizontal, vertical; } UphipDirection; /* primitives.h:40-43 */
typedef struct { bool left, top, right, bottom; } UphipEdges; /* primitives.h:54-59 */
typedef struct { uint8_t r, g, b; } UphipPixel;               /* primitives.h:61-65 */
typedef struct { UphipPoint vertex[2]; } UphipRectangle;      /* primitives.h:72-74, inclusive */
typedef struct { int32_t width, height; } UphipRectangleSize; /* primitives.h:76-79 */

/* masks.h:84-89 */
typedef struct { int32_t left, top, right, bottom; } UphipBorder;

/* masks.h:65-70 (MAX_WIPES == MAX_MASKS) */
typedef struct {
  size_t count;
  UphipRectangle areas[UPHIP_MAX_MASKS];
} UphipWipes;

/* interpolate.h:10-15 */
typedef enum {
  UPHIP_INTERP_NN = 0,
  UPHIP_INTERP_LINEAR = 1,
  UPHIP_INTERP_CUBIC = 2,
} UphipInterpolation;

/* blit.h:25-27 */
typedef int8_t UphipRotationDirection;
#define UPHIP_ROTATE_CLOCKWISE ((UphipRotationDirection)1)
#define UPHIP_ROTATE_ANTICLOCKWISE ((UphipRotationDirection)-1)

/* constants.h:18-23 */
typedef enum {
  UPHIP_LAYOUT_NONE = 0,
  UPHIP_LAYOUT_SINGLE = 1,
  UPHIP_LAYOUT_DOUBLE = 2,
} UphipLayout;

/* Pixel formats the reference accepts natively (sheet_stages.c:75-92,
 * cuda_kernels_format.h:27-34). Values are ours, not FFmpeg's. */
typedef enum {
  UPHIP_FMT_NONE = -1,
  UPHIP_FMT_GRAY8 = 0,
  UPHIP_FMT_Y400A = 1,
  UPHIP_FMT_RGB24 = 2,
  UPHIP_FMT_MONOWHITE = 3,
  UPHIP_FMT_MONOBLACK = 4,
} UphipPixelFormat;

/* filters.h:12-31 — exclusions are an inline array here (the reference keeps a
 * caller-owned Rectangle* next to a count). */
typedef struct {
  UphipRectangleSize scan_size;
  UphipDelta scan_step;
  struct { uint32_t horizontal, vertical; } scan_depth;
  UphipDirection scan_direction;
  uint8_t abs_threshold;
  int32_t intensity;
  size_t exclusions_count;
  UphipRectangle exclusions[UPHIP_MAX_MASKS];
} UphipBlackfilterParameters;

/* filters.h:43-49 */
typedef struct {
  UphipRectangleSize scan_size;
  UphipDelta scan_step;
  float intensity;
} UphipBlurfilterParameters;

/* filters.h:59-65 */
typedef struct {
  UphipRectangleSize scan_size;
  UphipDelta scan_step;
  uint8_t abs_threshold;
} UphipGrayfilterParameters;

/* masks.h:14-37 */
typedef struct {
  UphipRectangleSize scan_size;
  UphipDelta scan_step;
  struct { int32_t horizontal, vertical; } scan_depth;
  UphipDirection scan_direction;
  struct { float horizontal, vertical; } scan_threshold;
  int32_t minimum_width;
  int32_t maximum_width;
  int32_t minimum_height;
  int32_t maximum_height;
} UphipMaskDetectionParameters;

/* masks.h:53-56 */
typedef struct {
  UphipEdges alignment;
  UphipDelta margin;
} UphipMaskAlignmentParameters;

/* masks.h:90-100 */
typedef struct {
  UphipRectangleSize scan_size;
  UphipDelta scan_step;
  struct { int32_t horizontal, vertical; } scan_threshold;
  UphipDirection scan_direction;
} UphipBorderScanParameters;

/* deskew.h:13-20 (radians) */
typedef struct {
  float deskewScanRangeRad;
  float deskewScanStepRad;
  float deskewScanDeviationRad;
  int deskewScanSize;
  float deskewScanDepth;
  UphipEdges scan_edges;
} UphipDeskewParameters;

/* ---------------------------------------------------------------------------
 * Device frames and images — imageprocess/image.h:11-38
 * ------------------------------------------------------------------------- */
typedef struct UphipFrame UphipFrame; /* device-resident AVFrame peer */

typedef struct {
  UphipFrame *frame;
  UphipPixel background;
  uint8_t abs_black_threshold;
} UphipImage;

/* create_image (image.c:19-44): allocate on the current device; rows are
 * pitched for coalesced access; `fill` wipes with `background`. */
UphipImage uphip_create_image(UphipRectangleSize size, UphipPixelFormat format,
                              bool fill, UphipPixel background,
                              uint8_t abs_black_threshold);
/* free_image (image.c:51-54) */
void uphip_free_image(UphipImage *image);
/* replace_image (image.c:46-50) */
void uphip_replace_image(UphipImage *image, UphipImage *new_image);
/* create_compatible_image (image.c:56-59) */
UphipImage uphip_create_compatible_image(UphipImage source,
                                         UphipRectangleSize size, bool fill);
/* size_of_image (image.c:61-66) */
UphipRectangleSize uphip_size_of_image(UphipImage image);
UphipPixelFormat uphip_image_format(UphipImage image);
/* image_ensure_cuda / image_ensure_cpu (image.h:32-38, image_cuda.c:135-269):
 * explicit H2D / D2H of the frame contents.  `linesize` is the host row stride
 * in bytes (>= bytes per row of `format`).  Synchronous w.r.t. the host. */
int uphip_image_upload(UphipImage image, const void *host, int64_t linesize);
int uphip_image_download(UphipImage image, void *host, int64_t linesize);
/* Device pointer + pitch of a frame (image_get_gpu_ptr / _pitch, image.h:52-58). */
void *uphip_image_device_ptr(UphipImage image);
int64_t uphip_image_device_pitch(UphipImage image);

/* ---------------------------------------------------------------------------
 * ImageBackend ops — imageprocess/backend.h:22-56, same argument meaning.
 * ------------------------------------------------------------------------- */
void uphip_wipe_rectangle(UphipImage image, UphipRectangle input_area,
                          UphipPixel color);
void uphip_copy_rectangle(UphipImage source, UphipImage target,
                          UphipRectangle source_area, UphipPoint target_coords);
void uphip_center_image(UphipImage source, UphipImage target,
                        UphipPoint target_origin, UphipRectangleSize target_size);
void uphip_stretch_and_replace(UphipImage *pImage, UphipRectangleSize size,
                               UphipInterpolation interpolate_type);
void uphip_resize_and_replace(UphipImage *pImage, UphipRectangleSize size,
                              UphipInterpolation interpolate_type);
void uphip_flip_rotate_90(UphipImage *pImage, UphipRotationDirection direction);
void uphip_mirror(UphipImage image, UphipDirection direction);
void uphip_shift_image(UphipImage *pImage, UphipDelta d);
void uphip_apply_masks(UphipImage image, const UphipRectangle masks[],
                       size_t masks_count, UphipPixel color);
void uphip_apply_wipes(UphipImage image, UphipWipes wipes, UphipPixel color);
void uphip_apply_border(UphipImage image, const UphipBorder border,
                        UphipPixel color);
size_t uphip_detect_masks(UphipImage image, UphipMaskDetectionParameters params,
                          const UphipPoint points[], size_t points_count,
                          UphipRectangle masks[]);
void uphip_align_mask(UphipImage image, const UphipRectangle inside_area,
                      const UphipRectangle outside,
                      UphipMaskAlignmentParameters params);
UphipBorder uphip_detect_border(UphipImage image, UphipBorderScanParameters params,
                                const UphipRectangle outside_mask);
void uphip_blackfilter(UphipImage image, UphipBlackfilterParameters params);
void uphip_blurfilter(UphipImage image, UphipBlurfilterParameters params,
                      uint8_t abs_white_threshold);
void uphip_noisefilter(UphipImage image, uint64_t intensity,
                       uint8_t min_white_level);
void uphip_grayfilter(UphipImage image, UphipGrayfilterParameters params);
float uphip_detect_rotation(UphipImage image, UphipRectangle mask,
                            const UphipDeskewParameters params);
/* The peaks uphip_detect_rotation chooses from: detect_edge_rotation_peak
 * (deskew.c:48-146) of every enabled edge (left, top, right, bottom, in that
 * order) x every angle of detect_edge_rotation's loop (deskew.c:153-174, 0,
 * -step, +step, ...) into peaks[edge * nangles + angle].  Returns the count
 * written, or -1 (error, or more than `capacity`).  Not a backend entry. */
int32_t uphip_detect_rotation_peaks(UphipImage image, UphipRectangle mask,
                                    const UphipDeskewParameters params, int32_t *peaks,
                                    int32_t capacity);
void uphip_deskew(UphipImage source, UphipRectangle mask, float radians,
                  UphipInterpolation interpolate_type);

/* The vtable itself, field-for-field ImageBackend (backend.h:19-57). */
typedef struct {
  const char *name;
  void (*wipe_rectangle)(UphipImage, UphipRectangle, UphipPixel);
  void (*copy_rectangle)(UphipImage, UphipImage, UphipRectangle, UphipPoint);
  void (*center_image)(UphipImage, UphipImage, UphipPoint, UphipRectangleSize);
  void (*stretch_and_replace)(UphipImage *, UphipRectangleSize, UphipInterpolation);
  void (*resize_and_replace)(UphipImage *, UphipRectangleSize, UphipInterpolation);
  void (*flip_rotate_90)(UphipImage *, UphipRotationDirection);
  void (*mirror)(UphipImage, UphipDirection);
  void (*shift_image)(UphipImage *, UphipDelta);
  void (*apply_masks)(UphipImage, const UphipRectangle[], size_t, UphipPixel);
  void (*apply_wipes)(UphipImage, UphipWipes, UphipPixel);
  void (*apply_border)(UphipImage, const UphipBorder, UphipPixel);
  size_t (*detect_masks)(UphipImage, UphipMaskDetectionParameters,
                         const UphipPoint[], size_t, UphipRectangle[]);
  void (*align_mask)(UphipImage, const UphipRectangle, const UphipRectangle,
                     UphipMaskAlignmentParameters);
  UphipBorder (*detect_border)(UphipImage, UphipBorderScanParameters,
                               const UphipRectangle);
  void (*blackfilter)(UphipImage, UphipBlackfilterParameters);
  void (*blurfilter)(UphipImage, UphipBlurfilterParameters, uint8_t);
  void (*noisefilter)(UphipImage, uint64_t, uint8_t);
  void (*grayfilter)(UphipImage, UphipGrayfilterParameters);
  float (*detect_rotation)(UphipImage, UphipRectangle, const UphipDeskewParameters);
  void (*deskew)(UphipImage, UphipRectangle, float, UphipInterpolation);
} UphipBackend;

/* image_backend_get() for UNPAPER_DEVICE_HIP (backend.c:135-157). */
const UphipBackend *uphip_backend(void);

/* ---------------------------------------------------------------------------
 * Runtime — cuda_runtime.h / cuda_stream_pool.h peers.  One process may drive
 * several GPUs: the current device and current stream are thread-local
 * (cuda_runtime.c:70 keeps only a TLS stream; we add the device).
 * ------------------------------------------------------------------------- */
typedef enum {
  UPHIP_INIT_OK = 0,
  UPHIP_INIT_NO_RUNTIME = 1,
  UPHIP_INIT_NO_DEVICE = 2,
  UPHIP_INIT_ERROR = 3,
} UphipInitStatus;

UphipInitStatus uphip_try_init(void);
const char *uphip_init_status_string(UphipInitStatus st);
int uphip_device_count(void);
int uphip_set_device(int device);     /* TLS current device */
int uphip_get_device(void);
/* Per-device stream pool (cuda_stream_pool_global_acquire/release). */
void *uphip_stream_acquire(void);
void uphip_stream_release(void *stream);
void uphip_set_current_stream(void *stream); /* TLS; NULL = per-thread default */
/* Before destroying a stream of your own that was current for ops: waits for
 * it and frees the op scratch the library keeps per stream. */
void uphip_stream_forget(void *stream);
void *uphip_get_current_stream(void);
int uphip_synchronize(void);           /* current stream */
/* Error reporting.  The reference's errOutput() exits (lib/logging.h); here a
 * failing op records the message and returns, and the caller checks.  Set
 * `fatal` to restore exit-on-error. */
const char *uphip_last_error(void);    /* NULL when no error since clear */
void uphip_clear_error(void);
void uphip_set_fatal_errors(bool fatal);
const char *uphip_version(void);
/* Layout introspection for the drop-in check: sizeof of a UphipXxx type and
 * offsetof of one of its fields ("scan_depth.horizontal", "vertex[1].x"),
 * (size_t)-1 if unknown; compared with the reference headers' layout in
 * tests/test_abi.py (tests/golden/abi_layout.json). */
size_t uphip_abi_sizeof(const char *type);
size_t uphip_abi_offsetof(const char *type, const char *field);

/* ---------------------------------------------------------------------------
 * Per-sheet options — lib/options.h:32-127 (processing subset) plus the
 * SheetProcessConfig fields (sheet_process.h:22-37).  Per-sheet "--no-xxx"
 * multi-indexes are resolved by the caller into `disable` bits for the sheet.
 * ------------------------------------------------------------------------- */
enum {
  UPHIP_NO_BLACKFILTER = 1u << 0,
  UPHIP_NO_NOISEFILTER = 1u << 1,
  UPHIP_NO_BLURFILTER = 1u << 2,
  UPHIP_NO_GRAYFILTER = 1u << 3,
  UPHIP_NO_MASK_SCAN = 1u << 4,
  UPHIP_NO_MASK_CENTER = 1u << 5,
  UPHIP_NO_DESKEW = 1u << 6,
  UPHIP_NO_WIPE = 1u << 7,
  UPHIP_NO_BORDER = 1u << 8,
  UPHIP_NO_BORDER_SCAN = 1u << 9,
  UPHIP_NO_BORDER_ALIGN = 1u << 10,
};

typedef struct {
  int32_t layout;               /* UphipLayout */
  int32_t input_count;          /* --input-pages (1..2) */
  int32_t output_count;         /* --output-pages (1..2) */
  int32_t output_pixel_format;  /* UPHIP_FMT_NONE = same as first input */
  uint32_t disable;             /* UPHIP_NO_* bits for this sheet */

  int16_t pre_rotate, post_rotate; /* 0, 90, -90 */
  UphipDirection pre_mirror, post_mirror;
  UphipDelta pre_shift, post_shift;
  UphipRectangleSize sheet_size, page_size, post_page_size;
  UphipRectangleSize stretch_size, post_stretch_size;
  float pre_zoom_factor, post_zoom_factor;

  UphipPixel sheet_background;
  UphipPixel mask_color;
  uint8_t abs_black_threshold;
  uint8_t abs_white_threshold;

  UphipBorder pre_border, border, post_border;
  UphipWipes pre_wipes, wipes, post_wipes;

  UphipDeskewParameters deskew_parameters;
  UphipMaskDetectionParameters mask_detection_parameters;
  UphipMaskAlignmentParameters mask_alignment_parameters;
  UphipBorderScanParameters border_scan_parameters;
  int32_t interpolate_type;     /* UphipInterpolation */
  UphipGrayfilterParameters grayfilter_parameters;
  UphipBlackfilterParameters blackfilter_parameters; /* exclusions = config */
  UphipBlurfilterParameters blurfilter_parameters;
  uint64_t noisefilter_intensity;

  /* SheetProcessConfig */
  size_t pre_mask_count;
  UphipRectangle pre_masks[UPHIP_MAX_MASKS];
  size_t point_count;           /* initial points (0 = layout default) */
  UphipPoint points[UPHIP_MAX_POINTS];
  int32_t middle_wipe[2];
} UphipOptions;

/* options_init + options_init_filter_defaults (lib/options.c:23-173) with the
 * CLI's derived thresholds (cli_options.c:229-269,1108-1109). */
void uphip_options_init(UphipOptions *o);

/* ---------------------------------------------------------------------------
 * Device batch pipeline — the MI355X-native peer of lib/batch_worker.c's
 * per-job loop over process_sheet (sheet_process.c:134).  A batch holds up to
 * `capacity` sheets of identical input geometry resident in HBM; one run pushes
 * every sheet through the full stage table of src/core/sheet_stages.c:660-672
 * with one kernel launch per stage per batch, no host synchronisation between
 * stages.  Results are bit-identical to process_sheet on the CPU backend.
 * ------------------------------------------------------------------------- */
typedef struct UphipBatch UphipBatch;

typedef struct {
  int32_t capacity;        /* sheets per batch */
  int32_t page_width;      /* input page geometry (all pages) */
  int32_t page_height;
  int32_t page_format;     /* UphipPixelFormat of the inputs */
} UphipBatchGeometry;

UphipBatch *uphip_batch_create(const UphipOptions *options,
                               const UphipBatchGeometry *geometry);
void uphip_batch_destroy(UphipBatch *batch);
/* Output geometry every sheet of this batch will have. */
int uphip_batch_output_info(UphipBatch *batch, int32_t *width, int32_t *height,
                            int32_t *format, int64_t *bytes_per_sheet);
/* Device pointer of input slot `i` (page j of the sheet: i*input_count + j),
 * pitch in bytes.  Caller may write input pages there directly (device-side
 * decode / pre-staged inputs). */
void *uphip_batch_input_ptr(UphipBatch *batch, int32_t slot, int64_t *pitch);
/* Host → device copy of one page (async on the batch stream: `host` must
 * stay valid until the stream has passed the copy, i.e. until
 * uphip_batch_wait or uphip_batch_query() == 1). */
int uphip_batch_set_input(UphipBatch *batch, int32_t slot, const void *host,
                          int64_t linesize);
/* Run the pipeline on sheets [0, count) whose pages sit in the batch's input
 * slots.  Asynchronous: returns after enqueueing; uphip_batch_wait() joins
 * and reports device-side failures. */
int uphip_batch_run(UphipBatch *batch, int32_t count);
/* Same, reading the pages in place from device memory: page j of sheet s is
 * at pages + (s*input_count + j)*page_stride, rows `pitch` bytes apart
 * (pre-staged / device-decoded inputs, no copy).  When pages, pitch and
 * page_stride are 16-byte aligned the GRAY8 decode reads rows as 16-byte
 * vectors: the buffer must then extend to round_up(row bytes, 16) past the
 * last page's last row start. */
int uphip_batch_run_device(UphipBatch *batch, int32_t count, const void *pages,
                           int64_t pitch, int64_t page_stride);
int uphip_batch_wait(UphipBatch *batch);
/* Device → host copy of output sheet `i` (output page j for output_count 2 is
 * returned side by side, exactly as the sheet). */
int uphip_batch_get_output(UphipBatch *batch, int32_t sheet, void *host,
                           int64_t linesize);
void *uphip_batch_output_ptr(UphipBatch *batch, int32_t sheet, int64_t *pitch);
/* Per-sheet results for inspection / tests: masks, rotation, borders. */
typedef struct {
  int32_t mask_count;
  UphipRectangle masks[UPHIP_MAX_PAGES];
  float rotation[UPHIP_MAX_PAGES];
  UphipRectangle border_masks[UPHIP_MAX_PAGES];
  int32_t width, height;
  uint32_t flags;
} UphipSheetReport;
int uphip_batch_get_report(UphipBatch *batch, int32_t sheet,
                           UphipSheetReport *report);
/* Asynchronous staging for host-fed pipelines (the pinned, double-buffered
 * staging of src/pipeline/image_pipeline.c:226-376; uphip_runner_* drives
 * these).  All work is queued on the batch stream; with pinned host buffers
 * the copies run on the DMA engines and overlap other batches' kernels.
 *   upload_async:   pages i = 0 .. count*input_count-1 from host + i*page_stride
 *                   (rows `linesize` apart) into the input slots.
 *   download_async: every sheet s of the last run into host + s*sheet_stride;
 *                   only after the run has finished (uphip_batch_query() == 1).
 *   query:          1 = all queued work done, 0 = running, -1 = error.
 *   stream:         the batch's hipStream_t (for events). */
int uphip_batch_upload_async(UphipBatch *batch, int32_t count, const void *host,
                             int64_t linesize, int64_t page_stride);
int uphip_batch_download_async(UphipBatch *batch, void *host, int64_t linesize,
                               int64_t sheet_stride);
int uphip_batch_query(UphipBatch *batch);
void *uphip_batch_stream(UphipBatch *batch);
/* The GPU JPEG output branch for a whole batch (encode_queue_submit_gpu,
 * lib/encode_queue.c:860-990, per sheet in the reference): queued on the
 * batch stream after uphip_batch_run*, it encodes every output page of the
 * last run (count * output_count pages; page j of a sheet is its j-th
 * output_count-th, side by side as the PNM sinks split it) from the finished
 * working sheet -- GRAY8 sheets as one component, RGB24 ones as YCbCr --
 * and packs the files one after another in device memory, then copies their
 * sizes to the host.  After the stream is idle (uphip_batch_query() == 1):
 *   jpeg_sizes:           sizes[i] of page i (-1: larger than the batch's
 *                         encode buffers, re-encode it with uphip_jpeg_encode
 *                         from uphip_batch_jpeg_page); returns the packed total
 *   jpeg_download_async:  the packed files into host memory (total bytes)
 *   jpeg_page:            device pointer / pitch / size of output page i. */
int uphip_batch_encode_jpeg_async(UphipBatch *batch, int32_t quality, int32_t sampling);
int64_t uphip_batch_jpeg_sizes(UphipBatch *batch, int64_t *sizes, int32_t max_pages);
int uphip_batch_jpeg_download_async(UphipBatch *batch, void *host, int64_t capacity);
int uphip_batch_jpeg_page(UphipBatch *batch, int32_t page, const void **device_src,
                          int64_t *pitch, int32_t *width, int32_t *height, int32_t *format);
/* Row pitch of the output sheets on the device: host staging with this
 * linesize (and pitch * height per sheet) downloads as linear DMA copies. */
int uphip_batch_output_pitch(UphipBatch *batch, int64_t *pitch);
/* Device memory the batch holds (planes, inputs, scratch, tables). */
int uphip_batch_device_bytes(UphipBatch *batch, int64_t *bytes);

/* ---------------------------------------------------------------------------
 * Host codec — the PNM half of loadImage/saveImage (file.c:29-259).
 * P4/P1 -> MONOWHITE, P5/P2 -> GRAY8, P6/P3 -> RGB24 (8-bit samples); writing
 * GRAY8 -> P5, RGB24 -> P6, MONOWHITE -> P4 (saveImageDirect, file.c:133-176).
 * ------------------------------------------------------------------------- */
typedef struct {
  int32_t width, height, format;
} UphipPnmInfo;
int uphip_pnm_probe(const char *path, UphipPnmInfo *info);
/* Decode into `dst` (rows `linesize` apart); fails when `expect` is given and
 * the file's geometry differs. */
int uphip_pnm_read(const char *path, void *dst, int64_t linesize,
                   const UphipPnmInfo *expect);
int uphip_pnm_write(const char *path, const void *src, int64_t linesize,
                    int32_t width, int32_t height, int32_t format);
/* PNG half of loadImage (file.c:29-131; the reference's test sources are
 * PNG), formats as FFmpeg's PNG decoder reports them: 1-bit gray ->
 * MONOBLACK, 2/4/8-bit gray -> GRAY8, gray+alpha (or 8-bit gray + tRNS) ->
 * Y400A, RGB -> RGB24, palette -> RGB24 (the PAL8 case, file.c:110-120);
 * 16-bit samples and RGBA fail like loadImage's "unsupported pixel format".
 * Adam7 interlacing supported.  Output stays PNM (saveImage, file.c:260-300). */
int uphip_png_probe(const char *path, UphipPnmInfo *info);
int uphip_png_read(const char *path, void *dst, int64_t linesize,
                   const UphipPnmInfo *expect);
/* JPEG decode peer of nvimgcodec_decode / _decode_file
 * (imageprocess/nvimgcodec.c:679-1007) and of loadImage's FFmpeg JPEG path
 * (file.c:29-128): baseline / extended-sequential Huffman, 8-bit; 1 component
 * -> GRAY8, 3 components (YCbCr, or RGB per the Adobe marker) -> RGB24 (the
 * batch decode queue's swscale conversion, sheet_stages.c:99-122); sampling
 * factors 1 or 2.  Huffman decoding on the host; dequantisation, IDCT, chroma
 * upsampling and colour conversion on the current device (libjpeg's islow
 * IDCT, fancy upsampling and ycc_rgb_convert).  Progressive, arithmetic,
 * 12-bit and CMYK files fail.  uphip_jpeg_read returns pixels in host memory;
 * uphip_jpeg_decode decodes a file image in memory into device memory (rows
 * `pitch` apart; info: in = expected geometry when width > 0, out = geometry).
 * Both synchronise the current stream. */
int uphip_jpeg_probe(const char *path, UphipPnmInfo *info);
int uphip_jpeg_read(const char *path, void *dst, int64_t linesize,
                    const UphipPnmInfo *expect);
int uphip_jpeg_decode(const void *data, size_t size, void *device_dst, int64_t pitch,
                      UphipPnmInfo *info);
/* The host half alone (no device needed): the packed coefficient image of
 * csrc/jpeg.h (header, per-block counts, per-MCU-row offsets, zigzag
 * coefficient prefixes) written to `packed` when `capacity` suffices.
 * Returns its size in bytes, or -1. */
int64_t uphip_jpeg_entropy_decode(const void *data, size_t size, void *packed,
                                  int64_t capacity);
/* JPEG encode peer of nvimgcodec_encode / nvimgcodec_encode_jpeg
 * (imageprocess/nvimgcodec.c:1007-1148), the GPU output branch of
 * sheet_stage_output (src/core/sheet_stages.c:554-581): a device image
 * (GRAY8 -> one component, RGB24 -> YCbCr with `sampling`; rows `pitch`
 * bytes apart) encoded on the current device/stream as a baseline JPEG file
 * with the Annex K tables scaled by `quality` (1..100, 0 = 85, the
 * reference's default: lib/options.h:42, nvimgcodec.c:451).  The bytes equal
 * libjpeg-turbo's for the same quality and sampling (PIL's encoder;
 * nvImageCodec's own output is unpinned).  Returns the file size; the bytes
 * are copied to `out` (host memory) only when `capacity` suffices (out =
 * NULL sizes a buffer).  Synchronous; -1 on error. */
#define UPHIP_JPEG_DEFAULT_QUALITY 85
typedef enum {
  UPHIP_JPEG_444 = 0, /* nvImageCodec's default (no chroma subsampling) */
  UPHIP_JPEG_422 = 1,
  UPHIP_JPEG_420 = 2, /* libjpeg's default */
} UphipJpegSampling;
int64_t uphip_jpeg_encode(const void *device_src, int64_t pitch, int32_t width,
                          int32_t height, int32_t format, int32_t quality,
                          int32_t sampling, void *out, int64_t capacity);
/* JPEG 2000 peer of the JP2 half of nvImageCodec (imageprocess/nvimgcodec.c
 * NVIMGCODEC_FORMAT_JPEG2000 decode, lib/decode_queue.c:53-71 is_jp2_file
 * routing .jp2/.j2k/.j2c to it; nvimgcodec_encode_jp2 with
 * nvimgcodec_default_jp2_lossless_params, lib/encode_queue.c:883-962).
 * Decode: JP2 files or raw codestreams, 8-bit unsigned, 1 or 3 components
 * (-> GRAY8 / RGB24), no subsampling, code-block style 0, any tiling,
 * precincts, progression order, layers, 5/3 or 9/7 (csrc/j2k.h).  Packet
 * headers are read on the host; the EBCOT code-block decoder (a lane per
 * block), the inverse wavelet and component transforms, the DC shift and
 * the store run on the current device.  Pixels equal OpenJPEG's (PIL's decoder) for reversible
 * and irreversible files.  uphip_jp2_read returns host pixels,
 * uphip_jp2_decode writes device memory (rows `pitch` apart; info: in =
 * expected geometry when width > 0, out = geometry).  Both synchronise. */
int uphip_jp2_probe(const char *path, UphipPnmInfo *info);
int uphip_jp2_read(const char *path, void *dst, int64_t linesize,
                   const UphipPnmInfo *expect);
int uphip_jp2_decode(const void *data, size_t size, void *device_dst, int64_t pitch,
                     UphipPnmInfo *info);
/* A host decode of the coefficient planes (no device needed; the
 * code-blocks through the host reference coder, csrc/j2k_t1.h): written to
 * `coef` (csrc/j2k.h layout; int32 for 5/3 files, float for 9/7) when
 * `capacity` suffices; info = geometry.  Returns their size in bytes, or
 * -1.  Test and tooling entry; the decode paths above do not use it. */
int64_t uphip_jp2_entropy_decode(const void *data, size_t size, void *coef, int64_t capacity,
                                 UphipPnmInfo *info);
/* Lossless JP2 encode of a device image (GRAY8 or RGB24, rows `pitch`
 * apart): forward RCT, 5/3 wavelet and the code-blocks on the current
 * device, packets on the host; one tile, one layer, LRCP, 64x64
 * code-blocks, up to 5 decomposition levels.  Returns the file size; the bytes are copied to
 * `out` only when `capacity` suffices (out = NULL sizes a buffer).
 * Synchronous; -1 on error. */
int64_t uphip_jp2_encode(const void *device_src, int64_t pitch, int32_t width,
                         int32_t height, int32_t format, void *out, int64_t capacity);
/* Any codec, picked by the file's signature (PNG, JPEG, JPEG 2000 or PNM). */
int uphip_image_probe(const char *path, UphipPnmInfo *info);
int uphip_image_read(const char *path, void *dst, int64_t linesize,
                     const UphipPnmInfo *expect);

/* ---------------------------------------------------------------------------
 * PDF container (csrc/pdf.h) — the reference's pdf/pdf_reader.h and
 * pdf/pdf_writer.h without MuPDF: a reader of scanned documents (one image
 * per page: classic and stream cross-reference sections, object streams,
 * incremental updates, a file scan when the xref is damaged) and an
 * image-per-page writer; JBIG2 and CCITT fax pages decode on the host.  Not
 * provided: rendering of vector / text pages (pdf_render_page*) and
 * decryption (pdf_doc_authenticate) -- pages that need them fail with an
 * error naming the cause.
 * Functions returning int give 0 on success, -1 on error (uphip_last_error).
 * ------------------------------------------------------------------------- */
typedef struct UphipPdfDocument UphipPdfDocument;
typedef struct UphipPdfWriter UphipPdfWriter;
/* pdf_reader.h:19-28 */
typedef enum {
  UPHIP_PDF_IMAGE_UNKNOWN = 0,
  UPHIP_PDF_IMAGE_JPEG = 1,
  UPHIP_PDF_IMAGE_JP2 = 2,
  UPHIP_PDF_IMAGE_JBIG2 = 3,
  UPHIP_PDF_IMAGE_CCITT = 4,
  UPHIP_PDF_IMAGE_PNG = 5,
  UPHIP_PDF_IMAGE_RAW = 6,
  UPHIP_PDF_IMAGE_FLATE = 7,
} UphipPdfImageFormat;
/* pdf_reader.h:31-44: the bytes as stored (a trailing DCT / JPX / JBIG2 /
 * CCITT / Flate filter not applied, filters before it applied) */
typedef struct {
  uint8_t *data;
  size_t size;
  int32_t width, height;
  int32_t components, bits_per_component;
  int32_t format;   /* UphipPdfImageFormat */
  int32_t is_mask;
  uint8_t *jbig2_globals;
  size_t jbig2_globals_size;
} UphipPdfImage;
/* pdf_reader.h:47-56: UTF-8 strings, NULL when absent */
typedef struct {
  char *title, *author, *subject, *keywords, *creator, *producer;
  char *creation_date, *modification_date;
} UphipPdfMetadata;
/* pdf_reader.h:59-63 */
typedef struct {
  float width, height;  /* points, the page bounds after /Rotate */
  int32_t rotation;     /* the page's /Rotate */
} UphipPdfPageInfo;
/* pdf_reader.c:72-214 (pdf_open, pdf_open_memory: the buffer must outlive
 * the document, pdf_close) */
UphipPdfDocument *uphip_pdf_open(const char *path);
UphipPdfDocument *uphip_pdf_open_memory(const uint8_t *data, size_t size);
void uphip_pdf_close(UphipPdfDocument *doc);
int uphip_pdf_page_count(UphipPdfDocument *doc);      /* -1 on error */
int uphip_pdf_needs_password(UphipPdfDocument *doc);  /* 1 = encrypted */
int uphip_pdf_get_page_info(UphipPdfDocument *doc, int page, UphipPdfPageInfo *info);
/* pdf_reader.c:290-433: the page's largest image XObject; free with
 * uphip_pdf_free_image */
int uphip_pdf_extract_page_image(UphipPdfDocument *doc, int page, UphipPdfImage *image);
void uphip_pdf_free_image(UphipPdfImage *image);
int uphip_pdf_get_metadata(UphipPdfDocument *doc, UphipPdfMetadata *meta);
void uphip_pdf_free_metadata(UphipPdfMetadata *meta);
const char *uphip_pdf_image_format_name(int32_t format);
int uphip_pdf_is_pdf_file(const char *filename);  /* by extension, pdf_reader.c:60-70 */
/* A page's pixels (pdf_pipeline_decode.c:278-320 without the render
 * fallback): JPEG / JPEG 2000 images decode on the current device; Flate and
 * raw 8-bit gray / RGB and 1-bit images, JBIG2 and CCITT fax images (both
 * expanded to GRAY8, black 0) on the host.  dpi > 0 applies the
 * reference's size check (the image within 4 px of the page at `dpi`,
 * pdf_pipeline_decode.c:69-111; a mismatch would need rendering and fails);
 * dpi 0 takes the image as it is.  read: `expect` as uphip_image_read. */
int uphip_pdf_page_probe(UphipPdfDocument *doc, int page, int32_t dpi, UphipPnmInfo *info);
int uphip_pdf_read_page(UphipPdfDocument *doc, int page, int32_t dpi, void *dst,
                        int64_t linesize, const UphipPnmInfo *expect);
/* pdf_writer.h: pages are streamed to "<path>.part" as they are added and
 * the file is renamed into place by close; abort removes it.  dpi <= 0 in
 * create = 72; dpi 0 in add_page = the writer's.  Producer is "unpaper". */
UphipPdfWriter *uphip_pdf_writer_create(const char *path, const UphipPdfMetadata *meta,
                                        int32_t dpi);
int uphip_pdf_writer_add_page_jpeg(UphipPdfWriter *writer, const uint8_t *data, size_t len,
                                   int32_t width, int32_t height, int32_t dpi);
int uphip_pdf_writer_add_page_jp2(UphipPdfWriter *writer, const uint8_t *data, size_t len,
                                  int32_t width, int32_t height, int32_t dpi);
/* format: 0 = GRAY8, 1 = RGB24 (PdfPixelFormat) */
int uphip_pdf_writer_add_page_pixels(UphipPdfWriter *writer, const uint8_t *pixels,
                                     int32_t width, int32_t height, int32_t stride,
                                     int32_t format, int32_t dpi);
int uphip_pdf_writer_page_count(UphipPdfWriter *writer);
/* lib/jbig2_decode.h:19-45 (jbig2_decode over jbig2dec): an embedded JBIG2
 * stream (+ its globals) to a 1-bit page, MSB first, 1 = black, rows
 * `stride` bytes; free with uphip_jbig2_free_image.  Generic regions
 * (arithmetic, templates 0-3, TPGDON), symbol dictionaries and text
 * regions (csrc/jbig2.h). */
typedef struct {
  uint8_t *data;
  uint32_t width, height, stride;
} UphipJbig2Image;
int uphip_jbig2_decode(const uint8_t *data, size_t size, const uint8_t *globals,
                       size_t globals_size, UphipJbig2Image *out);
void uphip_jbig2_free_image(UphipJbig2Image *image);
int uphip_pdf_writer_close(UphipPdfWriter *writer);  /* frees the writer */
void uphip_pdf_writer_abort(UphipPdfWriter *writer); /* frees the writer */

/* ---------------------------------------------------------------------------
 * Multi-device runner — the peer of lib/batch_worker.c (batch_process_parallel,
 * :273) + lib/threadpool.c + the decode/encode queues (lib/decode_queue.c,
 * lib/encode_queue.c) + the pinned per-stream staging of
 * src/pipeline/image_pipeline.c:226-376.  One host thread per device, each
 * with `batches_per_device` batches (HIP streams) of `capacity` sheets in
 * flight; jobs are pulled in chunks from one shared counter (BatchQueue),
 * no collective.  Job j reads pages j*input_count .. j*input_count+input_count-1.
 * ------------------------------------------------------------------------- */
#define UPHIP_RUNNER_MAX_DEVICES 16
typedef struct UphipRunner UphipRunner;
typedef struct UphipSource UphipSource;
typedef struct UphipSink UphipSink;
/* Auto-sizing (the reference's VRAM tiers, src/pipeline/image_pipeline.c:
 * 237-285, there 1 stream per 3 GB capped at 8, 3 buffers per stream):
 *   geometry->capacity <= 0: sheets per batch = 2 GiB / (the sheet's input
 *     pages + its two working planes), clamped to [1, 64];
 *   batches_per_device <= 0: in-flight batches per device = as many as fit
 *     in half of the device's free memory after the first, clamped to
 *     [1, 16] (16 x 64 A4 sheets is where one MI355X stops gaining,
 *     profiles/r01_bench_sweep.txt).
 * uphip_runner_layout() reports what was chosen. */
typedef struct {
  int32_t ndevices;            /* devices used */
  const int32_t *devices;      /* their ids (NULL = 0 .. ndevices-1) */
  int32_t batches_per_device;  /* HIP streams (in-flight batches) per device; <= 0: auto */
  int32_t host_threads;        /* load/store worker threads (0 = 4 per device) */
  int32_t timing;              /* stage timing on every batch */
} UphipRunnerConfig;
typedef struct {
  const void *pages;           /* device-resident pages of this device's shard */
  int64_t pitch, page_stride;
  int64_t count;               /* sheets (jobs) in the shard */
} UphipDevicePages;
typedef struct {
  int64_t jobs_done, jobs_failed;
  int64_t jobs_per_device[UPHIP_RUNNER_MAX_DEVICES];
  double wall_s;               /* last run */
  double load_s, store_s;      /* summed over the host pool's load / store tasks */
} UphipRunnerStats;
/* Sources fill page `page` of job `job` into pinned staging; sinks receive a
 * finished sheet in the output format (pages side by side for output_count 2).
 * Called concurrently from host worker threads; return 0 on success. */
typedef int (*UphipLoadFn)(void *user, int64_t job, int32_t page, void *dst,
                           int64_t linesize);
typedef int (*UphipStoreFn)(void *user, int64_t job, const void *sheet,
                            int64_t linesize, int32_t width, int32_t height,
                            int32_t format);
UphipSource *uphip_source_callback(UphipLoadFn load, void *user);
/* page i at base + i*page_stride, rows `linesize` apart.  Memory sources and
 * sinks are page-locked (hipHostRegister) over the extent the runner reads or
 * writes on their first run and unregistered by uphip_source_destroy /
 * uphip_sink_destroy: the buffer must outlive the source or sink.  Pages that
 * overlap (page_stride 0 included) or rows shorter than the page are read
 * through the staged path. */
UphipSource *uphip_source_memory(const void *base, int64_t linesize,
                                 int64_t page_stride, int64_t npages);
/* page i decoded from paths[i] (PNM, PNG or JPEG, uphip_image_read) straight into
 * the staging slot */
UphipSource *uphip_source_pnm(const char *const *paths, int64_t npaths);
void uphip_source_destroy(UphipSource *source);
UphipSink *uphip_sink_callback(UphipStoreFn store, void *user);
UphipSink *uphip_sink_memory(void *base, int64_t linesize, int64_t sheet_stride,
                             int64_t nsheets);
/* PNM files: printf(pattern, k) with k = job*output_count + page (mod wrap
 * when wrap > 0) */
UphipSink *uphip_sink_pnm(const char *pattern, int64_t wrap);
UphipSink *uphip_sink_discard(void);
/* JPEG files (the GPU encode branch): pages encoded on the device right after
 * their batch (uphip_batch_encode_jpeg_async), only the files cross PCIe;
 * names as uphip_sink_pnm.  quality 0 = 85. */
UphipSink *uphip_sink_jpeg(const char *pattern, int64_t wrap, int32_t quality,
                           int32_t sampling);
/* Lossless JPEG 2000 files (uphip_jp2_encode of each output page, from the
 * batch's device planes, on the store tasks): the .jp2 output branch of
 * lib/encode_queue.c:883-962 (nvimgcodec_default_jp2_lossless_params). */
UphipSink *uphip_sink_jp2(const char *pattern, int64_t wrap);
/* The PDF pipeline (pdf/pdf_pipeline_cpu_batch.c:381-496, 504-628):
 * uphip_source_pdf reads page i of the document for input page i (JPEG /
 * JPEG 2000 images through the device decode of the batch, Flate / raw on
 * the load tasks; dpi as uphip_pdf_read_page).  uphip_sink_pdf writes
 * every output page into one PDF: mode UPHIP_PDF_FAST = JPEG pages (the
 * device encode of uphip_sink_jpeg, quality 0 = 85), UPHIP_PDF_HIGH =
 * lossless JPEG 2000 pages (as uphip_sink_jp2); pages in output order,
 * failed ones left out (pdf_page_accumulator.c:90-130); dpi sizes the
 * pages (0 = 300, the reference's PDF_RENDER_DPI).  uphip_sink_finish
 * completes the file (0 / -1); a PDF sink destroyed unfinished leaves no
 * file. */
#define UPHIP_PDF_FAST 0
#define UPHIP_PDF_HIGH 1
UphipSource *uphip_source_pdf(const char *path, int32_t dpi);
int64_t uphip_source_page_count(UphipSource *source);
UphipSink *uphip_sink_pdf(const char *path, const UphipPdfMetadata *meta, int32_t dpi,
                          int32_t quality, int32_t mode);
int uphip_sink_finish(UphipSink *sink);
void uphip_sink_destroy(UphipSink *sink);

UphipRunner *uphip_runner_create(const UphipOptions *options,
                                 const UphipBatchGeometry *geometry,
                                 const UphipRunnerConfig *config);
void uphip_runner_destroy(UphipRunner *runner);
/* Device-resident shards: device i processes shards[i] in place, `passes`
 * times back to back without draining between passes (benchmark steps);
 * each chunk runs on a batch whose stream is idle (the first chunks on
 * batches 0, 1, ... in order, later ones on whichever finishes first), and
 * each batch's last chunk stays resident (uphip_runner_batch,
 * uphip_runner_slot_chunk).  Returns the number of failed jobs. */
int uphip_runner_run_device(UphipRunner *runner, const UphipDevicePages *shards,
                            int32_t passes);
/* Host-fed run of jobs [0, njobs): source -> pinned staging -> device ->
 * pinned staging -> sink.  Returns the number of failed jobs. */
int uphip_runner_run_host(UphipRunner *runner, int64_t njobs, UphipSource *source,
                          UphipSink *sink);
int uphip_runner_get_stats(UphipRunner *runner, UphipRunnerStats *stats);
/* The batch layout in use (after auto-sizing): batches per device, sheets
 * per batch, device bytes per batch. */
int uphip_runner_layout(UphipRunner *runner, int32_t *batches_per_device,
                        int32_t *capacity, int64_t *batch_bytes);
int uphip_runner_output_info(UphipRunner *runner, int32_t *width, int32_t *height,
                             int32_t *format, int64_t *linesize);
UphipBatch *uphip_runner_batch(UphipRunner *runner, int32_t device_index,
                               int32_t slot);
/* The chunk batch `slot` of device `device_index` ran last (its outputs are
 * resident): first job (index into the device's shard or the host-fed job
 * range) and sheet count; -1 when the batch has run none. */
int64_t uphip_runner_slot_chunk(UphipRunner *runner, int32_t device_index, int32_t slot,
                                int32_t *count);
/* Host placement of device `device_index` (the peer of the reference's
 * per-device pools and stream-bound workers, image_pipeline.c:226-376,
 * batch_worker.c:174-253): the NUMA node of the GPU (sysfs via its PCI bus
 * id; -1 when unknown), the CPUs of that node the device thread and its
 * load/store pool are bound to (0 = not bound), and that pool's threads.
 * Pinned staging is allocated by a thread on the node, with the device
 * current (hipHostMalloc places it nearest the device). */
int uphip_runner_placement(UphipRunner *runner, int32_t device_index, int32_t *numa_node,
                           int32_t *ncpus, int32_t *pool_threads);

/* Stage timing (off by default): when on, every run records a HIP event at
 * each stage boundary on the batch stream, kept until
 * uphip_batch_kernel_times() reads and frees them. */
int uphip_batch_set_timing(UphipBatch *batch, int32_t enable);
/* Per-stage device time summed over every run since the previous call (HIP
 * events recorded between stages on the batch stream, cf. the reference's
 * --perf stage timers, lib/perf.c).  Synchronises the batch stream, returns
 * the number of stages written and clears the record. */
int uphip_batch_kernel_times(UphipBatch *batch, const char **names, float *ms,
                             int max_entries);

/* ---------------------------------------------------------------------------
 * Benchmark / test support (not part of the reference interface): the
 * deterministic synthetic page generator of BASELINE.md §3 (identical bytes
 * on host and device) and raw device buffers.
 * ------------------------------------------------------------------------- */
int uphip_synth_pages(void *device_dst, int64_t pitch, int64_t page_stride,
                      int32_t width, int32_t height, uint32_t first_page,
                      int32_t count);
/* C4 workload: RGB24 double-page sheets (two W/2 x H pages side by side). */
int uphip_synth_sheets_rgb(void *device_dst, int64_t pitch, int64_t sheet_stride,
                           int32_t width, int32_t height, uint32_t first_sheet,
                           int32_t count);
void uphip_synth_sheet_rgb_host(uint8_t *host, int64_t linesize, int32_t width,
                                int32_t height, uint32_t sheet);
void uphip_synth_page_host(uint8_t *host, int64_t linesize, int32_t width,
                           int32_t height, uint32_t page);
void *uphip_device_alloc(size_t bytes);
void uphip_device_free(void *ptr);
int uphip_memcpy_htod(void *dst, const void *src, size_t bytes);
int uphip_memcpy_dtoh(void *dst, const void *src, size_t bytes);
/* Self-check of the device's restatement of glibc sinf/cosf/powf(x, 2)
 * (csrc/libm_glibc.h; the batch path's rotation select for more than two
 * deskew edges, deskew.c:226,260-261) against this host's libm: every
 * `stride`-th float of |x| < 120 (sin/cos) and 2^-60 <= |x| < 2^61 (pow),
 * both signs.  counts = {sinf, cosf, powf mismatches, inputs}.  */
int uphip_check_libm(uint32_t stride, uint64_t counts[4]);
/* Pinned (page-locked) host memory, DMA-capable from every device. */
void *uphip_host_alloc(size_t bytes);
void uphip_host_free(void *ptr);

#ifdef __cplusplus
}
#endif

#endif /* UNPAPER_HIP_H */
