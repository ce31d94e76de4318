// Sanitizer build only (make sanitize): the host codecs are linked without the
// device kernels, so the JPEG device halves are stubs that report no device.
#include "jpeg.h"
#include "runtime.h"

namespace uph {
bool jpeg_launch(const JpegHeader&, const uint8_t*, uint8_t*, uint8_t*, int64_t, hipStream_t) {
  return fail("jpeg: no device in the sanitizer build");
}
size_t jdec_scratch_bytes(const JdecHeader&) { return 0; }
bool jdec_launch(const JdecHeader&, const uint8_t*, uint8_t*, uint8_t*, int32_t*, hipStream_t) {
  return fail("jpeg: no device in the sanitizer build");
}
}  // namespace uph
