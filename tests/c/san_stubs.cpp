// Sanitizer build only (make sanitize): the host codecs are linked without the
// device kernels, so the JPEG and JPEG 2000 device halves are stubs that report no device.
#include "j2k.h"
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
namespace j2k {
size_t decode_tmp_bytes(const Image&) { return 0; }
size_t t1_slot_bytes(int, int) { return 0; }
size_t t1enc_slot_bytes(int, int) { return 0; }
bool t1enc_launch(const T1EncJob*, int, const uint32_t*, uint8_t*, uint32_t*, uint8_t*, void*, int, int,
                  int, hipStream_t) {
  return fail("jp2: no device in the sanitizer build");
}
bool t1enc_pack(const T1EncJob*, int, const uint8_t*, const uint32_t*, uint32_t*, uint8_t*, uint64_t, int32_t*,
                bool, hipStream_t) {
  return fail("jp2: no device in the sanitizer build");
}
bool t1_launch(const T1Job*, int, const uint8_t*, uint32_t*, void*, int, int, int, hipStream_t) {
  return fail("jp2: no device in the sanitizer build");
}
bool decode_launch(const Image&, uint32_t*, uint8_t*, int64_t, void*, hipStream_t) {
  return fail("jp2: no device in the sanitizer build");
}
bool encode_launch(const Image&, const uint8_t*, int64_t, uint32_t*, void*, hipStream_t) {
  return fail("jp2: no device in the sanitizer build");
}
}  // namespace j2k
}  // namespace uph
