// CCITT fax decoding (ITU-T T.4 Group 3 one- and two-dimensional, T.6
// Group 4) for PDF /CCITTFaxDecode images: what PIL and most scanning
// tools write for bilevel pages (Group 4).  The reference renders such
// pages with MuPDF (pdf_pipeline_decode.c:259-276 decodes only JPEG / PNG /
// JBIG2 itself); here they decode on the host like JBIG2 pages and expand
// to GRAY8 with the image's /BlackIs1 and /Decode.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace uph {
namespace ccitt {

// /DecodeParms of the filter (PDF 32000-1 Table 11)
struct Params {
  int32_t k = 0;            // < 0 Group 4; 0 Group 3 1-D; > 0 Group 3 mixed
  int32_t columns = 1728;
  bool byte_align = false;  // EncodedByteAlign
  bool eol = false;         // EndOfLine
  bool black_is_1 = false;  // BlackIs1
};

struct Image {
  int32_t width = 0, height = 0;
  int64_t stride = 0;
  std::vector<uint8_t> bits;  // 1 = black run, MSB first
};

// Decodes `rows` rows (rows the data does not reach stay white).
bool decode(const uint8_t* data, size_t n, const Params& prm, int32_t rows, Image* out, const char* name);

}  // namespace ccitt
}  // namespace uph
