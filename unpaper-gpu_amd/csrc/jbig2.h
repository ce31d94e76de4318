// JBIG2 (ITU-T T.88) decoding of embedded streams (PDF /JBIG2Decode, the
// embedded organisation of T.88 Annex D.3) for the PDF pipeline's JBIG2
// pages.  The reference decodes them with jbig2dec (lib/jbig2_decode.c:42-127)
// on the host and expands 1 = black to GRAY8 0 (jbig2_expand_to_gray8,
// lib/jbig2_decode.c:136-170); this is a host decoder of the parts generic
// scanned pages use:
//   - page information, end of stripe / page / file, striped pages of
//     unknown height;
//   - immediate generic regions (arithmetic coding, templates 0-3, typical
//     prediction, adaptive template pixels, unknown data length);
//   - symbol dictionaries and immediate text regions with arithmetic coding
//     (no refinement, no Huffman tables), from the stream or its globals.
// Refinement, halftone, pattern, MMR-coded and Huffman-coded segments fail
// with an error naming the segment type.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace uph {
namespace jbig2 {

struct Page {
  int32_t width = 0, height = 0;
  int64_t stride = 0;           // bytes per row
  std::vector<uint8_t> bits;    // 1 bit per pixel, MSB first, 1 = black
};

// The page's size from its page information segment (height 0 = striped,
// known only after decoding).
bool probe(const uint8_t* data, size_t n, int32_t* width, int32_t* height, const char* name);
bool decode(const uint8_t* data, size_t n, const uint8_t* globals, size_t gn, Page* out, const char* name);

}  // namespace jbig2
}  // namespace uph
