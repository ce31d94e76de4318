// CCITT fax decoding (ITU-T T.4 / T.6) of PDF /CCITTFaxDecode images (ccitt.h).
#include "ccitt.h"

#include <algorithm>
#include <cstring>

#include "runtime.h"

namespace uph {
namespace ccitt {

namespace {

struct Code {
  uint16_t bits;  // the code, MSB first
  uint8_t len;
  int16_t run;    // run length (terminating 0-63, make-up 64-2560)
};

// T.4 Tables 2 and 3 (terminating and make-up codes) and the extended
// make-up codes shared by both colours.
const Code kWhite[] = {
    {0x35, 8, 0},   {0x7, 6, 1},    {0x7, 4, 2},    {0x8, 4, 3},    {0xB, 4, 4},    {0xC, 4, 5},
    {0xE, 4, 6},    {0xF, 4, 7},    {0x13, 5, 8},   {0x14, 5, 9},   {0x7, 5, 10},   {0x8, 5, 11},
    {0x8, 6, 12},   {0x3, 6, 13},   {0x34, 6, 14},  {0x35, 6, 15},  {0x2A, 6, 16},  {0x2B, 6, 17},
    {0x27, 7, 18},  {0xC, 7, 19},   {0x8, 7, 20},   {0x17, 7, 21},  {0x3, 7, 22},   {0x4, 7, 23},
    {0x28, 7, 24},  {0x2B, 7, 25},  {0x13, 7, 26},  {0x24, 7, 27},  {0x18, 7, 28},  {0x2, 8, 29},
    {0x3, 8, 30},   {0x1A, 8, 31},  {0x1B, 8, 32},  {0x12, 8, 33},  {0x13, 8, 34},  {0x14, 8, 35},
    {0x15, 8, 36},  {0x16, 8, 37},  {0x17, 8, 38},  {0x28, 8, 39},  {0x29, 8, 40},  {0x2A, 8, 41},
    {0x2B, 8, 42},  {0x2C, 8, 43},  {0x2D, 8, 44},  {0x4, 8, 45},   {0x5, 8, 46},   {0xA, 8, 47},
    {0xB, 8, 48},   {0x52, 8, 49},  {0x53, 8, 50},  {0x54, 8, 51},  {0x55, 8, 52},  {0x24, 8, 53},
    {0x25, 8, 54},  {0x58, 8, 55},  {0x59, 8, 56},  {0x5A, 8, 57},  {0x5B, 8, 58},  {0x4A, 8, 59},
    {0x4B, 8, 60},  {0x32, 8, 61},  {0x33, 8, 62},  {0x34, 8, 63},  {0x1B, 5, 64},  {0x12, 5, 128},
    {0x17, 6, 192}, {0x37, 7, 256}, {0x36, 8, 320}, {0x37, 8, 384}, {0x64, 8, 448}, {0x65, 8, 512},
    {0x68, 8, 576}, {0x67, 8, 640}, {0xCC, 9, 704}, {0xCD, 9, 768}, {0xD2, 9, 832}, {0xD3, 9, 896},
    {0xD4, 9, 960}, {0xD5, 9, 1024}, {0xD6, 9, 1088}, {0xD7, 9, 1152}, {0xD8, 9, 1216},
    {0xD9, 9, 1280}, {0xDA, 9, 1344}, {0xDB, 9, 1408}, {0x98, 9, 1472}, {0x99, 9, 1536},
    {0x9A, 9, 1600}, {0x18, 6, 1664}, {0x9B, 9, 1728},
};
const Code kBlack[] = {
    {0x37, 10, 0},  {0x2, 3, 1},    {0x3, 2, 2},    {0x2, 2, 3},    {0x3, 3, 4},    {0x3, 4, 5},
    {0x2, 4, 6},    {0x3, 5, 7},    {0x5, 6, 8},    {0x4, 6, 9},    {0x4, 7, 10},   {0x5, 7, 11},
    {0x7, 7, 12},   {0x4, 8, 13},   {0x7, 8, 14},   {0x18, 9, 15},  {0x17, 10, 16}, {0x18, 10, 17},
    {0x8, 10, 18},  {0x67, 11, 19}, {0x68, 11, 20}, {0x6C, 11, 21}, {0x37, 11, 22}, {0x28, 11, 23},
    {0x17, 11, 24}, {0x18, 11, 25}, {0xCA, 12, 26}, {0xCB, 12, 27}, {0xCC, 12, 28}, {0xCD, 12, 29},
    {0x68, 12, 30}, {0x69, 12, 31}, {0x6A, 12, 32}, {0x6B, 12, 33}, {0xD2, 12, 34}, {0xD3, 12, 35},
    {0xD4, 12, 36}, {0xD5, 12, 37}, {0xD6, 12, 38}, {0xD7, 12, 39}, {0x6C, 12, 40}, {0x6D, 12, 41},
    {0xDA, 12, 42}, {0xDB, 12, 43}, {0x54, 12, 44}, {0x55, 12, 45}, {0x56, 12, 46}, {0x57, 12, 47},
    {0x64, 12, 48}, {0x65, 12, 49}, {0x52, 12, 50}, {0x53, 12, 51}, {0x24, 12, 52}, {0x37, 12, 53},
    {0x38, 12, 54}, {0x27, 12, 55}, {0x28, 12, 56}, {0x58, 12, 57}, {0x59, 12, 58}, {0x2B, 12, 59},
    {0x2C, 12, 60}, {0x5A, 12, 61}, {0x66, 12, 62}, {0x67, 12, 63}, {0xF, 10, 64},  {0xC8, 12, 128},
    {0xC9, 12, 192}, {0x5B, 12, 256}, {0x33, 12, 320}, {0x34, 12, 384}, {0x35, 12, 448},
    {0x6C, 13, 512}, {0x6D, 13, 576}, {0x4A, 13, 640}, {0x4B, 13, 704}, {0x4C, 13, 768},
    {0x4D, 13, 832}, {0x72, 13, 896}, {0x73, 13, 960}, {0x74, 13, 1024}, {0x75, 13, 1088},
    {0x76, 13, 1152}, {0x77, 13, 1216}, {0x52, 13, 1280}, {0x53, 13, 1344}, {0x54, 13, 1408},
    {0x55, 13, 1472}, {0x5A, 13, 1536}, {0x5B, 13, 1600}, {0x64, 13, 1664}, {0x65, 13, 1728},
};
const Code kExtended[] = {
    {0x8, 11, 1792},  {0xC, 11, 1856},  {0xD, 11, 1920},  {0x12, 12, 1984}, {0x13, 12, 2048},
    {0x14, 12, 2112}, {0x15, 12, 2176}, {0x16, 12, 2240}, {0x17, 12, 2304}, {0x1C, 12, 2368},
    {0x1D, 12, 2432}, {0x1E, 12, 2496}, {0x1F, 12, 2560},
};

// Lookup tables indexed by the next 13 bits: (run << 4 | length), 0 = no code.
struct Tables {
  std::vector<uint32_t> white, black;
  Tables() : white(1 << 13, 0), black(1 << 13, 0) {
    auto put = [](std::vector<uint32_t>& t, const Code& c) {
      const int free = 13 - c.len;
      const uint32_t base = (uint32_t)c.bits << free;
      for (uint32_t k = 0; k < (1u << free); k++) t[base | k] = (uint32_t)c.run << 4 | c.len;
    };
    for (const Code& c : kWhite) put(white, c);
    for (const Code& c : kBlack) put(black, c);
    for (const Code& c : kExtended) {
      put(white, c);
      put(black, c);
    }
  }
};
const Tables& tables() {
  static const Tables t;
  return t;
}

struct Bits {
  const uint8_t* p;
  size_t n;
  size_t pos = 0;  // bit position
  uint32_t peek(int k) const {  // the next k (<= 25) bits, zeros past the end
    uint32_t v = 0;
    const size_t byte = pos >> 3;
    for (int i = 0; i < 4; i++) v = v << 8 | (byte + i < n ? p[byte + i] : 0);
    return (v << (pos & 7)) >> (32 - k);
  }
  void skip(int k) { pos += (size_t)k; }
  bool done() const { return pos >= 8 * n; }
  void align() { pos = (pos + 7) & ~(size_t)7; }
};

// A run of one colour: make-up codes then a terminating code; -1 on error.
int32_t read_run(Bits& b, bool black) {
  const std::vector<uint32_t>& t = black ? tables().black : tables().white;
  int32_t total = 0;
  for (int guard = 0; guard < 64; guard++) {
    if (b.done()) return -1;
    const uint32_t e = t[b.peek(13)];
    if (!e) return -1;
    b.skip((int)(e & 15));
    const int32_t run = (int32_t)(e >> 4);
    total += run;
    if (run < 64) return total;
  }
  return -1;
}

// 2D mode codes (T.4 Table 4)
enum Mode { kPass, kHoriz, kV0, kVR1, kVR2, kVR3, kVL1, kVL2, kVL3, kExt, kEol, kBad };

Mode read_mode(Bits& b) {
  const uint32_t v = b.peek(12);
  if (v >> 11) return b.skip(1), kV0;                     // 1
  if ((v >> 9) == 3) return b.skip(3), kVR1;              // 011
  if ((v >> 9) == 2) return b.skip(3), kVL1;              // 010
  if ((v >> 9) == 1) return b.skip(3), kHoriz;            // 001
  if ((v >> 8) == 1) return b.skip(4), kPass;             // 0001
  if ((v >> 6) == 3) return b.skip(6), kVR2;              // 000011
  if ((v >> 6) == 2) return b.skip(6), kVL2;              // 000010
  if ((v >> 5) == 3) return b.skip(7), kVR3;              // 0000011
  if ((v >> 5) == 2) return b.skip(7), kVL3;              // 0000010
  if ((v >> 5) == 1) return b.skip(7), kExt;              // 0000001xxx
  if (v == 1) return b.skip(12), kEol;                    // 000000000001
  return kBad;
}

bool at_eol(const Bits& b) { return b.peek(12) == 1; }

// skips fill bits (zeros) up to and including an EOL; false if none follows
bool skip_eol(Bits& b) {
  size_t save = b.pos;
  int zeros = 0;
  while (!b.done() && b.peek(1) == 0 && zeros < 4096) {
    b.skip(1);
    zeros++;
  }
  if (zeros >= 11 && !b.done() && b.peek(1) == 1) {
    b.skip(1);
    return true;
  }
  b.pos = save;
  return false;
}

}  // namespace

bool decode(const uint8_t* data, size_t n, const Params& prm, int32_t rows, Image* out, const char* name) {
  const int32_t W = prm.columns;
  if (W <= 0 || W > (1 << 20)) return fail("ccitt: %s: %d columns", name, W);
  if (rows <= 0 || rows > (1 << 20) || (int64_t)W * rows > ((int64_t)1 << 31))
    return fail("ccitt: %s: %d rows", name, rows);
  out->width = W;
  out->height = rows;
  out->stride = ((int64_t)W + 7) / 8;
  // every pixel starts white; black runs are written
  out->bits.assign((size_t)(out->stride * rows), 0);
  std::vector<int32_t> ref{W, W}, cur;  // changing elements (T.4 4.2.1.3.1), then W, W
  ref.reserve((size_t)W + 4);
  cur.reserve((size_t)W + 4);
  Bits b{data, n};
  int32_t y = 0;
  for (; y < rows; y++) {
    if (prm.byte_align && prm.k < 0) b.align();
    bool two_d = prm.k < 0;
    if (prm.k >= 0) {
      // a line starts on a byte boundary (EncodedByteAlign without EOLs), or
      // after an optional EOL (its fill bits included)
      if (prm.byte_align && !prm.eol) b.align();
      skip_eol(b);
      if (prm.k > 0) {  // the tag bit: 1 = one-dimensional line
        if (b.done()) break;
        two_d = b.peek(1) == 0;
        b.skip(1);
      }
    } else if (at_eol(b)) {  // EOFB (two EOLs) ends a G4 block
      b.skip(12);
      if (at_eol(b)) break;
      return fail("ccitt: %s: EOL inside a G4 stream (row %d)", name, y);
    }
    if (b.done()) break;
    uint8_t* row = out->bits.data() + (int64_t)y * out->stride;
    auto fill_black = [&](int32_t x0, int32_t x1) {
      x0 = std::max(x0, 0);
      x1 = std::min(x1, W);
      for (int32_t x = x0; x < x1; x++) row[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
    };
    cur.clear();
    int32_t a0 = -1;
    bool black = false;
    if (!two_d) {  // one-dimensional (modified Huffman) line
      int32_t x = 0;
      while (x < W) {
        const int32_t r = read_run(b, black);
        if (r < 0) return fail("ccitt: %s: bad run code (row %d, column %d)", name, y, x);
        if (black) fill_black(x, x + r);
        x += r;
        if (x > W) return fail("ccitt: %s: runs pass the row (row %d)", name, y);
        cur.push_back(x);
        black = !black;
      }
    } else {
      size_t i = 0;  // index into ref of the current b1 search
      while (a0 < W) {
        // b1: the first changing element right of a0 whose colour is the
        // opposite of a0's (changes to black sit at even indices)
        while (i > 0 && ref[i - 1] > a0) i--;
        while (i < ref.size() - 2 && (ref[i] <= a0 || (int)(i & 1) != (int)black)) i++;
        const int32_t b1 = ref[i], b2 = ref[i + 1 < ref.size() ? i + 1 : i];
        const Mode m = read_mode(b);
        switch (m) {
          case kPass:
            if (black) fill_black(a0, b2);
            a0 = b2;
            break;
          case kHoriz: {
            const int32_t r1 = read_run(b, black);
            const int32_t r2 = r1 < 0 ? -1 : read_run(b, !black);
            if (r1 < 0 || r2 < 0) return fail("ccitt: %s: bad run code (row %d)", name, y);
            const int32_t s = std::max(a0, 0), a1 = s + r1, a2 = a1 + r2;
            if (black) fill_black(s, a1); else fill_black(a1, a2);
            cur.push_back(a1);
            cur.push_back(a2);
            a0 = a2;
            break;
          }
          case kV0: case kVR1: case kVR2: case kVR3: case kVL1: case kVL2: case kVL3: {
            static const int kD[] = {0, 0, 0, 1, 2, 3, -1, -2, -3};
            const int32_t a1 = b1 + kD[m];
            if (a1 < std::max(a0, 0) || a1 > W) return fail("ccitt: %s: bad vertical code (row %d)", name, y);
            if (black) fill_black(a0, a1);
            cur.push_back(a1);
            a0 = a1;
            black = !black;
            break;
          }
          default:
            return fail("ccitt: %s: %s (row %d, column %d)", name,
                        m == kExt ? "extension codes are not supported" : m == kEol ? "unexpected EOL"
                                                                                     : "bad mode code",
                        y, a0);
        }
        if (a0 > W) return fail("ccitt: %s: runs pass the row (row %d)", name, y);
      }
    }
    ref.assign(cur.begin(), cur.end());
    ref.push_back(W);
    ref.push_back(W);
  }
  // rows past the data's end stay white (as readers render a short stream)
  return true;
}

}  // namespace ccitt
}  // namespace uph
