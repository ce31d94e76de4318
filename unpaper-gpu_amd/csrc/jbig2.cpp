// JBIG2 embedded-stream decoder (jbig2.h).  Section numbers are ITU-T T.88's.
#include "jbig2.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "unpaper_hip.h"
#include "j2k_t1.h"  // the MQ coder's state table (T.88 Table E.1 = T.800 Table C.2)
#include "runtime.h"

namespace uph {
namespace jbig2 {

namespace {

constexpr int64_t kMaxPixels = (int64_t)1 << 31;  // a page or region bitmap

// E.3 arithmetic decoder; contexts are one byte each: state index | mps << 7.
struct Mq {
  const uint8_t* bp;
  const uint8_t* end;
  uint32_t a, c;
  int ct;
  uint8_t at(const uint8_t* p) const { return p < end ? *p : 0xFF; }
  void bytein() {  // E.3.4 BYTEIN: past the end reads as 0xFF (a marker)
    if (at(bp) == 0xFF) {
      if (at(bp + 1) > 0x8F) {
        c += 0xFF00;
        ct = 8;
      } else {
        bp++;
        c += (uint32_t)at(bp) << 9;
        ct = 7;
      }
    } else {
      bp++;
      c += (uint32_t)at(bp) << 8;
      ct = 8;
    }
  }
  void init(const uint8_t* p, size_t n) {
    bp = p;
    end = p + n;
    c = (uint32_t)at(bp) << 16;
    bytein();
    c <<= 7;
    ct -= 7;
    a = 0x8000;
  }
  int decode(uint8_t* cx) {
    const int idx = *cx & 127, mps = *cx >> 7;
    const j2k::MqState& s = j2k::kMq[idx];
    a -= s.qe;
    int d;
    if ((c >> 16) < s.qe) {
      if (a < s.qe) {
        d = mps;
        *cx = (uint8_t)(s.nmps | mps << 7);
      } else {
        d = 1 - mps;
        *cx = (uint8_t)(s.nlps | (s.sw ? 1 - mps : mps) << 7);
      }
      a = s.qe;
    } else {
      c -= (uint32_t)s.qe << 16;
      if (a & 0x8000) return mps;
      if (a < s.qe) {
        d = 1 - mps;
        *cx = (uint8_t)(s.nlps | (s.sw ? 1 - mps : mps) << 7);
      } else {
        d = mps;
        *cx = (uint8_t)(s.nmps | mps << 7);
      }
    }
    do {
      if (ct == 0) bytein();
      a <<= 1;
      c <<= 1;
      ct--;
    } while (a < 0x8000);
    return d;
  }
};

// A.2 integer decoding procedure (IAx); false = OOB.
struct IntCx {
  uint8_t cx[512];
  IntCx() { memset(cx, 0, sizeof cx); }
  bool decode(Mq& mq, int32_t* v) {
    int prev = 1;
    auto bit = [&]() {
      const int b = mq.decode(&cx[prev]);
      prev = prev < 256 ? (prev << 1) | b : (((prev << 1) | b) & 511) | 256;
      return b;
    };
    const int s = bit();
    int nbits, offset;
    if (!bit()) {
      nbits = 2, offset = 0;
    } else if (!bit()) {
      nbits = 4, offset = 4;
    } else if (!bit()) {
      nbits = 6, offset = 20;
    } else if (!bit()) {
      nbits = 8, offset = 84;
    } else if (!bit()) {
      nbits = 12, offset = 340;
    } else {
      nbits = 32, offset = 4436;
    }
    uint32_t x = 0;
    for (int k = 0; k < nbits; k++) x = (x << 1) | (uint32_t)bit();
    const int64_t val = (int64_t)x + offset;
    if (s && val == 0) return false;
    if (val > 0x7FFFFFFF) {
      *v = s ? -0x7FFFFFFF : 0x7FFFFFFF;
      return true;
    }
    *v = s ? -(int32_t)val : (int32_t)val;
    return true;
  }
};

// A.3 IAID
struct IdCx {
  std::vector<uint8_t> cx;
  int len = 0;
  explicit IdCx(int l) : cx((size_t)2 << l, 0), len(l) {}
  uint32_t decode(Mq& mq) {
    uint32_t prev = 1;
    for (int k = 0; k < len; k++) prev = (prev << 1) | (uint32_t)mq.decode(&cx[prev]);
    return prev - (1u << len);
  }
};

// A bitmap, one byte per pixel (0/1) with a margin so that template pixels
// left of, right of and above the region read 0 without bounds checks.
struct Bitmap {
  int32_t w = 0, h = 0;
  std::vector<uint8_t> px;  // (h + kTop) rows of (w + 2 * kSide)
  static constexpr int kSide = 8, kTop = 2;
  int64_t pitch() const { return (int64_t)w + 2 * kSide; }
  bool alloc(int32_t W, int32_t H, uint8_t fill) {
    if (W < 0 || H < 0 || (int64_t)W * H > kMaxPixels) return false;
    w = W;
    h = H;
    px.assign((size_t)(pitch() * ((int64_t)H + kTop)), 0);
    if (fill)
      for (int32_t y = 0; y < H; y++) memset(row(y), 1, (size_t)W);
    return true;
  }
  uint8_t* row(int32_t y) { return px.data() + ((int64_t)y + kTop) * pitch() + kSide; }
  const uint8_t* row(int32_t y) const { return px.data() + ((int64_t)y + kTop) * pitch() + kSide; }
};

int8_t s8(uint8_t b) { return (int8_t)b; }
uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

struct GenericParams {
  int tmpl = 0;
  bool tpgdon = false;
  int8_t at[8] = {3, -1, -3, -1, 2, -2, -2, -2};
};

// 6.2.5 generic region decoding (MMR = 0) into `bm` (already allocated),
// contexts `gb` (65536 / 8192 / 1024 bytes by template).
bool generic_decode(Mq& mq, const GenericParams& gp, uint8_t* gb, Bitmap* bm) {
  const int32_t W = bm->w, H = bm->h;
  const int8_t* at = gp.at;
  // AT pixels must stay inside the margin (they do for every conforming file:
  // |x| <= 8 columns, up to 2 rows above... larger ones are read through a check)
  bool at_ok = true;
  const int nat = gp.tmpl == 0 ? 4 : 1;
  for (int k = 0; k < nat; k++)
    at_ok &= at[2 * k] >= -Bitmap::kSide && at[2 * k] <= Bitmap::kSide && at[2 * k + 1] >= -Bitmap::kTop &&
             at[2 * k + 1] <= 0 && !(at[2 * k + 1] == 0 && at[2 * k] >= 0);
  if (!at_ok) return fail("jbig2: adaptive template pixel out of the supported range");
  static const uint32_t kSltp[4] = {0x9B25, 0x0795, 0x00E5, 0x0195};
  static const int8_t kNominal0[8] = {3, -1, -3, -1, 2, -2, -2, -2};
  // UPH_JBIG2_GENERIC: the per-pixel form for every region (tests compare the two)
  static const bool generic_only = getenv("UPH_JBIG2_GENERIC") != nullptr;
  const bool nominal0 = gp.tmpl == 0 && memcmp(at, kNominal0, 8) == 0 && !generic_only;
  int ltp = 0;
  for (int32_t y = 0; y < H; y++) {
    uint8_t* r0 = bm->row(y);
    const uint8_t* r1 = bm->row(y - 1);
    const uint8_t* r2 = bm->row(y - 2);
    if (gp.tpgdon) {
      ltp ^= mq.decode(&gb[kSltp[gp.tmpl]]);
      if (ltp) {  // a row equal to the one above (all 0 above the region)
        memcpy(r0, r1, (size_t)W);
        continue;
      }
    }
    if (nominal0) {
      // template 0 with the nominal AT pixels: the context is three sliding
      // windows -- row y: x-1..x-4 (bits 0-3), row y-1: x+3..x-3 (bits
      // 4-10), row y-2: x+2..x-2 (bits 11-15), the rightmost pixel lowest
      uint32_t w0 = 0;
      uint32_t w1 = (uint32_t)r1[-3] << 6 | (uint32_t)r1[-2] << 5 | (uint32_t)r1[-1] << 4 | (uint32_t)r1[0] << 3 |
                    (uint32_t)r1[1] << 2 | (uint32_t)r1[2] << 1 | r1[3];
      uint32_t w2 = (uint32_t)r2[-2] << 4 | (uint32_t)r2[-1] << 3 | (uint32_t)r2[0] << 2 | (uint32_t)r2[1] << 1 | r2[2];
      // the coder's registers in locals: stores through the byte pointers
      // (contexts, pixels) may alias the struct, which would reload it
      Mq m = mq;
      for (int32_t x = 0; x < W; x++) {
        const uint32_t b = (uint32_t)m.decode(&gb[w2 << 11 | w1 << 4 | w0]);
        r0[x] = (uint8_t)b;
        w0 = ((w0 << 1) | b) & 0xF;
        w1 = ((w1 << 1) | r1[x + 4]) & 0x7F;
        w2 = ((w2 << 1) | r2[x + 3]) & 0x1F;
      }
      mq = m;
      continue;
    }
    auto P = [&](int dx, int dy) -> uint32_t { return bm->row(y + dy)[dx]; };
    for (int32_t x = 0; x < W; x++) {
      uint32_t cx;
      const uint8_t* c0 = r0 + x;
      const uint8_t* c1 = r1 + x;
      const uint8_t* c2 = r2 + x;
      switch (gp.tmpl) {
        case 0:
          cx = (uint32_t)c0[-1] | (uint32_t)c0[-2] << 1 | (uint32_t)c0[-3] << 2 | (uint32_t)c0[-4] << 3 |
               P(x + at[0], at[1]) << 4 | (uint32_t)c1[2] << 5 | (uint32_t)c1[1] << 6 | (uint32_t)c1[0] << 7 |
               (uint32_t)c1[-1] << 8 | (uint32_t)c1[-2] << 9 | P(x + at[2], at[3]) << 10 |
               P(x + at[4], at[5]) << 11 | (uint32_t)c2[1] << 12 | (uint32_t)c2[0] << 13 |
               (uint32_t)c2[-1] << 14 | P(x + at[6], at[7]) << 15;
          break;
        case 1:
          cx = (uint32_t)c0[-1] | (uint32_t)c0[-2] << 1 | (uint32_t)c0[-3] << 2 | P(x + at[0], at[1]) << 3 |
               (uint32_t)c1[2] << 4 | (uint32_t)c1[1] << 5 | (uint32_t)c1[0] << 6 | (uint32_t)c1[-1] << 7 |
               (uint32_t)c1[-2] << 8 | (uint32_t)c2[2] << 9 | (uint32_t)c2[1] << 10 | (uint32_t)c2[0] << 11 |
               (uint32_t)c2[-1] << 12;
          break;
        case 2:
          cx = (uint32_t)c0[-1] | (uint32_t)c0[-2] << 1 | P(x + at[0], at[1]) << 2 | (uint32_t)c1[1] << 3 |
               (uint32_t)c1[0] << 4 | (uint32_t)c1[-1] << 5 | (uint32_t)c1[-2] << 6 | (uint32_t)c2[1] << 7 |
               (uint32_t)c2[0] << 8 | (uint32_t)c2[-1] << 9;
          break;
        default:
          cx = (uint32_t)c0[-1] | (uint32_t)c0[-2] << 1 | (uint32_t)c0[-3] << 2 | (uint32_t)c0[-4] << 3 |
               P(x + at[0], at[1]) << 4 | (uint32_t)c1[1] << 5 | (uint32_t)c1[0] << 6 | (uint32_t)c1[-1] << 7 |
               (uint32_t)c1[-2] << 8 | (uint32_t)c1[-3] << 9;
          break;
      }
      r0[x] = (uint8_t)mq.decode(&gb[cx]);
    }
  }
  return true;
}

size_t gb_contexts(int tmpl) { return tmpl == 0 ? 65536 : tmpl == 1 ? 8192 : 1024; }

// 6.3.6 combination of a bitmap onto another at (x, y); only the rows and
// columns inside dst are walked.  Returns the number of pixels combined.
int64_t compose(Bitmap* dst, const Bitmap& src, int64_t x, int64_t y, int op) {
  const int64_t r0 = std::max<int64_t>(0, -y), r1 = std::min<int64_t>(src.h, (int64_t)dst->h - y);
  const int64_t x0 = std::max<int64_t>(0, -x), x1 = std::min<int64_t>(src.w, (int64_t)dst->w - x);
  if (r1 <= r0 || x1 <= x0) return 0;
  for (int64_t r = r0; r < r1; r++) {
    const int64_t ty = y + r;
    const uint8_t* s = src.row((int32_t)r);
    uint8_t* d = dst->row((int32_t)ty);
    for (int64_t c = x0; c < x1; c++) {
      uint8_t& o = d[x + c];
      const uint8_t v = s[c];
      switch (op) {
        case 0: o |= v; break;
        case 1: o &= v; break;
        case 2: o ^= v; break;
        case 3: o = (uint8_t)(1 - (o ^ v)); break;
        default: o = v; break;
      }
    }
  }
  return (r1 - r0) * (x1 - x0);
}

struct Segment {
  uint32_t number = 0;
  int type = 0;
  std::vector<uint32_t> refs;
  const uint8_t* data = nullptr;
  size_t len = 0;
};

// 7.2 segment headers of an embedded stream; an immediate generic region
// of unknown length ends at its 0xFFAC marker + 4-byte row count (7.2.7).
bool parse_segments(const uint8_t* p, size_t n, std::vector<Segment>* out, const char* name) {
  size_t i = 0;
  while (i < n) {
    if (n - i < 11) return fail("jbig2: %s: truncated segment header", name);
    Segment s;
    s.number = be32(p + i);
    const uint8_t flags = p[i + 4];
    s.type = flags & 63;
    const bool big_page = flags & 64;
    i += 5;
    uint32_t nref = p[i] >> 5;
    if (nref == 7) {
      if (n - i < 4) return fail("jbig2: %s: truncated segment header", name);
      nref = be32(p + i) & 0x1FFFFFFF;
      i += 4 + (nref + 8) / 8;
    } else {
      i += 1;
    }
    if (nref > 1 << 16) return fail("jbig2: %s: %u referred-to segments", name, nref);
    const int rs = s.number <= 256 ? 1 : s.number <= 65536 ? 2 : 4;
    if (n < i || n - i < (size_t)nref * rs + (big_page ? 4 : 1) + 4)
      return fail("jbig2: %s: truncated segment header", name);
    for (uint32_t k = 0; k < nref; k++) {
      s.refs.push_back(rs == 1 ? p[i] : rs == 2 ? be16(p + i) : be32(p + i));
      i += (size_t)rs;
    }
    i += big_page ? 4 : 1;
    uint32_t len = be32(p + i);
    i += 4;
    if (len == 0xFFFFFFFF) {
      if (s.type != 38) return fail("jbig2: %s: unknown data length on segment type %d", name, s.type);
      // region info (17) + flags (1): then the coded data up to FF AC
      size_t q = i + 18;
      bool found = false;
      for (; q + 6 <= n; q++)
        if (p[q] == 0xFF && p[q + 1] == 0xAC) {
          found = true;
          break;
        }
      if (!found) return fail("jbig2: %s: generic region end marker not found", name);
      len = (uint32_t)(q + 6 - i);
    }
    if (len > n - i) return fail("jbig2: %s: segment %u data passes the end", name, s.number);
    s.data = p + i;
    s.len = len;
    i += len;
    out->push_back(std::move(s));
    if (out->back().type == 51) break;  // end of file
  }
  return true;
}

struct Dict {
  std::vector<Bitmap> syms;  // exported symbols
};

struct Decoder {
  const char* name;
  std::vector<std::pair<uint32_t, Dict>> dicts;  // by segment number
  Bitmap page;
  bool have_page = false;
  bool striped = false;
  int32_t page_h_known = 0;  // 0 = unknown (striped)
  uint8_t page_default = 0;
  int page_op = 0;
  int32_t end_row = 0;
  bool page_touched = false;  // a region has been placed

  const Dict* dict(uint32_t num) const {
    for (const auto& d : dicts)
      if (d.first == num) return &d.second;
    return nullptr;
  }

  // a striped page of unknown height grows as regions land
  bool ensure_rows(int64_t rows) {
    if (!striped || rows <= page.h) return true;
    if (rows > (1 << 20) || (int64_t)page.w * rows > kMaxPixels) return fail("jbig2: %s: page too large", name);
    const int64_t old_h = page.h;
    page.h = (int32_t)rows;
    page.px.resize((size_t)(page.pitch() * (rows + Bitmap::kTop)), 0);
    if (page_default)
      for (int64_t y = old_h; y < rows; y++) memset(page.row((int32_t)y), 1, (size_t)page.w);
    return true;
  }

  bool region_info(const Segment& s, int32_t* w, int32_t* h, int32_t* x, int32_t* y, int* op) {
    if (s.len < 17) return fail("jbig2: %s: short region segment", name);
    const uint32_t W = be32(s.data), H = be32(s.data + 4);
    if (W > (1u << 24) || H > (1u << 24) || (int64_t)W * H > kMaxPixels)
      return fail("jbig2: %s: region %ux%u", name, W, H);
    // a region no larger than its page (a crafted header must not size a
    // bitmap, or a decode loop, beyond what the page can show)
    if (!have_page) return fail("jbig2: %s: region before the page information", name);
    if ((int64_t)W > page.w || (!striped && (int64_t)H > page.h) || H > (1u << 20))
      return fail("jbig2: %s: region %ux%u larger than the page %dx%d", name, W, H, page.w, page.h);
    *w = (int32_t)W;
    *h = (int32_t)H;
    *x = (int32_t)be32(s.data + 8);
    *y = (int32_t)be32(s.data + 12);
    *op = s.data[16] & 7;
    return true;
  }

  bool place(const Bitmap& region, int32_t x, int32_t y, int op) {
    if (!have_page) return fail("jbig2: %s: region before the page information", name);
    page_touched = true;
    if (!ensure_rows((int64_t)y + region.h)) return false;
    compose(&page, region, x, y, op);
    return true;
  }

  bool page_info(const Segment& s) {
    if (s.len < 19) return fail("jbig2: %s: short page information", name);
    const uint32_t W = be32(s.data), H = be32(s.data + 4);
    const uint8_t flags = s.data[16];
    page_default = (flags >> 2) & 1;
    page_op = (flags >> 3) & 3;
    striped = H == 0xFFFFFFFF;
    if (W == 0 || W > (1u << 24) || (!striped && (H == 0 || H > (1u << 24))))
      return fail("jbig2: %s: page %ux%u", name, W, H);
    if (!page.alloc((int32_t)W, striped ? 0 : (int32_t)H, page_default))
      return fail("jbig2: %s: page %ux%u too large", name, W, H);
    have_page = true;
    return true;
  }

  bool generic_region(const Segment& s) {
    int32_t w, h, x, y;
    int op;
    if (!region_info(s, &w, &h, &x, &y, &op)) return false;
    if (s.len < 18) return fail("jbig2: %s: short generic region", name);
    const uint8_t f = s.data[17];
    if (f & 1) return fail("jbig2: %s: MMR-coded generic regions are not supported", name);
    if (f & 16) return fail("jbig2: %s: extended-template generic regions are not supported", name);
    GenericParams gp;
    gp.tmpl = (f >> 1) & 3;
    gp.tpgdon = (f >> 3) & 1;
    const size_t nat = gp.tmpl == 0 ? 8 : 2;
    if (s.len < 18 + nat) return fail("jbig2: %s: short generic region", name);
    for (size_t k = 0; k < nat; k++) gp.at[k] = s8(s.data[18 + k]);
    size_t dlen = s.len - 18 - nat;
    const uint8_t* d = s.data + 18 + nat;
    // unknown-length form: the row count after the end marker bounds the rows
    if (dlen >= 6 && d[dlen - 6] == 0xFF && d[dlen - 5] == 0xAC && striped) {
      const uint32_t rows = be32(d + dlen - 4);
      if (rows < (uint32_t)h) h = (int32_t)rows;
    }
    std::vector<uint8_t> gb(gb_contexts(gp.tmpl), 0);
    Mq mq;
    mq.init(d, dlen);
    // the common page (jbig2 -p): one region covering a fresh all-0 page,
    // combined by OR / XOR / REPLACE -- the result is the region itself, so
    // it is decoded into the page's bitmap directly
    if (!page_touched && !striped && page_default == 0 && x == 0 && y == 0 && w == page.w && h == page.h &&
        (op == 0 || op == 2 || op == 4)) {
      page_touched = true;
      return generic_decode(mq, gp, gb.data(), &page);
    }
    Bitmap bm;
    if (!bm.alloc(w, h, 0)) return fail("jbig2: %s: region %dx%d too large", name, w, h);
    if (!generic_decode(mq, gp, gb.data(), &bm)) return false;
    return place(bm, x, y, op);
  }

  bool symbol_dict(const Segment& s) {
    if (s.len < 2) return fail("jbig2: %s: short symbol dictionary", name);
    const uint16_t f = be16(s.data);
    const bool huff = f & 1, refagg = f & 2;
    if (huff) return fail("jbig2: %s: Huffman-coded symbol dictionaries are not supported", name);
    if (refagg) return fail("jbig2: %s: refinement/aggregate symbol dictionaries are not supported", name);
    if (f & 0x100) return fail("jbig2: %s: symbol dictionaries reusing coding contexts are not supported", name);
    GenericParams gp;
    gp.tmpl = (f >> 10) & 3;
    size_t i = 2;
    const size_t nat = gp.tmpl == 0 ? 8 : 2;
    if (s.len < i + nat + 8) return fail("jbig2: %s: short symbol dictionary", name);
    for (size_t k = 0; k < nat; k++) gp.at[k] = s8(s.data[i + k]);
    i += nat;
    const uint32_t nex = be32(s.data + i), nnew = be32(s.data + i + 4);
    i += 8;
    if (nnew > (1u << 20) || nex > (1u << 21)) return fail("jbig2: %s: %u symbols", name, nnew);
    std::vector<const Bitmap*> in;
    for (uint32_t r : s.refs)
      if (const Dict* d = dict(r))
        for (const Bitmap& b : d->syms) in.push_back(&b);
    Mq mq;
    mq.init(s.data + i, s.len - i);
    IntCx iadh, iadw, iaex;
    std::vector<uint8_t> gb(gb_contexts(gp.tmpl), 0);
    std::vector<Bitmap> fresh;
    fresh.reserve(nnew);
    int64_t hc = 0, area = 0;
    for (uint32_t classes = 0; fresh.size() < nnew; classes++) {
      if (classes > nnew + 16) return fail("jbig2: %s: empty height classes", name);
      int32_t dh;
      if (!iadh.decode(mq, &dh)) return fail("jbig2: %s: symbol height OOB", name);
      hc += dh;
      if (hc <= 0 || hc > (1 << 24)) return fail("jbig2: %s: symbol height %lld", name, (long long)hc);
      int64_t sw = 0;
      for (;;) {
        int32_t dw;
        if (!iadw.decode(mq, &dw)) break;  // end of the height class
        if (fresh.size() >= nnew) return fail("jbig2: %s: more symbols than declared", name);
        sw += dw;
        if (sw < 0 || sw > (1 << 24) || sw * hc > (1 << 24))
          return fail("jbig2: %s: symbol %lldx%lld", name, (long long)sw, (long long)hc);
        area += sw * hc;
        if (area > (1 << 28)) return fail("jbig2: %s: symbol dictionary too large", name);
        Bitmap b;
        b.alloc((int32_t)sw, (int32_t)hc, 0);
        if (sw > 0 && !generic_decode(mq, gp, gb.data(), &b)) return false;
        fresh.push_back(std::move(b));
      }
    }
    // 6.5.10 exported symbols: runs alternating not-exported / exported
    Dict out;
    const size_t total = in.size() + fresh.size();
    size_t idx = 0;
    bool exflag = false;
    while (idx < total) {
      int32_t run;
      if (!iaex.decode(mq, &run) || run < 0 || (size_t)run > total - idx)
        return fail("jbig2: %s: bad export run", name);
      for (int32_t k = 0; k < run; k++, idx++)
        if (exflag) out.syms.push_back(idx < in.size() ? *in[idx] : fresh[idx - in.size()]);
      exflag = !exflag;
    }
    if (out.syms.size() != nex) return fail("jbig2: %s: %zu symbols exported, %u declared", name, out.syms.size(), nex);
    dicts.emplace_back(s.number, std::move(out));
    return true;
  }

  bool text_region(const Segment& s) {
    int32_t w, h, x, y;
    int op;
    if (!region_info(s, &w, &h, &x, &y, &op)) return false;
    size_t i = 17;
    if (s.len < i + 2) return fail("jbig2: %s: short text region", name);
    const uint16_t f = be16(s.data + i);
    i += 2;
    if (f & 1) return fail("jbig2: %s: Huffman-coded text regions are not supported", name);
    if (f & 2) return fail("jbig2: %s: refinement text regions are not supported", name);
    const int logstrips = (f >> 2) & 3, corner = (f >> 4) & 3, combop = (f >> 7) & 3;
    const bool transposed = (f >> 6) & 1;
    const uint8_t defpix = (f >> 9) & 1;
    int dsoff = (f >> 10) & 31;
    if (dsoff > 15) dsoff -= 32;
    if (s.len < i + 4) return fail("jbig2: %s: short text region", name);
    const uint32_t ninst = be32(s.data + i);
    i += 4;
    if (ninst > (1u << 22)) return fail("jbig2: %s: %u symbol instances", name, ninst);
    std::vector<const Bitmap*> syms;
    for (uint32_t r : s.refs)
      if (const Dict* d = dict(r))
        for (const Bitmap& b : d->syms) syms.push_back(&b);
    if (syms.empty()) return fail("jbig2: %s: text region without symbols", name);
    int codelen = 0;
    while ((1ull << codelen) < syms.size()) codelen++;
    Bitmap bm;
    if (!bm.alloc(w, h, defpix)) return fail("jbig2: %s: region %dx%d too large", name, w, h);
    Mq mq;
    mq.init(s.data + i, s.len - i);
    IntCx iadt, iafs, iads, iait;
    IdCx iaid(codelen);
    const int strips = 1 << logstrips;
    int32_t v;
    if (!iadt.decode(mq, &v)) return fail("jbig2: %s: bad strip", name);
    int64_t stript = -(int64_t)v * strips, firsts = 0;
    uint32_t n = 0;
    int64_t placed = 0;
    const int64_t place_cap = 16 * (int64_t)w * h + ((int64_t)1 << 24);
    while (n < ninst) {
      if (!iadt.decode(mq, &v)) return fail("jbig2: %s: bad strip", name);
      stript += (int64_t)v * strips;
      bool first = true;
      int64_t curs = 0;
      for (;;) {
        if (first) {
          if (!iafs.decode(mq, &v)) return fail("jbig2: %s: bad first S", name);
          firsts += v;
          curs = firsts;
          first = false;
        } else {
          if (!iads.decode(mq, &v)) break;  // end of strip
          curs += v + dsoff;
        }
        if (n >= ninst) return fail("jbig2: %s: more symbol instances than declared", name);
        int32_t curt = 0;
        if (strips != 1 && !iait.decode(mq, &curt)) return fail("jbig2: %s: bad T", name);
        const int64_t t = stript + curt;
        const uint32_t id = iaid.decode(mq);
        if (id >= syms.size()) return fail("jbig2: %s: symbol id %u of %zu", name, id, syms.size());
        const Bitmap& ib = *syms[id];
        const int64_t wi = ib.w, hi = ib.h;
        // 6.4.5 (3)(c)(x): the reference corner (0 bottom-left, 1 top-left,
        // 2 bottom-right, 3 top-right)
        if (!transposed && (corner == 2 || corner == 3)) curs += wi - 1;
        if (transposed && (corner == 0 || corner == 2)) curs += hi - 1;
        const int64_t si = curs;
        int64_t px, py;
        if (!transposed) {
          px = (corner == 2 || corner == 3) ? si - wi + 1 : si;
          py = (corner == 0 || corner == 2) ? t - hi + 1 : t;
        } else {
          px = (corner == 2 || corner == 3) ? t - wi + 1 : t;
          py = (corner == 0 || corner == 2) ? si - hi + 1 : si;
        }
        // instances are bounded by the region, not their total: a crafted
        // stream could stack millions of region-sized symbols
        placed += compose(&bm, ib, px, py, combop);
        if (placed > place_cap)
          return fail("jbig2: %s: text region places %lld pixels into %dx%d", name, (long long)placed,
                      w, h);
        if (!transposed && (corner == 0 || corner == 1)) curs += wi - 1;
        if (transposed && (corner == 1 || corner == 3)) curs += hi - 1;
        n++;
      }
    }
    return place(bm, x, y, op);
  }

  bool run(const std::vector<Segment>& segs, bool globals) {
    for (const Segment& s : segs) {
      switch (s.type) {
        case 0:
          if (!symbol_dict(s)) return false;
          break;
        case 48:
          if (globals) return fail("jbig2: %s: page information in the globals", name);
          if (have_page) return fail("jbig2: %s: more than one page", name);
          if (!page_info(s)) return false;
          break;
        case 38:
        case 39:
          if (!generic_region(s)) return false;
          break;
        case 6:
        case 7:
          if (!text_region(s)) return false;
          break;
        case 50:  // end of stripe
          if (s.len >= 4 && striped) {
            const uint32_t row = be32(s.data);
            if (row < (1u << 24) && !ensure_rows((int64_t)row + 1)) return false;
            end_row = (int32_t)std::min<uint32_t>(row + 1, 1u << 24);
          }
          break;
        case 49:  // end of page
        case 51:  // end of file
        case 52:  // profiles
        case 53:  // tables (only Huffman segments use them)
        case 62:  // extension
          break;
        default:
          return fail("jbig2: %s: segment type %d (%s) is not supported", name, s.type,
                      s.type == 4 ? "intermediate text region"
                      : s.type == 16 ? "pattern dictionary"
                      : s.type >= 20 && s.type <= 23 ? "halftone region"
                      : s.type == 36 ? "intermediate generic region"
                      : s.type >= 40 && s.type <= 43 ? "generic refinement region"
                                                     : "unknown");
      }
    }
    return true;
  }
};

}  // namespace

bool probe(const uint8_t* data, size_t n, int32_t* width, int32_t* height, const char* name) {
  std::vector<Segment> segs;
  if (!parse_segments(data, n, &segs, name)) return false;
  for (const Segment& s : segs)
    if (s.type == 48) {
      if (s.len < 19) return fail("jbig2: %s: short page information", name);
      const uint32_t W = be32(s.data), H = be32(s.data + 4);
      if (W == 0 || W > (1u << 24) || (H != 0xFFFFFFFF && (H == 0 || H > (1u << 24))))
        return fail("jbig2: %s: page %ux%u", name, W, H);
      *width = (int32_t)W;
      *height = H == 0xFFFFFFFF ? 0 : (int32_t)H;
      return true;
    }
  return fail("jbig2: %s: no page information segment", name);
}

bool decode(const uint8_t* data, size_t n, const uint8_t* globals, size_t gn, Page* out, const char* name) {
  Decoder dec;
  dec.name = name;
  if (globals && gn) {
    std::vector<Segment> gs;
    if (!parse_segments(globals, gn, &gs, name) || !dec.run(gs, true)) return false;
  }
  std::vector<Segment> segs;
  if (!parse_segments(data, n, &segs, name) || !dec.run(segs, false)) return false;
  if (!dec.have_page) return fail("jbig2: %s: no page information segment", name);
  if (dec.striped && dec.end_row > dec.page.h && !dec.ensure_rows(dec.end_row)) return false;
  const Bitmap& pg = dec.page;
  out->width = pg.w;
  out->height = pg.h;
  out->stride = ((int64_t)pg.w + 7) / 8;
  out->bits.assign((size_t)(out->stride * pg.h), 0);
  for (int32_t y = 0; y < pg.h; y++) {
    const uint8_t* r = pg.row(y);
    uint8_t* o = out->bits.data() + (int64_t)y * out->stride;
    for (int32_t x = 0; x < pg.w; x++)
      if (r[x]) o[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
  }
  return true;
}

}  // namespace jbig2
}  // namespace uph

// ---------------------------------------------------------------------------
// C ABI (include/unpaper_hip.h): lib/jbig2_decode.h's decode on this decoder
// ---------------------------------------------------------------------------
extern "C" {

int uphip_jbig2_decode(const uint8_t* data, size_t size, const uint8_t* globals, size_t globals_size,
                       UphipJbig2Image* out) {
  if (!out) return uph::fail("jbig2_decode: null output"), -1;
  memset(out, 0, sizeof(*out));
  if (!data || !size) return uph::fail("jbig2_decode: no data"), -1;
  uph::jbig2::Page pg;
  if (!uph::jbig2::decode(data, size, globals, globals_size, &pg, "<memory>")) return -1;
  out->data = (uint8_t*)malloc(pg.bits.size() ? pg.bits.size() : 1);
  if (!out->data) return uph::fail("jbig2_decode: out of memory"), -1;
  memcpy(out->data, pg.bits.data(), pg.bits.size());
  out->width = (uint32_t)pg.width;
  out->height = (uint32_t)pg.height;
  out->stride = (uint32_t)pg.stride;
  return 0;
}

void uphip_jbig2_free_image(UphipJbig2Image* image) {
  if (!image) return;
  free(image->data);
  memset(image, 0, sizeof(*image));
}

}  // extern "C"
