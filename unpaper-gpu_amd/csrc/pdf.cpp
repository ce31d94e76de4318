// PDF container reader and writer (pdf.h).  The reference's pdf/ layer sits
// on MuPDF; this file reimplements the part of it the pipeline uses:
// open / page count / page info / page image extraction / metadata
// (pdf/pdf_reader.h) and the image-per-page writer (pdf/pdf_writer.h).
#include "pdf.h"

#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <set>

#include <fcntl.h>
#include <sys/uio.h>
#include <unistd.h>

#include <thread>

#include "ccitt.h"
#include "j2k.h"
#include "jbig2.h"
#include "jpeg.h"
#include "runtime.h"

namespace uph {
namespace pdf {

namespace {

constexpr int kMaxDepth = 64;                      // nesting of arrays / dicts / references
constexpr size_t kStreamCap = (size_t)1 << 30;     // decoded non-image streams
constexpr int64_t kMaxObjects = (int64_t)1 << 24;  // xref size accepted
constexpr int kMaxPages = 1 << 20;

bool is_ws(uint8_t c) { return c == 0 || c == 9 || c == 10 || c == 12 || c == 13 || c == 32; }
bool is_delim(uint8_t c) {
  return c == '(' || c == ')' || c == '<' || c == '>' || c == '[' || c == ']' || c == '{' ||
         c == '}' || c == '/' || c == '%';
}
bool is_regular(uint8_t c) { return !is_ws(c) && !is_delim(c); }
int hexval(uint8_t c) {
  return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10
                                        : c >= 'A' && c <= 'F' ? c - 'A' + 10
                                                               : -1;
}

// Tokens and objects over a byte range (the file, or a decoded object stream).
struct Parser {
  const uint8_t* p;
  size_t n;
  size_t pos;

  void ws() {
    while (pos < n) {
      if (is_ws(p[pos])) {
        pos++;
      } else if (p[pos] == '%') {
        while (pos < n && p[pos] != '\n' && p[pos] != '\r') pos++;
      } else {
        break;
      }
    }
  }
  // the keyword kw at pos, ending at a delimiter / whitespace / the end
  bool at_keyword(const char* kw) const {
    const size_t L = strlen(kw);
    if (pos + L > n || memcmp(p + pos, kw, L) != 0) return false;
    return pos + L == n || !is_regular(p[pos + L]);
  }
  bool keyword(const char* kw) {
    ws();
    if (!at_keyword(kw)) return false;
    pos += strlen(kw);
    return true;
  }
  // an unsigned integer token
  bool uint(int64_t* v) {
    ws();
    size_t q = pos;
    int64_t x = 0;
    int digits = 0;
    while (q < n && p[q] >= '0' && p[q] <= '9') {
      if (++digits > 18) return false;
      x = x * 10 + (p[q++] - '0');
    }
    if (!digits || (q < n && is_regular(p[q]))) return false;  // 12abc, 1.5
    pos = q;
    *v = x;
    return true;
  }

  bool number(Obj* o) {
    size_t q = pos;
    bool neg = false, real = false;
    if (q < n && (p[q] == '+' || p[q] == '-')) neg = p[q++] == '-';
    // some writers emit "--5" or "+-5": take the last sign (MuPDF does similar)
    while (q < n && (p[q] == '+' || p[q] == '-')) neg = p[q++] == '-';
    double v = 0, scale = 1;
    int64_t iv = 0;
    int digits = 0;
    for (; q < n; q++) {
      const uint8_t c = p[q];
      if (c >= '0' && c <= '9') {
        digits++;
        if (real) {
          scale /= 10;
          v += (c - '0') * scale;
        } else {
          v = v * 10 + (c - '0');
          if (iv < ((int64_t)1 << 58)) iv = iv * 10 + (c - '0');
        }
      } else if (c == '.' && !real) {
        real = true;
      } else {
        break;
      }
    }
    if (!digits && !real) return false;
    pos = q;
    if (real || v >= (double)((int64_t)1 << 58)) {
      o->t = T::Real;
      o->r = neg ? -v : v;
    } else {
      o->t = T::Int;
      o->i = neg ? -iv : iv;
    }
    return true;
  }

  bool name(std::string* s) {
    pos++;  // '/'
    s->clear();
    while (pos < n && is_regular(p[pos])) {
      if (p[pos] == '#' && pos + 2 < n && hexval(p[pos + 1]) >= 0 && hexval(p[pos + 2]) >= 0) {
        s->push_back((char)(hexval(p[pos + 1]) * 16 + hexval(p[pos + 2])));
        pos += 3;
      } else {
        s->push_back((char)p[pos++]);
      }
    }
    return true;
  }

  bool literal(std::string* s) {
    pos++;  // '('
    int depth = 1;
    s->clear();
    while (pos < n) {
      uint8_t c = p[pos++];
      if (c == '(') {
        depth++;
      } else if (c == ')') {
        if (--depth == 0) return true;
      } else if (c == '\\') {
        if (pos >= n) return false;
        c = p[pos++];
        switch (c) {
          case 'n': s->push_back('\n'); continue;
          case 'r': s->push_back('\r'); continue;
          case 't': s->push_back('\t'); continue;
          case 'b': s->push_back('\b'); continue;
          case 'f': s->push_back('\f'); continue;
          case '\r':
            if (pos < n && p[pos] == '\n') pos++;
            continue;
          case '\n': continue;
          default:
            if (c >= '0' && c <= '7') {
              int v = c - '0';
              for (int k = 0; k < 2 && pos < n && p[pos] >= '0' && p[pos] <= '7'; k++)
                v = v * 8 + (p[pos++] - '0');
              s->push_back((char)(v & 255));
            } else {
              s->push_back((char)c);  // \( \) \\ and unknown escapes: the character
            }
            continue;
        }
      } else if (c == '\r') {  // end-of-line in a string reads as \n
        if (pos < n && p[pos] == '\n') pos++;
        c = '\n';
      }
      s->push_back((char)c);
    }
    return false;
  }

  bool hexstring(std::string* s) {
    pos++;  // '<'
    s->clear();
    int hi = -1;
    while (pos < n) {
      const uint8_t c = p[pos++];
      if (c == '>') {
        if (hi >= 0) s->push_back((char)(hi << 4));
        return true;
      }
      if (is_ws(c)) continue;
      const int v = hexval(c);
      if (v < 0) return false;
      if (hi < 0) {
        hi = v;
      } else {
        s->push_back((char)(hi * 16 + v));
        hi = -1;
      }
    }
    return false;
  }

  bool parse(Obj* o, int depth) {
    if (depth > kMaxDepth) return false;
    ws();
    if (pos >= n) return false;
    const uint8_t c = p[pos];
    *o = Obj();
    if (c == '/') {
      o->t = T::Name;
      return name(&o->s);
    }
    if (c == '(') {
      o->t = T::Str;
      return literal(&o->s);
    }
    if (c == '<') {
      if (pos + 1 < n && p[pos + 1] == '<') {
        pos += 2;
        o->t = T::Dict;
        for (;;) {
          ws();
          if (pos + 1 < n && p[pos] == '>' && p[pos + 1] == '>') {
            pos += 2;
            return true;
          }
          if (pos >= n || p[pos] != '/') return false;
          std::string key;
          name(&key);
          Obj v;
          if (!parse(&v, depth + 1)) return false;
          o->d.emplace_back(std::move(key), std::move(v));
        }
      }
      o->t = T::Str;
      return hexstring(&o->s);
    }
    if (c == '[') {
      pos++;
      o->t = T::Arr;
      for (;;) {
        ws();
        if (pos < n && p[pos] == ']') {
          pos++;
          return true;
        }
        Obj v;
        if (!parse(&v, depth + 1)) return false;
        o->a.push_back(std::move(v));
      }
    }
    if ((c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.') {
      if (!number(o)) return false;
      // "num gen R"
      if (o->t == T::Int && o->i >= 0 && c != '+' && c != '-') {
        const size_t save = pos;
        int64_t gen = 0;
        if (uint(&gen) && keyword("R")) {
          o->t = T::Ref;
          o->gen = (int32_t)std::min<int64_t>(gen, 65535);
          return true;
        }
        pos = save;
      }
      return true;
    }
    if (at_keyword("true") || at_keyword("false")) {
      o->t = T::Bool;
      o->i = p[pos] == 't';
      pos += o->i ? 4 : 5;
      return true;
    }
    if (at_keyword("null")) {
      pos += 4;
      return true;
    }
    return false;
  }

  // finds `kw` at or after `from` (a plain byte search)
  size_t find(const char* kw, size_t from) const {
    const size_t L = strlen(kw);
    for (size_t q = from; q + L <= n; q++)
      if (p[q] == (uint8_t)kw[0] && memcmp(p + q, kw, L) == 0) return q;
    return std::string::npos;
  }
};

std::string canonical_filter(const std::string& f) {
  if (f == "AHx") return "ASCIIHexDecode";
  if (f == "A85") return "ASCII85Decode";
  if (f == "LZW") return "LZWDecode";
  if (f == "Fl") return "FlateDecode";
  if (f == "RL") return "RunLengthDecode";
  if (f == "CCF") return "CCITTFaxDecode";
  if (f == "DCT") return "DCTDecode";
  return f;
}

bool ascii_hex(const uint8_t* p, size_t n, std::vector<uint8_t>* out) {
  out->clear();
  int hi = -1;
  for (size_t i = 0; i < n; i++) {
    if (p[i] == '>') break;
    if (is_ws(p[i])) continue;
    const int v = hexval(p[i]);
    if (v < 0) return fail("pdf: ASCIIHexDecode: bad digit");
    if (hi < 0) {
      hi = v;
    } else {
      out->push_back((uint8_t)(hi * 16 + v));
      hi = -1;
    }
  }
  if (hi >= 0) out->push_back((uint8_t)(hi << 4));
  return true;
}

bool ascii85(const uint8_t* p, size_t n, std::vector<uint8_t>* out) {
  out->clear();
  uint32_t tuple = 0;
  int cnt = 0;
  for (size_t i = 0; i < n; i++) {
    const uint8_t c = p[i];
    if (is_ws(c)) continue;
    if (c == '~') break;
    if (c == 'z' && cnt == 0) {
      out->insert(out->end(), 4, 0);
      continue;
    }
    if (c < '!' || c > 'u') return fail("pdf: ASCII85Decode: bad character");
    tuple = tuple * 85 + (uint32_t)(c - '!');
    if (++cnt == 5) {
      for (int k = 3; k >= 0; k--) out->push_back((uint8_t)(tuple >> (8 * k)));
      tuple = 0;
      cnt = 0;
    }
  }
  if (cnt == 1) return fail("pdf: ASCII85Decode: truncated group");
  if (cnt > 1) {
    for (int k = cnt; k < 5; k++) tuple = tuple * 85 + 84;
    for (int k = 0; k < cnt - 1; k++) out->push_back((uint8_t)(tuple >> (24 - 8 * k)));
  }
  return true;
}

bool run_length(const uint8_t* p, size_t n, std::vector<uint8_t>* out, size_t cap) {
  out->clear();
  size_t i = 0;
  while (i < n) {
    const int len = p[i++];
    if (len == 128) break;
    if (len < 128) {
      const size_t L = (size_t)len + 1;
      if (i + L > n) return fail("pdf: RunLengthDecode: truncated run");
      out->insert(out->end(), p + i, p + i + L);
      i += L;
    } else {
      if (i >= n) return fail("pdf: RunLengthDecode: truncated run");
      out->insert(out->end(), (size_t)(257 - len), p[i++]);
    }
    if (out->size() > cap) return fail("pdf: RunLengthDecode: output too large");
  }
  return true;
}

// LZWDecode (PDF 32000-1 §7.4.4): 9..12-bit codes, MSB first, 256 clear,
// 257 end; EarlyChange 1 (the default) widens the code one entry early.
bool lzw(const uint8_t* p, size_t n, int early, std::vector<uint8_t>* out, size_t cap) {
  out->clear();
  std::vector<uint32_t> prefix(4096);
  std::vector<uint8_t> suffix(4096), first(4096);
  std::vector<uint16_t> len(4096);
  for (int k = 0; k < 256; k++) {
    prefix[(size_t)k] = 0xFFFFFFFFu;
    suffix[(size_t)k] = first[(size_t)k] = (uint8_t)k;
    len[(size_t)k] = 1;
  }
  int next = 258, width = 9, prev = -1;
  uint32_t acc = 0;
  int bits = 0;
  size_t i = 0;
  std::vector<uint8_t> tmp;
  for (;;) {
    while (bits < width && i < n) {
      acc = (acc << 8) | p[i++];
      bits += 8;
    }
    if (bits < width) break;
    const int code = (int)((acc >> (bits - width)) & ((1u << width) - 1));
    bits -= width;
    if (code == 256) {
      next = 258;
      width = 9;
      prev = -1;
      continue;
    }
    if (code == 257) break;
    int cur = code;
    if (code >= next) {
      if (code != next || prev < 0) return fail("pdf: LZWDecode: bad code");
      cur = prev;  // KwKwK: prev's string + its first byte
    }
    tmp.resize(len[(size_t)cur]);
    for (int c = cur, k = (int)tmp.size() - 1; k >= 0; k--) {
      tmp[(size_t)k] = suffix[(size_t)c];
      c = (int)prefix[(size_t)c];
    }
    if (code >= next) tmp.push_back(first[(size_t)prev]);
    out->insert(out->end(), tmp.begin(), tmp.end());
    if (out->size() > cap) return fail("pdf: LZWDecode: output too large");
    if (prev >= 0 && next < 4096) {
      prefix[(size_t)next] = (uint32_t)prev;
      suffix[(size_t)next] = tmp[0];
      first[(size_t)next] = first[(size_t)prev];
      len[(size_t)next] = (uint16_t)(len[(size_t)prev] + 1);
      next++;
    }
    prev = code;
    if (next + early >= (1 << width) && width < 12) width++;
  }
  return true;
}

// PDFDocEncoding 0x80..0x9F as Unicode (PDF 32000-1 Annex D)
const uint16_t kDocEnc80[32] = {0x2022, 0x2020, 0x2021, 0x2026, 0x2014, 0x2013, 0x0192, 0x2044,
                                0x2039, 0x203A, 0x2212, 0x2030, 0x201E, 0x201C, 0x201D, 0x2018,
                                0x2019, 0x201A, 0x2122, 0xFB01, 0xFB02, 0x0141, 0x0152, 0x0160,
                                0x0178, 0x017D, 0x0131, 0x0142, 0x0153, 0x0161, 0x017E, 0xFFFD};

void put_utf8(std::string* s, uint32_t cp) {
  if (cp < 0x80) {
    s->push_back((char)cp);
  } else if (cp < 0x800) {
    s->push_back((char)(0xC0 | (cp >> 6)));
    s->push_back((char)(0x80 | (cp & 63)));
  } else if (cp < 0x10000) {
    s->push_back((char)(0xE0 | (cp >> 12)));
    s->push_back((char)(0x80 | ((cp >> 6) & 63)));
    s->push_back((char)(0x80 | (cp & 63)));
  } else {
    s->push_back((char)(0xF0 | (cp >> 18)));
    s->push_back((char)(0x80 | ((cp >> 12) & 63)));
    s->push_back((char)(0x80 | ((cp >> 6) & 63)));
    s->push_back((char)(0x80 | (cp & 63)));
  }
}

// A PDF text string (UTF-16BE with BOM, UTF-8 with BOM, or PDFDocEncoding) as
// UTF-8 -- what pdf_to_text_string gives the reference (pdf_reader.c:776-787).
std::string text_string(const std::string& b) {
  std::string s;
  const uint8_t* u = (const uint8_t*)b.data();
  const size_t n = b.size();
  if (n >= 2 && u[0] == 0xFE && u[1] == 0xFF) {
    for (size_t i = 2; i + 1 < n; i += 2) {
      uint32_t cp = (uint32_t)u[i] << 8 | u[i + 1];
      if (cp >= 0xD800 && cp < 0xDC00 && i + 3 < n) {
        const uint32_t lo = (uint32_t)u[i + 2] << 8 | u[i + 3];
        if (lo >= 0xDC00 && lo < 0xE000) {
          cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          i += 2;
        }
      }
      put_utf8(&s, cp);
    }
    return s;
  }
  if (n >= 3 && u[0] == 0xEF && u[1] == 0xBB && u[2] == 0xBF) return b.substr(3);
  for (size_t i = 0; i < n; i++)
    put_utf8(&s, u[i] >= 0x80 && u[i] < 0xA0 ? kDocEnc80[u[i] - 0x80] : u[i]);
  return s;
}

// The components of a JPEG from its frame header (pdf_writer.c:195-220 scans
// for SOF0..2; every SOF marker is read here).
int jpeg_components(const uint8_t* d, size_t n) {
  size_t i = 2;
  while (i + 4 <= n) {
    if (d[i] != 0xFF) {
      i++;
      continue;
    }
    const uint8_t m = d[i + 1];
    if (m == 0xFF) {
      i++;
      continue;
    }
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {
      i += 2;
      continue;
    }
    const size_t L = (size_t)d[i + 2] << 8 | d[i + 3];
    if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)
      return i + 9 < n ? d[i + 9] : 0;
    i += 2 + L;
  }
  return 0;
}

}  // namespace

const Obj* Obj::get(const char* key) const {
  for (const auto& kv : d)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

// ---------------------------------------------------------------------------
// filters
// ---------------------------------------------------------------------------

bool inflate_bytes(const uint8_t* p, size_t n, std::vector<uint8_t>* out, size_t cap) {
  out->clear();
  for (int attempt = 0; attempt < 2; attempt++) {
    z_stream z{};
    // a zlib stream; a headerless deflate stream on the second try
    if (inflateInit2(&z, attempt == 0 ? 15 : -15) != Z_OK) return fail("pdf: zlib init failed");
    z.next_in = const_cast<Bytef*>(p);
    z.avail_in = (uInt)std::min<size_t>(n, 0x7FFFFFFF);
    size_t have = 0;
    out->resize(std::min<size_t>(std::max<size_t>(n * 4, 4096), cap + 1));
    int rc = Z_OK;
    for (;;) {
      if (have == out->size()) {
        if (out->size() > cap) break;
        out->resize(std::min(out->size() * 2, cap + 1));
      }
      z.next_out = out->data() + have;
      z.avail_out = (uInt)std::min<size_t>(out->size() - have, 0x7FFFFFFF);
      rc = inflate(&z, Z_NO_FLUSH);
      have = (size_t)(z.next_out - out->data());
      if (rc == Z_STREAM_END) break;
      if (rc == Z_BUF_ERROR && z.avail_in == 0) break;  // truncated: keep what decoded
      if (rc != Z_OK && rc != Z_BUF_ERROR) break;
    }
    inflateEnd(&z);
    if (have > cap) return fail("pdf: FlateDecode: output passes %zu bytes", cap);
    if (rc == Z_STREAM_END || (rc == Z_BUF_ERROR && have > 0) || (rc == Z_OK && have > 0)) {
      out->resize(have);
      return true;
    }
    if (attempt == 0 && rc == Z_DATA_ERROR && have == 0) continue;
    return fail("pdf: FlateDecode: corrupt data (zlib %d)", rc);
  }
  return fail("pdf: FlateDecode: corrupt data");
}

bool unpredict(std::vector<uint8_t>* data, int predictor, int colors, int bpc, int columns) {
  if (predictor <= 1) return true;
  if (colors < 1 || colors > 32 || columns < 1 || columns > (1 << 24) ||
      (bpc != 1 && bpc != 2 && bpc != 4 && bpc != 8 && bpc != 16))
    return fail("pdf: bad predictor parameters");
  const size_t rb = ((size_t)colors * bpc * columns + 7) / 8;
  const int bpp = std::max(1, colors * bpc / 8);
  std::vector<uint8_t>& d = *data;
  if (predictor == 2) {
    if (bpc != 8) return fail("pdf: TIFF predictor with %d bits per component is not supported", bpc);
    for (size_t r = 0; r + rb <= d.size(); r += rb)
      for (size_t x = (size_t)colors; x < rb; x++) d[r + x] = (uint8_t)(d[r + x] + d[r + x - colors]);
    return true;
  }
  if (predictor < 10) return fail("pdf: unknown predictor %d", predictor);
  const size_t rows = d.size() / (rb + 1);
  std::vector<uint8_t> out(rows * rb);
  std::vector<uint8_t> zero(rb, 0);
  for (size_t r = 0; r < rows; r++) {
    const uint8_t type = d[r * (rb + 1)];
    const uint8_t* in = d.data() + r * (rb + 1) + 1;
    uint8_t* o = out.data() + r * rb;
    const uint8_t* up = r ? out.data() + (r - 1) * rb : zero.data();
    for (size_t x = 0; x < rb; x++) {
      const int a = x >= (size_t)bpp ? o[x - bpp] : 0;
      const int b = up[x];
      const int c = x >= (size_t)bpp ? up[x - bpp] : 0;
      int v;
      switch (type) {
        case 0: v = in[x]; break;
        case 1: v = in[x] + a; break;
        case 2: v = in[x] + b; break;
        case 3: v = in[x] + ((a + b) >> 1); break;
        case 4: {
          const int pp = a + b - c, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - c);
          v = in[x] + (pa <= pb && pa <= pc ? a : pb <= pc ? b : c);
          break;
        }
        default: return fail("pdf: PNG predictor: bad row filter %d", type);
      }
      o[x] = (uint8_t)v;
    }
  }
  d.swap(out);
  return true;
}

namespace {

struct FilterSpec {
  std::string name;
  const Obj* parms = nullptr;
};

int parm_int(Document* doc, const Obj* parms, const char* key, int dflt) {
  if (!parms) return dflt;
  const Obj* v = doc->resolve(parms->get(key));
  return v && v->t == T::Int ? (int)std::max<int64_t>(-(1 << 30), std::min<int64_t>(v->i, 1 << 30)) : dflt;
}

bool filters_of(Document* doc, const Obj& dict, std::vector<FilterSpec>* out) {
  out->clear();
  const Obj* f = doc->resolve(dict.get("Filter"));
  if (!f) f = doc->resolve(dict.get("F"));
  const Obj* dp = doc->resolve(dict.get("DecodeParms"));
  if (!dp) dp = doc->resolve(dict.get("DP"));
  if (!f || f->t == T::Null) return true;
  if (f->t == T::Name) {
    out->push_back({canonical_filter(f->s), dp && dp->t == T::Dict ? dp : nullptr});
    return true;
  }
  if (f->t != T::Arr) return fail("pdf: %s: bad /Filter", doc->name().c_str());
  for (size_t k = 0; k < f->a.size(); k++) {
    const Obj* nm = doc->resolve(&f->a[k]);
    if (!nm || nm->t != T::Name) return fail("pdf: %s: bad /Filter entry", doc->name().c_str());
    const Obj* pk = nullptr;
    if (dp && dp->t == T::Arr && k < dp->a.size()) {
      pk = doc->resolve(&dp->a[k]);
      if (pk && pk->t != T::Dict) pk = nullptr;
    }
    out->push_back({canonical_filter(nm->s), pk});
  }
  return true;
}

bool apply_filter(Document* doc, const FilterSpec& fs, std::vector<uint8_t>* buf, size_t cap) {
  std::vector<uint8_t> out;
  const std::string& f = fs.name;
  if (f == "FlateDecode" || f == "LZWDecode") {
    if (f == "FlateDecode") {
      if (!inflate_bytes(buf->data(), buf->size(), &out, cap)) return false;
    } else if (!lzw(buf->data(), buf->size(), parm_int(doc, fs.parms, "EarlyChange", 1), &out, cap)) {
      return false;
    }
    if (!unpredict(&out, parm_int(doc, fs.parms, "Predictor", 1), parm_int(doc, fs.parms, "Colors", 1),
                   parm_int(doc, fs.parms, "BitsPerComponent", 8), parm_int(doc, fs.parms, "Columns", 1)))
      return false;
  } else if (f == "ASCIIHexDecode") {
    if (!ascii_hex(buf->data(), buf->size(), &out)) return false;
  } else if (f == "ASCII85Decode") {
    if (!ascii85(buf->data(), buf->size(), &out)) return false;
  } else if (f == "RunLengthDecode") {
    if (!run_length(buf->data(), buf->size(), &out, cap)) return false;
  } else {
    return fail("pdf: %s: filter /%s is not supported here", doc->name().c_str(), f.c_str());
  }
  if (out.size() > cap) return fail("pdf: %s: decoded stream passes %zu bytes", doc->name().c_str(), cap);
  buf->swap(out);
  return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// document
// ---------------------------------------------------------------------------

bool Document::open(std::vector<uint8_t>&& bytes, const char* name) {
  own_ = std::move(bytes);
  p_ = own_.data();
  n_ = own_.size();
  name_ = name ? name : "<memory>";
  return init();
}

bool Document::open_view(const uint8_t* p, size_t n, const char* name) {
  p_ = p;
  n_ = n;
  name_ = name ? name : "<memory>";
  return init();
}

void Document::set_entry(int64_t num, uint8_t type, int64_t a, int64_t b) {
  if (num < 0 || num >= kMaxObjects) return;
  if ((size_t)num >= xref_.size()) {
    xref_.resize((size_t)num + 1);
    seen_.resize((size_t)num + 1, false);
  }
  if (seen_[(size_t)num] || type == 0) return;  // newer sections first; free entries set nothing
  seen_[(size_t)num] = true;
  xref_[(size_t)num] = XEnt{type, a, b};
}

bool Document::read_xref_table(size_t pos, Obj* trailer) {
  Parser ps{p_, n_, pos};
  if (!ps.keyword("xref")) return false;
  for (;;) {
    ps.ws();
    if (ps.at_keyword("trailer")) break;
    int64_t start = 0, count = 0;
    if (!ps.uint(&start) || !ps.uint(&count) || count > kMaxObjects || start > kMaxObjects)
      return false;
    for (int64_t k = 0; k < count; k++) {
      int64_t off = 0, gen = 0;
      if (!ps.uint(&off) || !ps.uint(&gen)) return false;
      ps.ws();
      if (ps.pos >= n_) return false;
      const uint8_t t = p_[ps.pos++];
      if (t == 'n' && off > 0)
        set_entry(start + k, 1, off, gen);
      else if (t != 'n' && t != 'f')
        return false;
    }
  }
  if (!ps.keyword("trailer")) return false;
  return ps.parse(trailer, 0) && trailer->t == T::Dict;
}

bool Document::read_xref_stream(size_t pos, Obj* trailer) {
  Obj s;
  if (!parse_indirect_at(pos, -1, &s, 0) || s.t != T::Stream) return false;
  const Obj* type = s.get("Type");
  if (!type || !type->is_name("XRef")) return false;
  const Obj* W = s.get("W");
  if (!W || W->t != T::Arr || W->a.size() < 3) return false;
  int w[3];
  for (int k = 0; k < 3; k++) {
    if (W->a[(size_t)k].t != T::Int || W->a[(size_t)k].i < 0 || W->a[(size_t)k].i > 8) return false;
    w[k] = (int)W->a[(size_t)k].i;
  }
  const Obj* size = s.get("Size");
  if (!size || size->t != T::Int || size->i < 0 || size->i > kMaxObjects) return false;
  std::vector<int64_t> index;
  const Obj* ix = s.get("Index");
  if (ix && ix->t == T::Arr) {
    for (const Obj& v : ix->a) {
      if (v.t != T::Int || v.i < 0 || v.i > kMaxObjects) return false;
      index.push_back(v.i);
    }
    if (index.size() % 2) return false;
  } else {
    index = {0, size->i};
  }
  std::vector<uint8_t> data;
  // the stream's own /Length may not be a reference (it is parsed before the
  // xref exists), so stream_data works here
  if (!stream_data(s, &data, (size_t)kMaxObjects * 20)) return false;
  const size_t rec = (size_t)(w[0] + w[1] + w[2]);
  if (!rec) return false;
  size_t at = 0;
  for (size_t q = 0; q < index.size(); q += 2) {
    for (int64_t k = 0; k < index[q + 1]; k++) {
      if (at + rec > data.size()) return true;  // short: what is there counts
      int64_t f[3] = {1, 0, 0};
      for (int c = 0; c < 3; c++) {
        if (!w[c]) continue;
        int64_t v = 0;
        for (int b = 0; b < w[c]; b++) v = v << 8 | data[at++];
        f[c] = v;
      }
      if (f[0] == 1 || f[0] == 2) set_entry(index[q] + k, (uint8_t)f[0], f[1], f[2]);
    }
  }
  *trailer = Obj();
  trailer->t = T::Dict;
  trailer->d = s.d;
  return true;
}

bool Document::read_xref_chain(int64_t off) {
  std::set<int64_t> visited;
  bool first = true;
  while (off > 0) {
    if ((size_t)off >= n_ || !visited.insert(off).second || visited.size() > 4096) return false;
    Parser ps{p_, n_, (size_t)off};
    ps.ws();
    Obj tr;
    if (ps.at_keyword("xref")) {
      if (!read_xref_table(ps.pos, &tr)) return false;
      const Obj* xs = tr.get("XRefStm");  // hybrid file: the stream's entries next
      if (xs && xs->t == T::Int && xs->i > 0 && (size_t)xs->i < n_) {
        Obj ignored;
        read_xref_stream((size_t)xs->i, &ignored);
      }
    } else if (!read_xref_stream(ps.pos, &tr)) {
      return false;
    }
    if (first) {
      trailer_ = tr;
      first = false;
    } else {
      for (const char* key : {"Root", "Info", "Encrypt", "ID"})
        if (!trailer_.get(key) && tr.get(key)) trailer_.d.emplace_back(key, *tr.get(key));
    }
    const Obj* prev = tr.get("Prev");
    off = prev && prev->t == T::Int ? prev->i : 0;
  }
  return !first;
}

// The file scanned for "n g obj" (later definitions win) and its trailer
// (the last "trailer" dictionary, else an xref stream's, else the catalog),
// as readers do with damaged files.
bool Document::reconstruct() {
  reconstructed_ = true;
  std::vector<XEnt> x;
  std::vector<bool> s;
  Obj tr;
  bool have_tr = false;
  for (size_t q = 0; q + 3 <= n_; q++) {
    if (p_[q] == 't' && q + 7 <= n_ && memcmp(p_ + q, "trailer", 7) == 0) {
      Parser t{p_, n_, q + 7};
      Obj d;
      if (t.parse(&d, 0) && d.t == T::Dict && d.get("Root")) {
        tr = d;
        have_tr = true;
      }
      continue;
    }
    if (p_[q] != 'o' || memcmp(p_ + q, "obj", 3) != 0) continue;
    if (q + 3 < n_ && is_regular(p_[q + 3])) continue;
    // back over "num gen "
    size_t e = q;
    while (e > 0 && is_ws(p_[e - 1])) e--;
    size_t g = e;
    while (g > 0 && p_[g - 1] >= '0' && p_[g - 1] <= '9') g--;
    if (g == e) continue;
    size_t f = g;
    while (f > 0 && is_ws(p_[f - 1])) f--;
    if (f == g) continue;
    size_t b = f;
    while (b > 0 && p_[b - 1] >= '0' && p_[b - 1] <= '9') b--;
    if (b == f || f - b > 10) continue;
    if (b > 0 && is_regular(p_[b - 1])) continue;
    int64_t num = 0;
    for (size_t k = b; k < f; k++) num = num * 10 + (p_[k] - '0');
    if (num <= 0 || num >= kMaxObjects) continue;
    if ((size_t)num >= x.size()) {
      x.resize((size_t)num + 1);
      s.resize((size_t)num + 1, false);
    }
    x[(size_t)num] = XEnt{1, (int64_t)b, 0};
    s[(size_t)num] = true;
  }
  // keep the compressed entries the damaged xref did hold for objects the
  // scan did not find
  for (size_t k = 0; k < xref_.size() && k < (size_t)kMaxObjects; k++)
    if (xref_[k].type == 2 && (k >= s.size() || !s[k])) {
      if (k >= x.size()) {
        x.resize(k + 1);
        s.resize(k + 1, false);
      }
      x[k] = xref_[k];
      s[k] = true;
    }
  xref_.swap(x);
  seen_.swap(s);
  // cached objects stay: they parsed, and callers may hold pointers to them
  // objects inside object streams the scan cannot see
  for (size_t k = 0; k < xref_.size(); k++) {
    if (xref_[k].type != 1) continue;
    Obj o;
    if (!parse_indirect_at((size_t)xref_[k].a, (int64_t)k, &o, 0) || o.t != T::Stream) continue;
    const Obj* t = o.get("Type");
    if (t && t->is_name("XRef") && !have_tr && o.get("Root")) {
      tr = Obj();
      tr.t = T::Dict;
      tr.d = o.d;
      have_tr = true;
    }
    if (!t || !t->is_name("ObjStm")) continue;
    std::vector<uint8_t> d;
    const Obj* N = o.get("N");
    if (!N || N->t != T::Int || N->i <= 0 || N->i > 1000000 || !stream_data(o, &d, kStreamCap)) continue;
    Parser hp{d.data(), d.size(), 0};
    for (int64_t j = 0; j < N->i; j++) {
      int64_t num = 0, off = 0;
      if (!hp.uint(&num) || !hp.uint(&off)) break;
      if (num <= 0 || num >= kMaxObjects) continue;
      if ((size_t)num >= xref_.size()) {
        xref_.resize((size_t)num + 1);
        seen_.resize((size_t)num + 1, false);
      }
      if (!seen_[(size_t)num]) {
        xref_[(size_t)num] = XEnt{2, (int64_t)k, j};
        seen_[(size_t)num] = true;
      }
    }
  }
  if (!have_tr) {  // find the catalog
    for (size_t k = 0; k < xref_.size() && !have_tr; k++) {
      const Obj* o = load((int64_t)k, 0);
      const Obj* t = o && (o->t == T::Dict || o->t == T::Stream) ? o->get("Type") : nullptr;
      if (t && t->is_name("Catalog")) {
        tr = Obj();
        tr.t = T::Dict;
        Obj ref;
        ref.t = T::Ref;
        ref.i = (int64_t)k;
        tr.d.emplace_back("Root", ref);
        have_tr = true;
      }
    }
  }
  if (!have_tr) return fail("pdf: %s: no document catalog found", name_.c_str());
  trailer_ = tr;
  return true;
}

bool Document::parse_indirect_at(size_t pos, int64_t expect_num, Obj* out, int depth) {
  if (pos >= n_) return false;
  Parser ps{p_, n_, pos};
  int64_t num = 0, gen = 0;
  if (!ps.uint(&num) || !ps.uint(&gen) || !ps.keyword("obj")) return false;
  if (expect_num >= 0 && num != expect_num) return false;
  if (!ps.parse(out, depth)) {
    // "n g obj endobj": an empty object reads as null
    ps.ws();
    if (!ps.at_keyword("endobj")) return false;
    *out = Obj();
    return true;
  }
  if (out->t != T::Dict) return true;
  const size_t save = ps.pos;
  if (!ps.keyword("stream")) {
    ps.pos = save;
    return true;
  }
  // the data starts after CRLF or LF (a lone CR tolerated)
  size_t s = ps.pos;
  if (s < n_ && p_[s] == '\r') s++;
  if (s < n_ && p_[s] == '\n') s++;
  int64_t len = -1;
  const Obj* L = out->get("Length");
  if (L && L->t == T::Int) {
    len = L->i;
  } else if (L && L->t == T::Ref && depth < kMaxDepth) {
    const Obj* r = load(L->i, depth + 1);
    if (r && r->t == T::Int) len = r->i;
  }
  bool good = len >= 0 && (size_t)len <= n_ - s;
  if (good) {
    Parser e{p_, n_, s + (size_t)len};
    good = e.keyword("endstream");
  }
  if (!good) {  // a wrong /Length: up to the endstream keyword
    const size_t e = ps.find("endstream", s);
    if (e == std::string::npos) return false;
    size_t end = e;
    if (end > s && p_[end - 1] == '\n') end--;
    if (end > s && p_[end - 1] == '\r') end--;
    len = (int64_t)(end - s);
  }
  out->t = T::Stream;
  out->soff = s;
  out->slen = (size_t)len;
  return true;
}

bool Document::load_objstm(int64_t stm, int depth) {
  const Obj* o = load(stm, depth + 1);
  if (!o || o->t != T::Stream) return false;
  const Obj* N = o->get("N");
  const Obj* F = o->get("First");
  if (!N || N->t != T::Int || !F || F->t != T::Int || N->i <= 0 || N->i > 1000000 || F->i < 0)
    return false;
  std::vector<uint8_t> d;
  if (!stream_data(*o, &d, kStreamCap, depth + 1)) return false;
  Parser hp{d.data(), d.size(), 0};
  std::vector<std::pair<int64_t, int64_t>> idx;
  for (int64_t j = 0; j < N->i; j++) {
    int64_t num = 0, off = 0;
    if (!hp.uint(&num) || !hp.uint(&off)) break;
    idx.emplace_back(num, off);
  }
  for (size_t j = 0; j < idx.size(); j++) {
    const int64_t num = idx[j].first;
    // only objects the xref places in this stream (a later update may
    // have replaced others)
    if (num < 0 || (size_t)num >= xref_.size() || xref_[(size_t)num].type != 2 ||
        xref_[(size_t)num].a != stm || cache_.count(num))
      continue;
    const size_t at = (size_t)F->i + (size_t)idx[j].second;
    if (at >= d.size()) continue;
    Parser op{d.data(), d.size(), at};
    std::unique_ptr<Obj> v(new Obj());
    if (!op.parse(v.get(), depth + 1)) continue;
    cache_[num] = std::move(v);
  }
  return true;
}

const Obj* Document::load(int64_t num, int depth) {
  if (num <= 0 || depth > kMaxDepth) return nullptr;
  auto it = cache_.find(num);
  if (it != cache_.end()) return it->second.get();
  if ((size_t)num >= xref_.size() || xref_[(size_t)num].type == 0) return nullptr;
  if (loading_[num]++) {  // a reference cycle (e.g. a /Length pointing at its own object)
    loading_[num]--;
    return nullptr;
  }
  const XEnt e = xref_[(size_t)num];
  const Obj* result = nullptr;
  if (e.type == 1) {
    std::unique_ptr<Obj> v(new Obj());
    if (parse_indirect_at((size_t)e.a, num, v.get(), depth)) {
      result = v.get();
      cache_[num] = std::move(v);
    }
  } else if (e.type == 2) {
    if (load_objstm(e.a, depth)) {
      auto jt = cache_.find(num);
      if (jt != cache_.end()) result = jt->second.get();
    }
  }
  loading_[num]--;
  if (!result && !reconstructed_ && e.type == 1) {  // a stale offset: rebuild the xref once
    if (reconstruct()) return load(num, depth + 1);
  }
  return result;
}

const Obj* Document::resolve(const Obj* o, int depth) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  for (int k = 0; o && o->t == T::Ref; k++) {
    if (k > kMaxDepth) return nullptr;
    o = load(o->i, depth + 1);
  }
  return o;
}

bool Document::stream_data(const Obj& stream, std::vector<uint8_t>* out, size_t cap, int depth,
                           int first, int last) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  if (stream.t != T::Stream || depth > kMaxDepth) return fail("pdf: %s: not a stream", name_.c_str());
  std::vector<FilterSpec> fs;
  if (!filters_of(this, stream, &fs)) return false;
  if (last < 0 || last > (int)fs.size()) last = (int)fs.size();
  out->assign(p_ + stream.soff, p_ + stream.soff + stream.slen);
  for (int k = std::max(first, 0); k < last; k++)
    if (!apply_filter(this, fs[(size_t)k], out, cap)) return false;
  return true;
}

bool Document::build_pages() {
  const Obj* root = resolve(trailer_.get("Root"));
  if (!root || root->t != T::Dict) return fail("pdf: %s: no document catalog", name_.c_str());
  const Obj* tree = resolve(root->get("Pages"));
  if (!tree || tree->t != T::Dict) return fail("pdf: %s: no page tree", name_.c_str());
  struct Item {
    const Obj* node;
    Obj res, media, crop, rotate;  // inherited so far (Null = none)
    int depth;
  };
  std::vector<Item> stack;
  stack.push_back(Item{tree, Obj(), Obj(), Obj(), Obj(), 0});
  std::set<const Obj*> visited;
  while (!stack.empty()) {
    Item it = std::move(stack.back());
    stack.pop_back();
    const Obj* node = it.node;
    if (!node || (node->t != T::Dict && node->t != T::Stream)) continue;
    if (!visited.insert(node).second) return fail("pdf: %s: page tree has a cycle", name_.c_str());
    for (auto kv : {std::make_pair("Resources", &it.res), std::make_pair("MediaBox", &it.media),
                    std::make_pair("CropBox", &it.crop), std::make_pair("Rotate", &it.rotate)})
      if (const Obj* v = node->get(kv.first)) *kv.second = *v;
    const Obj* type = node->get("Type");
    const Obj* kids = resolve(node->get("Kids"));
    const bool is_tree = (type && type->is_name("Pages")) || (!type && kids && kids->t == T::Arr);
    if (is_tree) {
      if (!kids || kids->t != T::Arr) continue;
      if (it.depth > kMaxDepth) return fail("pdf: %s: page tree too deep", name_.c_str());
      for (size_t k = kids->a.size(); k-- > 0;) {  // reversed: the stack pops in order
        const Obj* kid = resolve(&kids->a[k]);
        stack.push_back(Item{kid, it.res, it.media, it.crop, it.rotate, it.depth + 1});
      }
      continue;
    }
    if ((int)pages_.size() >= kMaxPages) return fail("pdf: %s: too many pages", name_.c_str());
    PageRec pr;
    pr.dict.t = T::Dict;
    pr.dict.d = node->d;
    const Obj* own = resolve(node->get("Rotate"));
    pr.own_rotate = own && own->is_num() ? (int32_t)own->num() : 0;
    for (auto kv : {std::make_pair("Resources", &it.res), std::make_pair("MediaBox", &it.media),
                    std::make_pair("CropBox", &it.crop), std::make_pair("Rotate", &it.rotate)})
      if (!node->get(kv.first) && kv.second->t != T::Null) pr.dict.d.emplace_back(kv.first, *kv.second);
    pages_.push_back(std::move(pr));
  }
  return true;
}

bool Document::init() {
  if (!p_ || n_ < 8) return fail("pdf: %s: not a PDF (too short)", name_.c_str());
  // the header within the first 1 KiB (some files carry leading junk)
  Parser hp{p_, std::min<size_t>(n_, 1024), 0};
  if (hp.find("%PDF-", 0) == std::string::npos) return fail("pdf: %s: no %%PDF header", name_.c_str());
  // startxref near the end
  const size_t tail = n_ > 2048 ? n_ - 2048 : 0;
  size_t sx = std::string::npos;
  for (size_t q = n_ - 8; q-- > tail;)
    if (memcmp(p_ + q, "startxref", 9) == 0) {
      sx = q;
      break;
    }
  bool ok = false;
  if (sx != std::string::npos) {
    Parser ps{p_, n_, sx + 9};
    int64_t off = 0;
    if (ps.uint(&off) && off > 0) ok = read_xref_chain(off);
  }
  const Obj* root = nullptr;
  if (ok) root = resolve(trailer_.get("Root"));
  if (!ok || !root) {
    xref_.clear();
    seen_.clear();
    cache_.clear();
    trailer_ = Obj();
    if (!reconstruct()) return false;
  }
  encrypted_ = trailer_.get("Encrypt") != nullptr;
  if (encrypted_) return true;  // pages stay unread (pdf_doc_needs_password)
  if (!build_pages()) {
    if (reconstructed_) return false;
    pages_.clear();
    uphip_clear_error();
    if (!reconstruct() || !build_pages()) return false;
  }
  return true;
}

bool Document::page_box(int page, PageBox* out) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  if (page < 0 || page >= (int)pages_.size())
    return fail("pdf: %s: page %d out of range (%d pages)", name_.c_str(), page, (int)pages_.size());
  const Obj& pg = pages_[(size_t)page].dict;
  auto rect = [&](const char* key, float r[4]) {
    const Obj* a = resolve(pg.get(key));
    if (!a || a->t != T::Arr || a->a.size() < 4) return false;
    for (int k = 0; k < 4; k++) {
      const Obj* v = resolve(&a->a[(size_t)k]);
      if (!v || !v->is_num()) return false;
      r[k] = (float)v->num();
    }
    if (r[0] > r[2]) std::swap(r[0], r[2]);
    if (r[1] > r[3]) std::swap(r[1], r[3]);
    return true;
  };
  float m[4] = {0, 0, 612, 792}, c[4];  // US Letter when the box is missing (as MuPDF)
  rect("MediaBox", m);
  if (rect("CropBox", c)) {
    m[0] = std::max(m[0], c[0]);
    m[1] = std::max(m[1], c[1]);
    m[2] = std::min(m[2], c[2]);
    m[3] = std::min(m[3], c[3]);
    if (m[2] < m[0]) m[2] = m[0];
    if (m[3] < m[1]) m[3] = m[1];
  }
  const Obj* rot = resolve(pg.get("Rotate"));
  int r = rot && rot->is_num() ? (int)rot->num() : 0;
  r = ((r % 360) + 360) % 360;
  r = (r + 45) / 90 * 90 % 360;  // MuPDF rounds to a quarter turn
  out->width = m[2] - m[0];
  out->height = m[3] - m[1];
  if (r == 90 || r == 270) std::swap(out->width, out->height);
  out->rotation = pages_[(size_t)page].own_rotate;
  return true;
}

bool Document::extract_image(int page, PageImage* out) {
  std::unique_lock<std::recursive_mutex> lk(mu_);
  {  // reset, keeping the data buffer's capacity (load tasks reuse one per thread)
    std::vector<uint8_t> keep = std::move(out->data);
    keep.clear();
    *out = PageImage();
    out->data = std::move(keep);
  }
  if (encrypted_) return fail("pdf: %s is encrypted (decryption is not supported)", name_.c_str());
  if (page < 0 || page >= (int)pages_.size())
    return fail("pdf: %s: page %d out of range (%d pages)", name_.c_str(), page, (int)pages_.size());
  const Obj& pg = pages_[(size_t)page].dict;
  const Obj* res = resolve(pg.get("Resources"));
  const Obj* xo = res && res->t == T::Dict ? resolve(res->get("XObject")) : nullptr;
  if (!xo || xo->t != T::Dict)
    return fail("pdf: %s: page %d has no image XObject (pages that need rendering are not supported)",
                name_.c_str(), page);
  // the largest image, first one on ties (pdf_reader.c:311-333)
  const Obj* best = nullptr;
  double best_area = 0;  // in double: /Width and /Height may be any number
  int64_t best_num = 0;
  for (const auto& kv : xo->d) {
    const Obj* o = resolve(&kv.second);
    if (!o || o->t != T::Stream) continue;
    const Obj* st = resolve(o->get("Subtype"));
    if (!st || !st->is_name("Image")) continue;
    const Obj* w = resolve(o->get("Width"));
    const Obj* h = resolve(o->get("Height"));
    if (!w || !h || !w->is_num() || !h->is_num()) continue;
    const double area = std::trunc(w->num()) * std::trunc(h->num());
    if (area > best_area) {
      best = o;
      best_area = area;
      best_num = kv.second.t == T::Ref ? kv.second.i : 0;
    }
  }
  if (!best)
    return fail("pdf: %s: page %d has no image XObject (pages that need rendering are not supported)",
                name_.c_str(), page);
  const Obj& im = *best;
  out->object = (int32_t)best_num;
  const Obj* w = resolve(im.get("Width"));
  const Obj* h = resolve(im.get("Height"));
  if (w->num() < 1 || h->num() < 1 || w->num() > (1 << 20) || h->num() > (1 << 20) ||
      w->num() * h->num() > 2147483648.0)
    return fail("pdf: %s: page %d: image size %gx%g", name_.c_str(), page, w->num(), h->num());
  out->width = (int32_t)w->num();
  out->height = (int32_t)h->num();
  const Obj* mask = resolve(im.get("ImageMask"));
  if (!mask) mask = resolve(im.get("IM"));
  out->mask = mask && mask->t == T::Bool && mask->i;
  // components from the colour space
  const Obj* cs = resolve(im.get("ColorSpace"));
  if (!cs) cs = resolve(im.get("CS"));
  int comps = 0;
  if (out->mask) {
    comps = 1;
  } else if (cs && cs->t == T::Name) {
    const std::string& s = cs->s;
    comps = (s == "DeviceGray" || s == "G" || s == "CalGray") ? 1
            : (s == "DeviceRGB" || s == "RGB" || s == "CalRGB") ? 3
            : (s == "DeviceCMYK" || s == "CMYK") ? 4
                                                 : 0;
  } else if (cs && cs->t == T::Arr && !cs->a.empty()) {
    const Obj* fam = resolve(&cs->a[0]);
    const std::string f = fam && fam->t == T::Name ? fam->s : "";
    if (f == "ICCBased" && cs->a.size() > 1) {
      const Obj* icc = resolve(&cs->a[1]);
      const Obj* N = icc && (icc->t == T::Stream || icc->t == T::Dict) ? resolve(icc->get("N")) : nullptr;
      comps = N && N->t == T::Int ? (int)N->i : 0;
    } else if ((f == "Indexed" || f == "I") && cs->a.size() >= 4) {
      // [/Indexed base hival lookup]: one index per pixel, the palette's
      // entries of the base space (lookup a string or a stream)
      comps = 1;
      out->indexed = true;
      const Obj* base = resolve(&cs->a[1]);
      int bn = 0;
      if (base && base->t == T::Name)
        bn = (base->s == "DeviceGray" || base->s == "G" || base->s == "CalGray") ? 1
             : (base->s == "DeviceRGB" || base->s == "RGB" || base->s == "CalRGB") ? 3 : 0;
      else if (base && base->t == T::Arr && !base->a.empty()) {
        const Obj* bf = resolve(&base->a[0]);
        if (bf && bf->is_name("ICCBased") && base->a.size() > 1) {
          const Obj* icc = resolve(&base->a[1]);
          const Obj* N = icc && (icc->t == T::Stream || icc->t == T::Dict) ? resolve(icc->get("N")) : nullptr;
          bn = N && N->t == T::Int && (N->i == 1 || N->i == 3) ? (int)N->i : 0;
        } else if (bf && (bf->is_name("CalRGB") || bf->is_name("DeviceRGB"))) {
          bn = 3;
        } else if (bf && (bf->is_name("CalGray") || bf->is_name("DeviceGray"))) {
          bn = 1;
        }
      }
      const Obj* hv = resolve(&cs->a[2]);
      const Obj* lk = resolve(&cs->a[3]);
      const int hival = hv && hv->t == T::Int ? (int)hv->i : -1;
      if (bn && hival >= 0 && hival <= 255 && lk) {
        if (lk->t == T::Str)
          out->palette.assign(lk->s.begin(), lk->s.end());
        else if (lk->t == T::Stream && !stream_data(*lk, &out->palette, 1 << 16))
          out->palette.clear();
        if (out->palette.size() >= (size_t)(hival + 1) * bn) {
          out->palette.resize((size_t)(hival + 1) * bn);
          out->palette_comps = bn;
        } else {
          out->palette.clear();
        }
      }
    } else if (f == "CalGray" || f == "DeviceGray" || f == "G" || f == "Separation") {
      comps = 1;
    } else if (f == "CalRGB" || f == "Lab" || f == "DeviceRGB" || f == "RGB") {
      comps = 3;
    } else if (f == "DeviceN" && cs->a.size() > 1) {
      const Obj* names = resolve(&cs->a[1]);
      comps = names && names->t == T::Arr ? (int)names->a.size() : 0;
    }
  }
  const Obj* bpc = resolve(im.get("BitsPerComponent"));
  if (!bpc) bpc = resolve(im.get("BPC"));
  out->bpc = out->mask ? 1 : bpc && bpc->t == T::Int ? (int32_t)bpc->i : 0;
  const Obj* dec = resolve(im.get("Decode"));
  if (!dec) dec = resolve(im.get("D"));
  if (dec && dec->t == T::Arr && dec->a.size() >= 2) {
    const Obj* d0 = resolve(&dec->a[0]);
    const Obj* d1 = resolve(&dec->a[1]);
    out->inverted = d0 && d1 && d0->is_num() && d1->is_num() && d0->num() == 1 && d1->num() == 0;
  }
  // the filter chain: a trailing image codec keeps its bytes (the "zero
  // copy" path, pdf_reader.c:339-366), as does a trailing FlateDecode
  std::vector<FilterSpec> fs;
  if (!filters_of(this, im, &fs)) return false;
  const std::string last = fs.empty() ? "" : fs.back().name;
  int keep_from = (int)fs.size();  // filters [keep_from, end) stay applied
  if (last == "DCTDecode") {
    out->format = kJpeg;
    keep_from--;
  } else if (last == "JPXDecode") {
    out->format = kJp2;
    keep_from--;
  } else if (last == "JBIG2Decode") {
    out->format = kJbig2;
    keep_from--;
  } else if (last == "CCITTFaxDecode") {
    out->format = kCcitt;
    keep_from--;
    const Obj* pm = fs.back().parms;
    out->fax.k = parm_int(this, pm, "K", 0);
    out->fax.columns = parm_int(this, pm, "Columns", 1728);
    auto flag = [&](const char* key, bool dflt) {
      const Obj* v = pm ? resolve(pm->get(key)) : nullptr;
      return v && v->t == T::Bool ? v->i != 0 : dflt;
    };
    out->fax.byte_align = flag("EncodedByteAlign", false);
    out->fax.eol = flag("EndOfLine", false);
    out->fax.black_is_1 = flag("BlackIs1", false);
  } else if (last == "FlateDecode") {
    out->format = kFlate;
    keep_from--;
    const Obj* pm = fs.back().parms;
    out->predictor = parm_int(this, pm, "Predictor", 1);
    out->colors = parm_int(this, pm, "Colors", 1);
    out->pbpc = parm_int(this, pm, "BitsPerComponent", 8);
    out->columns = parm_int(this, pm, "Columns", 1);
  } else {
    out->format = kRaw;  // no filter, or only ones decoded here
  }
  if (out->format == kJbig2 && fs.back().parms) {
    const Obj* g = resolve(fs.back().parms->get("JBIG2Globals"));
    if (g && g->t == T::Stream && !stream_data(*g, &out->globals, kStreamCap)) return false;
  }
  if (keep_from == 0) {
    // the stream's bytes as stored: copied outside the document lock (the
    // file buffer never changes), so load tasks of other pages do not queue
    // behind a multi-MB copy
    const size_t off = im.soff, len = im.slen;
    lk.unlock();
    out->data.assign(p_ + off, p_ + off + len);
  } else {
    const size_t raw_cap = (size_t)out->width * out->height * std::max(comps, 1) * 2 + (1 << 20);
    if (!stream_data(im, &out->data, std::max(raw_cap, im.slen * 4 + (1 << 20)), 0, 0, keep_from))
      return false;
    lk.unlock();
  }
  // what the codestream says when the dictionary does not
  if (out->format == kJpeg && !comps) comps = jpeg_components(out->data.data(), out->data.size());
  if (out->format == kJp2 && (!comps || !out->bpc)) {
    UphipPnmInfo info{0, 0, 0};
    if (j2k::probe(out->data.data(), out->data.size(), name_.c_str(), &info)) {
      if (!comps) comps = info.format == UPHIP_FMT_GRAY8 ? 1 : 3;
      if (!out->bpc) out->bpc = 8;
    } else {
      uphip_clear_error();
    }
  }
  out->components = comps;
  return true;
}

bool Document::metadata(Meta* out) {
  std::lock_guard<std::recursive_mutex> lk(mu_);
  *out = Meta();
  const Obj* info = resolve(trailer_.get("Info"));
  if (!info || info->t != T::Dict) return true;
  std::string* fields[8] = {&out->title,   &out->author,   &out->subject,       &out->keywords,
                            &out->creator, &out->producer, &out->creation_date, &out->modification_date};
  const char* keys[8] = {"Title", "Author", "Subject", "Keywords", "Creator", "Producer", "CreationDate", "ModDate"};
  for (int k = 0; k < 8; k++) {
    const Obj* v = resolve(info->get(keys[k]));
    if (v && v->t == T::Str) {
      *fields[k] = text_string(v->s);
      out->has[k] = true;
    }
  }
  return true;
}

// ---------------------------------------------------------------------------
// pixels of Flate / raw images
// ---------------------------------------------------------------------------

int pixel_format(const PageImage& im) {
  if (im.format == kJbig2 || im.format == kCcitt) return UPHIP_FMT_GRAY8;  // expanded to 0 / 255
  if (im.indexed)  // palette images expand to their base space
    return im.palette_comps && (im.bpc == 1 || im.bpc == 2 || im.bpc == 4 || im.bpc == 8)
               ? (im.palette_comps == 3 ? UPHIP_FMT_RGB24 : UPHIP_FMT_GRAY8)
               : -1;
  if (im.components == 1 && im.bpc == 8) return UPHIP_FMT_GRAY8;
  if (im.components == 3 && im.bpc == 8) return UPHIP_FMT_RGB24;
  // one bit: 0 is black under the default /Decode [0 1] (FFmpeg's monoblack)
  if (im.components == 1 && im.bpc == 1) return im.inverted ? UPHIP_FMT_MONOWHITE : UPHIP_FMT_MONOBLACK;
  return -1;
}

bool decode_pixels(const PageImage& im, uint8_t* dst, int64_t linesize, const char* name) {
  const int fmt = pixel_format(im);
  if (fmt < 0)
    return fail("pdf: %s: page image has %d components at %d bits%s: not a pixel format here", name,
                im.components, im.bpc, im.indexed ? " (indexed)" : "");
  if (im.format == kCcitt) {
    if (linesize < im.width) return fail("pdf: %s: linesize too small", name);
    ccitt::Image cm;
    ccitt::Params prm = im.fax;
    if (prm.columns != im.width)
      return fail("pdf: %s: CCITT /Columns %d but the image is %d wide", name, prm.columns, im.width);
    if (!ccitt::decode(im.data.data(), im.data.size(), prm, im.height, &cm, name)) return false;
    // a black run is the sample 1 when /BlackIs1, else 0; DeviceGray 0 is
    // black, and /Decode [1 0] swaps the two
    const uint8_t on_black = (uint8_t)((prm.black_is_1 ^ im.inverted) ? 255 : 0);
    for (int32_t y = 0; y < cm.height; y++) {
      const uint8_t* s = cm.bits.data() + (int64_t)y * cm.stride;
      uint8_t* d = dst + (int64_t)y * linesize;
      for (int32_t x = 0; x < cm.width; x++)
        d[x] = (s[x >> 3] >> (7 - (x & 7)) & 1) ? on_black : (uint8_t)(255 - on_black);
    }
    return true;
  }
  if (im.format == kJbig2) {
    // lib/jbig2_decode.c:136-170: 1 (black) -> 0, 0 -> 255
    if (linesize < im.width) return fail("pdf: %s: linesize too small", name);
    jbig2::Page pg;
    if (!jbig2::decode(im.data.data(), im.data.size(), im.globals.data(), im.globals.size(), &pg, name))
      return false;
    if (pg.width != im.width || pg.height != im.height)
      return fail("pdf: %s: the JBIG2 page is %dx%d, its dictionary says %dx%d", name, pg.width, pg.height,
                  im.width, im.height);
    for (int32_t y = 0; y < pg.height; y++) {
      const uint8_t* s = pg.bits.data() + (int64_t)y * pg.stride;
      uint8_t* d = dst + (int64_t)y * linesize;
      for (int32_t x = 0; x < pg.width; x++) d[x] = (s[x >> 3] >> (7 - (x & 7)) & 1) ? 0 : 255;
    }
    return true;
  }
  const int64_t rb = ((int64_t)im.width * im.components * im.bpc + 7) / 8;
  if (linesize < (im.indexed ? (int64_t)im.width * im.palette_comps : rb))
    return fail("pdf: %s: linesize too small", name);
  std::vector<uint8_t> inflated;
  const std::vector<uint8_t>* px = &im.data;
  if (im.format == kFlate || im.format == kPng) {
    const size_t cap = (size_t)(rb + 1) * im.height + 4096;
    if (!inflate_bytes(im.data.data(), im.data.size(), &inflated, cap)) return false;
    if (!unpredict(&inflated, im.predictor, im.colors, im.pbpc, im.columns)) return false;
    px = &inflated;
  } else if (im.format != kRaw) {
    return fail("pdf: %s: image format %d has no pixel path", name, im.format);
  }
  if ((int64_t)px->size() < rb * im.height)
    return fail("pdf: %s: image data is short (%zu bytes for %dx%d)", name, px->size(), im.width, im.height);
  if (im.indexed) {
    // indices of bpc bits, MSB first; past hival they take the last entry
    // (as MuPDF clamps)
    const int bn = im.palette_comps, bpc = im.bpc;
    const int last = (int)im.palette.size() / bn - 1;
    for (int32_t y = 0; y < im.height; y++) {
      const uint8_t* s = px->data() + (int64_t)y * rb;
      uint8_t* d = dst + (int64_t)y * linesize;
      for (int32_t x = 0; x < im.width; x++) {
        const int64_t bit = (int64_t)x * bpc;
        int idx = bpc == 8 ? s[x] : (s[bit >> 3] >> (8 - bpc - (int)(bit & 7))) & ((1 << bpc) - 1);
        if (idx > last) idx = last;
        for (int c = 0; c < bn; c++) d[x * bn + c] = im.palette[(size_t)(idx * bn + c)];
      }
    }
    return true;
  }
  const bool invert8 = im.inverted && fmt == UPHIP_FMT_GRAY8;
  for (int32_t y = 0; y < im.height; y++) {
    const uint8_t* s = px->data() + (int64_t)y * rb;
    uint8_t* d = dst + (int64_t)y * linesize;
    if (invert8) {
      for (int64_t x = 0; x < rb; x++) d[x] = (uint8_t)(255 - s[x]);
    } else {
      memcpy(d, s, (size_t)rb);
    }
  }
  return true;
}

// ---------------------------------------------------------------------------
// writer
// ---------------------------------------------------------------------------

namespace {

// A real without exponent notation (PDF has none), trailing zeros dropped.
std::string real(double v) {
  char b[64];
  snprintf(b, sizeof(b), "%.4f", v);
  std::string s = b;
  while (!s.empty() && s.back() == '0') s.pop_back();
  if (!s.empty() && s.back() == '.') s.pop_back();
  return s.empty() || s == "-" ? "0" : s;
}

// A text string: literal when printable ASCII, else UTF-16BE with a BOM.
std::string pdf_text(const std::string& utf8) {
  bool ascii = true;
  for (unsigned char c : utf8) ascii &= c >= 0x20 && c < 0x7F;
  std::string o;
  if (ascii) {
    o.push_back('(');
    for (char c : utf8) {
      if (c == '(' || c == ')' || c == '\\') o.push_back('\\');
      o.push_back(c);
    }
    o.push_back(')');
    return o;
  }
  std::vector<uint32_t> cps;
  const unsigned char* u = (const unsigned char*)utf8.data();
  for (size_t i = 0; i < utf8.size();) {
    uint32_t cp = u[i];
    int extra = cp >= 0xF0 ? 3 : cp >= 0xE0 ? 2 : cp >= 0xC0 ? 1 : 0;
    if (extra) cp &= (0x3F >> extra);
    i++;
    for (int k = 0; k < extra && i < utf8.size(); k++, i++) cp = cp << 6 | (u[i] & 63);
    cps.push_back(cp);
  }
  char b[8];
  o = "<FEFF";
  for (uint32_t cp : cps) {
    if (cp >= 0x10000) {
      cp -= 0x10000;
      snprintf(b, sizeof(b), "%04X", 0xD800 + (cp >> 10));
      o += b;
      snprintf(b, sizeof(b), "%04X", 0xDC00 + (cp & 0x3FF));
    } else {
      snprintf(b, sizeof(b), "%04X", cp);
    }
    o += b;
  }
  o.push_back('>');
  return o;
}

}  // namespace

Writer::~Writer() { abort(); }

namespace {

// all of [p, p + n) at `off`
bool pwrite_all(int fd, const struct iovec* iov, int n, int64_t off) {
  std::vector<struct iovec> v(iov, iov + n);
  size_t k = 0;
  while (k < v.size()) {
    const ssize_t w = pwritev(fd, v.data() + k, (int)(v.size() - k), (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += w;
    size_t left = (size_t)w;
    while (k < v.size() && left >= v[k].iov_len) left -= v[k++].iov_len;
    if (k < v.size()) {
      v[k].iov_base = (uint8_t*)v[k].iov_base + left;
      v[k].iov_len -= left;
    }
  }
  return true;
}

}  // namespace

bool Writer::put(const void* p, size_t n) {
  if (failed_ || fd_ < 0) return false;
  struct iovec v = {const_cast<void*>(p), n};
  if (!pwrite_all(fd_, &v, 1, pos_)) {
    failed_ = true;
    return fail("pdf_writer: cannot write %s", part_.c_str());
  }
  pos_ += (int64_t)n;
  return true;
}

bool Writer::putf(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  const int n = vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (n < 0 || n >= (int)sizeof(buf)) return false;
  return put(buf, (size_t)n);
}

void Writer::drain() {
  while (inflight_.load(std::memory_order_acquire) > 0) std::this_thread::yield();
}

bool Writer::create(const char* path, const Meta* meta, int dpi) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!path || !*path) return fail("pdf_writer: NULL path");
  path_ = path;
  part_ = path_ + ".part";
  dpi_ = dpi > 0 ? dpi : 72;  // pdf_writer.c:91-93
  fd_ = ::open(part_.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd_ < 0) return fail("pdf_writer: cannot create %s: %s", part_.c_str(), strerror(errno));
  if (meta) {
    meta_ = *meta;
    has_meta_ = true;
  }
  // objects 1 (catalog), 2 (page tree) and 3 (info) are written by close()
  offsets_.assign(4, 0);
  static const char head[] = "%PDF-1.7\n%\xE2\xE3\xCF\xD3\n";
  return put(head, sizeof(head) - 1);
}

bool Writer::add_page(int64_t index, int kind, const uint8_t* data, size_t len, int width, int height,
                      int stride, int components, int dpi) {
  if (!data || !len) return fail("pdf_writer: Invalid arguments");
  if (width <= 0 || height <= 0) return fail("pdf_writer: Invalid dimensions: %dx%d", width, height);
  std::vector<uint8_t> z;
  const uint8_t* body = data;
  size_t blen = len;
  const char* filter = nullptr;
  if (kind == kJpeg) {
    filter = "DCTDecode";
    const int c = jpeg_components(data, len);
    components = c ? c : 3;  // pdf_writer.c:219: RGB when the header says nothing
  } else if (kind == kJp2) {
    filter = "JPXDecode";
    UphipPnmInfo info{0, 0, 0};
    if (j2k::probe(data, len, "<page>", &info)) {
      components = info.format == UPHIP_FMT_GRAY8 ? 1 : 3;
    } else {
      uphip_clear_error();
      components = 3;  // pdf_writer.c:339-341
    }
  } else if (kind == kRaw) {
    if (components != 1 && components != 3) return fail("pdf_writer: pixels must have 1 or 3 components");
    const size_t rb = (size_t)width * components;
    if (stride < (int)rb) return fail("pdf_writer: Invalid stride: %d (minimum %zu)", stride, rb);
    if (len < (size_t)stride * (height - 1) + rb) return fail("pdf_writer: pixel buffer too short");
    // packed rows, Flate-compressed (pdf_writer.c:390-419)
    std::vector<uint8_t> packed(rb * height);
    for (int y = 0; y < height; y++) memcpy(packed.data() + rb * y, data + (size_t)stride * y, rb);
    uLongf zl = compressBound((uLong)packed.size());
    z.resize(zl);
    if (compress2(z.data(), &zl, packed.data(), (uLong)packed.size(), Z_DEFAULT_COMPRESSION) != Z_OK)
      return fail("pdf_writer: zlib compression failed");
    z.resize(zl);
    body = z.data();
    blen = z.size();
    filter = "FlateDecode";
  } else {
    return fail("pdf_writer: unknown page kind %d", kind);
  }
  const char* cs = components == 1 ? "/DeviceGray" : components == 4 ? "/DeviceCMYK" : "/DeviceRGB";
  const int eff = dpi > 0 ? dpi : dpi_;
  const double pw = (double)width * 72.0 / eff, ph = (double)height * 72.0 / eff;
  const std::string spw = real(pw), sph = real(ph);
  char content[160];
  const int cl = snprintf(content, sizeof(content), "q %s 0 0 %s 0 0 cm /Im0 Do Q", spw.c_str(), sph.c_str());
  char h1[320], t1[640];
  int64_t off;
  int n1, n2;
  {
    // reserve the page's objects and bytes
    std::lock_guard<std::mutex> lk(mu_);
    if (fd_ < 0) return fail("pdf_writer: Writer has been closed or aborted");
    if (failed_) return false;
    const int64_t im = (int64_t)offsets_.size(), ct = im + 1, pg = im + 2;
    n1 = snprintf(h1, sizeof(h1),
                  "%lld 0 obj\n<< /Type /XObject /Subtype /Image /Width %d /Height %d /BitsPerComponent 8 "
                  "/ColorSpace %s /Filter /%s /Length %zu >>\nstream\n",
                  (long long)im, width, height, cs, filter, blen);
    const int a = snprintf(t1, sizeof(t1), "\nendstream\nendobj\n%lld 0 obj\n<< /Length %d >>\nstream\n%s\nendstream\nendobj\n",
                           (long long)ct, cl, content);
    const int b = snprintf(t1 + a, sizeof(t1) - (size_t)a,
                           "%lld 0 obj\n<< /Type /Page /Parent 2 0 R /MediaBox [0 0 %s %s] /Resources << /XObject "
                           "<< /Im0 %lld 0 R >> >> /Contents %lld 0 R >>\nendobj\n",
                           (long long)pg, spw.c_str(), sph.c_str(), (long long)im, (long long)ct);
    n2 = a + b;
    off = pos_;
    // object offsets: the image at off, the content after the image's
    // "endstream endobj" (18 bytes), the page after the content object
    const int64_t ct_at = off + n1 + (int64_t)blen + 18;
    const int64_t pg_at = off + n1 + (int64_t)blen + a;
    offsets_.push_back(off);
    offsets_.push_back(ct_at);
    offsets_.push_back(pg_at);
    pos_ += n1 + (int64_t)blen + n2;
    pages_.emplace_back(index, pg);
    inflight_.fetch_add(1, std::memory_order_acq_rel);
  }
  struct iovec v[3] = {{h1, (size_t)n1}, {const_cast<uint8_t*>(body), blen}, {t1, (size_t)n2}};
  const bool ok = pwrite_all(fd_, v, 3, off);
  if (!ok) failed_ = true;
  inflight_.fetch_sub(1, std::memory_order_acq_rel);
  return ok || fail("pdf_writer: cannot write %s", part_.c_str());
}

bool Writer::add_page_next(int kind, const uint8_t* data, size_t len, int width, int height, int stride,
                           int components, int dpi) {
  int64_t idx;
  {
    std::lock_guard<std::mutex> lk(mu_);
    idx = next_index_++;
  }
  return add_page(idx, kind, data, len, width, height, stride, components, dpi);
}

int Writer::page_count() {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)pages_.size();
}

bool Writer::close() {
  std::lock_guard<std::mutex> lk(mu_);
  if (fd_ < 0) return fail("pdf_writer: Writer has been closed or aborted");
  drain();
  bool ok = !failed_;
  std::stable_sort(pages_.begin(), pages_.end());
  // page tree
  offsets_[2] = pos_;
  ok = ok && putf("2 0 obj\n<< /Type /Pages /Count %zu /Kids [", pages_.size());
  for (size_t k = 0; ok && k < pages_.size(); k++) ok = putf(k ? " %lld 0 R" : "%lld 0 R", (long long)pages_[k].second);
  ok = ok && putf("] >>\nendobj\n");
  offsets_[1] = pos_;
  ok = ok && putf("1 0 obj\n<< /Type /Catalog /Pages 2 0 R >>\nendobj\n");
  // the input's metadata, Producer "unpaper" (pdf_writer.c:37-82)
  offsets_[3] = pos_;
  std::string info = "3 0 obj\n<<";
  if (has_meta_) {
    const std::string* f[8] = {&meta_.title,   &meta_.author,   &meta_.subject,       &meta_.keywords,
                               &meta_.creator, &meta_.producer, &meta_.creation_date, &meta_.modification_date};
    const char* keys[8] = {"Title", "Author", "Subject", "Keywords", "Creator", "Producer", "CreationDate", "ModDate"};
    for (int k = 0; k < 8; k++) {
      if (k == 5 || !meta_.has[k]) continue;
      info += " /";
      info += keys[k];
      info += " ";
      info += pdf_text(*f[k]);
    }
  }
  info += " /Producer (unpaper) >>\nendobj\n";
  ok = ok && put(info.data(), info.size());
  // the cross-reference table in one write
  const int64_t xref = pos_;
  std::string x;
  x.reserve(offsets_.size() * 20 + 128);
  char line[64];
  snprintf(line, sizeof(line), "xref\n0 %zu\n0000000000 65535 f\r\n", offsets_.size());
  x += line;
  for (size_t k = 1; k < offsets_.size(); k++) {
    snprintf(line, sizeof(line), "%010lld 00000 n\r\n", (long long)offsets_[k]);
    x += line;
  }
  snprintf(line, sizeof(line), "trailer\n<< /Size %zu /Root 1 0 R /Info 3 0 R >>\n", offsets_.size());
  x += line;
  snprintf(line, sizeof(line), "startxref\n%lld\n%%%%EOF\n", (long long)xref);
  x += line;
  ok = ok && put(x.data(), x.size());
  ok = (::close(fd_) == 0) && ok;
  fd_ = -1;
  if (ok && rename(part_.c_str(), path_.c_str()) != 0) ok = fail("pdf_writer: cannot rename %s", part_.c_str());
  if (!ok) {
    unlink(part_.c_str());
    return fail("pdf_writer: Failed to save PDF %s", path_.c_str());
  }
  return true;
}

void Writer::abort() {
  std::lock_guard<std::mutex> lk(mu_);
  if (fd_ < 0) return;
  drain();
  ::close(fd_);
  fd_ = -1;
  unlink(part_.c_str());
}

}  // namespace pdf
}  // namespace uph

// ---------------------------------------------------------------------------
// C ABI (include/unpaper_hip.h, the pdf/pdf_reader.h + pdf/pdf_writer.h peer)
// ---------------------------------------------------------------------------

struct UphipPdfDocument {
  uph::pdf::Document doc;
};
struct UphipPdfWriter {
  uph::pdf::Writer w;
};

namespace uph {
namespace pdf {

// The page's image and its pixel geometry (uphip_pdf_page_probe).
bool page_geometry(Document& doc, int page, int32_t dpi, PageImage* im, UphipPnmInfo* info) {
  if (!doc.extract_image(page, im)) return false;
  if (dpi > 0) {  // pdf_pipeline_decode.c:69-111
    PageBox box;
    if (!doc.page_box(page, &box)) return false;
    float wpt = box.width, hpt = box.height;
    int rot = box.rotation % 360;
    if (rot < 0) rot += 360;
    if (rot == 90 || rot == 270) std::swap(wpt, hpt);
    const int ew = (int)lroundf(wpt * (float)dpi / 72.0f), eh = (int)lroundf(hpt * (float)dpi / 72.0f);
    if (ew > 0 && eh > 0 && (std::abs(im->width - ew) > 4 || std::abs(im->height - eh) > 4))
      return fail("pdf: %s: page %d: its image is %dx%d but the page is %dx%d at %d dpi "
                  "(the reference renders such pages; rendering is not supported here -- dpi 0 takes the image)",
                  doc.name().c_str(), page, im->width, im->height, ew, eh, (int)dpi);
  }
  char name[64];
  snprintf(name, sizeof(name), "page %d", page);
  UphipPnmInfo g{0, 0, 0};
  if (im->format == kJpeg) {
    if (!jpeg_probe_mem(im->data.data(), im->data.size(), name, &g)) return false;
  } else if (im->format == kJp2) {
    if (!j2k::probe(im->data.data(), im->data.size(), name, &g)) return false;
  } else if (im->format == kCcitt) {
    g = UphipPnmInfo{im->width, im->height, UPHIP_FMT_GRAY8};
  } else if (im->format == kJbig2) {
    int32_t w = 0, h = 0;
    if (!jbig2::probe(im->data.data(), im->data.size(), &w, &h, name)) return false;
    g = UphipPnmInfo{w, h ? h : im->height, UPHIP_FMT_GRAY8};
  } else if (im->format == kFlate || im->format == kPng || im->format == kRaw) {
    const int fmt = pixel_format(*im);
    if (fmt < 0)
      return fail("pdf: %s: page %d: image has %d components at %d bits%s (not supported)", doc.name().c_str(),
                  page, im->components, im->bpc, im->indexed ? ", indexed colours" : "");
    g = UphipPnmInfo{im->width, im->height, fmt};
  } else {
    return fail("pdf: %s: page %d: images of unknown format are not supported", doc.name().c_str(), page);
  }
  if (g.width != im->width || g.height != im->height)
    return fail("pdf: %s: page %d: the image stream is %dx%d, its dictionary says %dx%d", doc.name().c_str(),
                page, g.width, g.height, im->width, im->height);
  *info = g;
  return true;
}

}  // namespace pdf
}  // namespace uph

extern "C" {

using uph::fail;

UphipPdfDocument* uphip_pdf_open(const char* path) {
  if (!path) return fail("pdf_open: NULL path"), nullptr;
  std::vector<uint8_t> bytes;
  if (!uph::jpeg_read_file(path, &bytes)) return nullptr;
  UphipPdfDocument* d = new UphipPdfDocument();
  if (!d->doc.open(std::move(bytes), path)) {
    delete d;
    return nullptr;
  }
  return d;
}

UphipPdfDocument* uphip_pdf_open_memory(const uint8_t* data, size_t size) {
  if (!data || !size) return fail("pdf_open_memory: Invalid data"), nullptr;
  UphipPdfDocument* d = new UphipPdfDocument();
  if (!d->doc.open_view(data, size, "<memory>")) {
    delete d;
    return nullptr;
  }
  return d;
}

void uphip_pdf_close(UphipPdfDocument* doc) { delete doc; }

int uphip_pdf_page_count(UphipPdfDocument* doc) { return doc ? doc->doc.page_count() : -1; }

int uphip_pdf_needs_password(UphipPdfDocument* doc) { return doc && doc->doc.encrypted() ? 1 : 0; }

int uphip_pdf_get_page_info(UphipPdfDocument* doc, int page, UphipPdfPageInfo* info) {
  if (!doc || !info) return fail("pdf_get_page_info: Invalid arguments"), -1;
  uph::pdf::PageBox b;
  if (!doc->doc.page_box(page, &b)) return -1;
  info->width = b.width;
  info->height = b.height;
  info->rotation = b.rotation;
  return 0;
}

int uphip_pdf_extract_page_image(UphipPdfDocument* doc, int page, UphipPdfImage* image) {
  if (!doc || !image) return fail("pdf_extract_page_image: Invalid arguments"), -1;
  memset(image, 0, sizeof(*image));
  uph::pdf::PageImage im;
  if (!doc->doc.extract_image(page, &im)) return -1;
  if (im.data.empty()) return fail("pdf: page %d: Empty buffer", page), -1;
  image->data = (uint8_t*)malloc(im.data.size());
  if (!image->data) return fail("pdf: Out of memory"), -1;
  memcpy(image->data, im.data.data(), im.data.size());
  image->size = im.data.size();
  if (!im.globals.empty()) {
    image->jbig2_globals = (uint8_t*)malloc(im.globals.size());
    if (image->jbig2_globals) {
      memcpy(image->jbig2_globals, im.globals.data(), im.globals.size());
      image->jbig2_globals_size = im.globals.size();
    }
  }
  image->width = im.width;
  image->height = im.height;
  image->components = im.components;
  image->bits_per_component = im.bpc;
  image->format = im.format;
  image->is_mask = im.mask;
  return 0;
}

void uphip_pdf_free_image(UphipPdfImage* image) {
  if (!image) return;
  free(image->data);
  free(image->jbig2_globals);
  memset(image, 0, sizeof(*image));
}

int uphip_pdf_get_metadata(UphipPdfDocument* doc, UphipPdfMetadata* meta) {
  if (!meta) return fail("pdf_get_metadata: Invalid arguments"), -1;
  memset(meta, 0, sizeof(*meta));
  if (!doc) return fail("pdf_get_metadata: Invalid arguments"), -1;
  uph::pdf::Meta m;
  if (!doc->doc.metadata(&m)) return -1;
  const std::string* f[8] = {&m.title,   &m.author,   &m.subject,       &m.keywords,
                             &m.creator, &m.producer, &m.creation_date, &m.modification_date};
  char** o[8] = {&meta->title,   &meta->author,   &meta->subject,       &meta->keywords,
                 &meta->creator, &meta->producer, &meta->creation_date, &meta->modification_date};
  for (int k = 0; k < 8; k++)
    if (m.has[k]) *o[k] = strdup(f[k]->c_str());
  return 0;
}

void uphip_pdf_free_metadata(UphipPdfMetadata* meta) {
  if (!meta) return;
  char** o[8] = {&meta->title,   &meta->author,   &meta->subject,       &meta->keywords,
                 &meta->creator, &meta->producer, &meta->creation_date, &meta->modification_date};
  for (int k = 0; k < 8; k++) {
    free(*o[k]);
    *o[k] = nullptr;
  }
}

const char* uphip_pdf_image_format_name(int32_t format) {
  switch (format) {
    case UPHIP_PDF_IMAGE_JPEG: return "JPEG";
    case UPHIP_PDF_IMAGE_JP2: return "JPEG2000";
    case UPHIP_PDF_IMAGE_JBIG2: return "JBIG2";
    case UPHIP_PDF_IMAGE_CCITT: return "CCITT";
    case UPHIP_PDF_IMAGE_PNG: return "PNG";
    case UPHIP_PDF_IMAGE_RAW: return "RAW";
    case UPHIP_PDF_IMAGE_FLATE: return "FLATE";
    default: return "UNKNOWN";
  }
}

int uphip_pdf_is_pdf_file(const char* filename) {
  if (!filename) return 0;
  const size_t n = strlen(filename);
  return n >= 4 && strcasecmp(filename + n - 4, ".pdf") == 0;
}

int uphip_pdf_page_probe(UphipPdfDocument* doc, int page, int32_t dpi, UphipPnmInfo* info) {
  if (!doc || !info) return fail("pdf_page_probe: Invalid arguments"), -1;
  uph::pdf::PageImage im;
  return uph::pdf::page_geometry(doc->doc, page, dpi, &im, info) ? 0 : -1;
}

int uphip_pdf_read_page(UphipPdfDocument* doc, int page, int32_t dpi, void* dst, int64_t linesize,
                        const UphipPnmInfo* expect) {
  if (!doc || !dst) return fail("pdf_read_page: Invalid arguments"), -1;
  uph::pdf::PageImage im;
  UphipPnmInfo g{0, 0, 0};
  if (!uph::pdf::page_geometry(doc->doc, page, dpi, &im, &g)) return -1;
  if (expect && (expect->width != g.width || expect->height != g.height || expect->format != g.format))
    return fail("pdf: %s page %d is %dx%d format %d, expected %dx%d format %d", doc->doc.name().c_str(), page,
                g.width, g.height, g.format, expect->width, expect->height, expect->format),
           -1;
  const int64_t rb = uph::row_bytes(g.width, g.format);
  if (linesize < rb) return fail("pdf_read_page: linesize too small"), -1;
  if (im.format != uph::pdf::kJpeg && im.format != uph::pdf::kJp2)
    return uph::pdf::decode_pixels(im, (uint8_t*)dst, linesize, doc->doc.name().c_str()) ? 0 : -1;
  if (!uph::runtime_ready()) return fail("pdf_read_page: no HIP device (JPEG / JPEG 2000 decode on the device)"), -1;
  const int64_t dpitch = uph::round_pitch(rb);
  void* dd = nullptr;
  if (!UPH_HIP(hipMalloc(&dd, (size_t)(dpitch * g.height)))) return -1;
  UphipPnmInfo in = g;
  const int rc = im.format == uph::pdf::kJpeg ? uphip_jpeg_decode(im.data.data(), im.data.size(), dd, dpitch, &in)
                                              : uphip_jp2_decode(im.data.data(), im.data.size(), dd, dpitch, &in);
  const bool ok = rc == 0 && UPH_HIP(hipMemcpy2D(dst, (size_t)linesize, dd, (size_t)dpitch, (size_t)rb,
                                                 (size_t)g.height, hipMemcpyDeviceToHost));
  hipFree(dd);
  return ok ? 0 : -1;
}

UphipPdfWriter* uphip_pdf_writer_create(const char* path, const UphipPdfMetadata* meta, int32_t dpi) {
  uph::pdf::Meta m;
  if (meta) {
    const char* f[8] = {meta->title,   meta->author,   meta->subject,       meta->keywords,
                        meta->creator, meta->producer, meta->creation_date, meta->modification_date};
    std::string* o[8] = {&m.title,   &m.author,   &m.subject,       &m.keywords,
                         &m.creator, &m.producer, &m.creation_date, &m.modification_date};
    for (int k = 0; k < 8; k++)
      if (f[k]) {
        *o[k] = f[k];
        m.has[k] = true;
      }
  }
  UphipPdfWriter* w = new UphipPdfWriter();
  if (!w->w.create(path, meta ? &m : nullptr, dpi)) {
    delete w;
    return nullptr;
  }
  return w;
}

int uphip_pdf_writer_add_page_jpeg(UphipPdfWriter* w, const uint8_t* data, size_t len, int32_t width,
                                   int32_t height, int32_t dpi) {
  if (!w) return fail("pdf_writer: Invalid arguments"), -1;
  return w->w.add_page_next(uph::pdf::kJpeg, data, len, width, height, 0, 0, dpi) ? 0 : -1;
}

int uphip_pdf_writer_add_page_jp2(UphipPdfWriter* w, const uint8_t* data, size_t len, int32_t width,
                                  int32_t height, int32_t dpi) {
  if (!w) return fail("pdf_writer: Invalid arguments"), -1;
  return w->w.add_page_next(uph::pdf::kJp2, data, len, width, height, 0, 0, dpi) ? 0 : -1;
}

int uphip_pdf_writer_add_page_pixels(UphipPdfWriter* w, const uint8_t* pixels, int32_t width, int32_t height,
                                     int32_t stride, int32_t format, int32_t dpi) {
  if (!w || !pixels) return fail("pdf_writer: Invalid arguments"), -1;
  if (format != 0 && format != 1) return fail("pdf_writer: unknown pixel format %d", format), -1;
  if (width <= 0 || height <= 0) return fail("pdf_writer: Invalid dimensions: %dx%d", width, height), -1;
  const int comps = format == 0 ? 1 : 3;
  const size_t len = (size_t)stride * (size_t)(height - 1) + (size_t)width * comps;
  return w->w.add_page_next(uph::pdf::kRaw, pixels, len, width, height, stride, comps, dpi) ? 0 : -1;
}

int uphip_pdf_writer_page_count(UphipPdfWriter* w) { return w ? w->w.page_count() : 0; }

int uphip_pdf_writer_close(UphipPdfWriter* w) {
  if (!w) return 0;
  const bool ok = w->w.close();
  delete w;
  return ok ? 0 : -1;
}

void uphip_pdf_writer_abort(UphipPdfWriter* w) {
  if (!w) return;
  w->w.abort();
  delete w;
}

}  // extern "C"
