// pnm.cpp — host PNM codec: the file-format half of the reference's
// loadImage/saveImage (file.c:29-259) for the formats the pipeline ships.
//
// Decode (loadImage via FFmpeg's pnm decoder, file.c:29-131): P4 -> MONOWHITE
// (1 = black, MSB first), P5 (maxval 255) -> GRAY8, P6 (maxval 255) -> RGB24;
// the plain variants P1/P2/P3 map to the same formats.  Pixels are written
// straight into the caller's buffer (a pinned staging slot in the runner), so
// decode is the only host copy on the way to the GPU.
// Encode (saveImageDirect, file.c:133-176): GRAY8 -> P5, RGB24 -> P6,
// MONOWHITE -> P4, rows written without padding.  The device pipeline already
// converted the sheet to the output format (saveImage's conversions,
// file.c:187-254, run on the GPU in the batch's output stage).
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "runtime.h"

namespace uph {
namespace {

struct Reader {
  FILE* f;
  int peekc = -2;
  int get() {
    if (peekc != -2) {
      const int c = peekc;
      peekc = -2;
      return c;
    }
    return fgetc(f);
  }
  // whitespace and '#' comments between header tokens (netpbm rules)
  int skip_ws() {
    int c = get();
    for (;;) {
      if (c == '#') {
        while (c != '\n' && c != '\r' && c != EOF) c = get();
      } else if (c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f') {
        c = get();
      } else {
        return c;
      }
    }
  }
  bool number(int64_t* v) {
    int c = skip_ws();
    if (c < '0' || c > '9') return false;
    int64_t n = 0;
    while (c >= '0' && c <= '9') {
      n = n * 10 + (c - '0');
      if (n > INT32_MAX) return false;  // widths/heights are int32_t downstream
      c = get();
    }
    peekc = c;
    *v = n;
    return true;
  }
};

// 1 M pixels a side (2.3x a 600 dpi A0 sheet), 16 GiB of RGB24 raster
constexpr int64_t kMaxSide = 1 << 20;
constexpr int64_t kMaxRaster = 1ll << 34;

struct Header {
  int kind = 0;  // 1..6
  int64_t w = 0, h = 0, maxval = 1;
};

bool read_header(Reader& r, Header* hd, const char* path) {
  if (r.get() != 'P') return fail("pnm: %s: not a PNM file", path);
  const int k = r.get();
  if (k < '1' || k > '6') return fail("pnm: %s: unsupported PNM type P%c", path, k);
  hd->kind = k - '0';
  if (!r.number(&hd->w) || !r.number(&hd->h) || hd->w <= 0 || hd->h <= 0)
    return fail("pnm: %s: bad size", path);
  // callers size staging from the probe: bound each side and the raster
  if (hd->w > kMaxSide || hd->h > kMaxSide || 3 * hd->w * hd->h > kMaxRaster)
    return fail("pnm: %s: %lldx%lld is too large", path, (long long)hd->w, (long long)hd->h);
  if (hd->kind != 1 && hd->kind != 4) {
    if (!r.number(&hd->maxval) || hd->maxval <= 0)
      return fail("pnm: %s: bad maxval", path);
    if (hd->maxval != 255)
      return fail("pnm: %s: maxval %lld unsupported (8-bit samples only)", path,
                  (long long)hd->maxval);
  }
  // raw formats: exactly one whitespace byte before the raster
  if (hd->kind >= 4) {
    const int c = r.get();
    if (!(c == ' ' || c == '\t' || c == '\n' || c == '\r')) return fail("pnm: %s: bad header", path);
  }
  return true;
}

int format_of(int kind) {
  switch (kind) {
    case 1: case 4: return UPHIP_FMT_MONOWHITE;
    case 2: case 5: return UPHIP_FMT_GRAY8;
    default: return UPHIP_FMT_RGB24;
  }
}

}  // namespace
}  // namespace uph

using namespace uph;

extern "C" {

int uphip_pnm_probe(const char* path, UphipPnmInfo* info) {
  if (!path || !info) return fail("pnm_probe: null argument"), -1;
  FILE* f = fopen(path, "rb");
  if (!f) return fail("pnm: cannot open %s: %s", path, strerror(errno)), -1;
  Reader r{f};
  Header hd;
  const bool ok = read_header(r, &hd, path);
  fclose(f);
  if (!ok) return -1;
  info->width = (int32_t)hd.w;
  info->height = (int32_t)hd.h;
  info->format = format_of(hd.kind);
  return 0;
}

int uphip_pnm_read(const char* path, void* dst, int64_t linesize, const UphipPnmInfo* expect) {
  if (!path || !dst) return fail("pnm_read: null argument"), -1;
  FILE* f = fopen(path, "rb");
  if (!f) return fail("pnm: cannot open %s: %s", path, strerror(errno)), -1;
  Reader r{f};
  Header hd;
  if (!read_header(r, &hd, path)) return fclose(f), -1;
  const int fmt = format_of(hd.kind);
  if (expect && (expect->width != hd.w || expect->height != hd.h || expect->format != fmt)) {
    fclose(f);
    return fail("pnm: %s is %lldx%lld format %d, expected %dx%d format %d", path,
                (long long)hd.w, (long long)hd.h, fmt, expect->width, expect->height,
                expect->format),
           -1;
  }
  const int64_t rb = row_bytes((int32_t)hd.w, fmt);
  if (linesize < rb) return fclose(f), fail("pnm_read: linesize too small"), -1;
  uint8_t* out = (uint8_t*)dst;
  bool ok = true;
  if (hd.kind >= 4) {
    if (r.peekc != -2) ok = false;  // cannot happen: the header ends on a consumed byte
    for (int64_t y = 0; ok && y < hd.h; y++)
      ok = fread(out + y * linesize, 1, (size_t)rb, f) == (size_t)rb;
  } else {
    for (int64_t y = 0; ok && y < hd.h; y++) {
      uint8_t* row = out + y * linesize;
      if (hd.kind == 1) memset(row, 0, (size_t)rb);
      const int64_t n = hd.kind == 3 ? hd.w * 3 : hd.w;
      for (int64_t x = 0; ok && x < n; x++) {
        int64_t v = 0;
        if (hd.kind == 1) {  // plain PBM: single digits, whitespace optional
          int c = r.skip_ws();
          if (c != '0' && c != '1') {
            ok = false;
            break;
          }
          if (c == '1') row[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
          continue;
        }
        ok = r.number(&v) && v <= 255;
        row[x] = (uint8_t)v;
      }
    }
  }
  fclose(f);
  if (!ok) return fail("pnm: %s: truncated or malformed raster", path), -1;
  return 0;
}

int uphip_pnm_write(const char* path, const void* src, int64_t linesize, int32_t width,
                    int32_t height, int32_t format) {
  if (!path || !src || width <= 0 || height <= 0) return fail("pnm_write: bad arguments"), -1;
  const char* magic = format == UPHIP_FMT_GRAY8   ? "P5"
                      : format == UPHIP_FMT_RGB24 ? "P6"
                      : format == UPHIP_FMT_MONOWHITE ? "P4"
                                                      : nullptr;
  if (!magic) return fail("pnm_write: format %d has no direct PNM encoding", format), -1;
  const int64_t rb = row_bytes(width, format);
  if (linesize < rb) return fail("pnm_write: linesize too small"), -1;
  FILE* f = fopen(path, "wb");
  if (!f) return fail("pnm: cannot create %s: %s", path, strerror(errno)), -1;
  // one buffered stream; large rows go straight through
  static thread_local std::vector<char> iobuf(1 << 20);
  setvbuf(f, iobuf.data(), _IOFBF, iobuf.size());
  bool ok = format == UPHIP_FMT_MONOWHITE ? fprintf(f, "%s\n%d %d\n", magic, width, height) > 0
                                          : fprintf(f, "%s\n%d %d\n255\n", magic, width, height) > 0;
  const uint8_t* s = (const uint8_t*)src;
  if (ok && linesize == rb)
    ok = fwrite(s, 1, (size_t)(rb * height), f) == (size_t)(rb * height);
  else
    for (int32_t y = 0; ok && y < height; y++)
      ok = fwrite(s + (int64_t)y * linesize, 1, (size_t)rb, f) == (size_t)rb;
  ok = (fclose(f) == 0) && ok;
  if (!ok) return fail("pnm: write to %s failed", path), -1;
  return 0;
}

}  // extern "C"
