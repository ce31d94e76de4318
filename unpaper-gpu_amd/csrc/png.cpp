// png.cpp — host PNG decoder: the PNG half of the reference's loadImage
// (file.c:29-131), which opens any file through FFmpeg; the reference's own
// test sources (tests/imgsrc*.png) are PNG.  The pixel formats follow what
// FFmpeg's PNG decoder hands loadImage (file.c:98-121):
//
//   gray, 1 bit               -> MONOBLACK (MSB first, 1 = white, bits as stored)
//   gray, 2/4/8 bit           -> GRAY8 (2/4-bit samples scaled by 0x55/0x11)
//   gray 8 bit + tRNS         -> Y400A (alpha 0 where the sample equals the key)
//   gray + alpha, 8 bit       -> Y400A
//   RGB, 8 bit                -> RGB24
//   palette, 1/2/4/8 bit      -> RGB24 (loadImage's PAL8 case: palette[index],
//                                indices past the PLTE entries are black)
//   anything else (16-bit samples, RGBA, RGB + tRNS) -> error, as loadImage's
//   "unsupported pixel format" (file.c:123).
//
// Adam7-interlaced files are supported.  Chunk CRCs are not checked (FFmpeg
// checks them only with -err_detect crccheck); the zlib stream's Adler-32 is.
// Non-interlaced rows are inflated and unfiltered one at a time straight into
// the caller's buffer (a pinned staging slot in the runner): no full-size
// temporary.  Output is always PNM (saveImage, file.c:260-300): no encoder.
#include <zlib.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "runtime.h"

namespace uph {
namespace {

constexpr uint8_t kSig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
constexpr int64_t kMaxSide = 1 << 20;    // as the PNM reader
constexpr int64_t kMaxRaster = 1ll << 34;
constexpr uint64_t kMaxIdat = 2ull * kMaxRaster;  // stored deflate blocks stay far below

uint32_t be32(const uint8_t* p) {
  return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

struct Png {
  int64_t w = 0, h = 0;
  int depth = 0, ctype = 0, interlace = 0;
  int fmt = UPHIP_FMT_NONE;
  int channels = 1;            // samples per pixel in the file
  int bpp = 1;                 // filter unit: bytes per complete pixel, >= 1
  uint8_t pal[256][3] = {};    // palette (zero = black past PLTE)
  int npal = 0;
  bool trns = false;
  uint16_t trns_gray = 0;
  std::vector<uint8_t> idat;   // the concatenated IDAT payload
};

int64_t file_row_bytes(const Png& p, int64_t w) {  // bytes of w pixels, unfiltered
  return (w * p.channels * p.depth + 7) / 8;
}

// Parse the chunks (header only when `full` is false).
bool parse(FILE* f, Png* p, bool full, const char* path) {
  uint8_t sig[8];
  if (fread(sig, 1, 8, f) != 8 || memcmp(sig, kSig, 8) != 0) return fail("png: %s: not a PNG file", path);
  bool have_ihdr = false, have_iend = false;
  std::vector<uint8_t> buf;
  // chunk lengths are checked against what the file holds before anything is
  // sized from them (a few crafted bytes must not allocate gigabytes)
  long file_size = -1;
  {
    const long at = ftell(f);
    if (at >= 0 && fseek(f, 0, SEEK_END) == 0) file_size = ftell(f);
    if (at < 0 || fseek(f, at, SEEK_SET) != 0) return fail("png: %s: cannot seek", path);
  }
  for (;;) {
    uint8_t hd[8];
    if (fread(hd, 1, 8, f) != 8) break;
    const uint32_t len = be32(hd);
    if (len > 0x7FFFFFFFu) return fail("png: %s: bad chunk length", path);
    const uint32_t type = be32(hd + 4);
    const bool want = type == 0x49484452u /*IHDR*/ || type == 0x504C5445u /*PLTE*/ ||
                      type == 0x74524E53u /*tRNS*/ || (full && type == 0x49444154u /*IDAT*/);
    if (!have_ihdr && type != 0x49484452u) return fail("png: %s: first chunk is not IHDR", path);
    if (file_size >= 0 && (long)len + 4 > file_size - ftell(f))
      return fail("png: %s: truncated chunk", path);
    if ((type == 0x49484452u && len != 13) || (type == 0x504C5445u && len > 768) ||
        (type == 0x74524E53u && len > 256))
      return fail("png: %s: bad chunk length", path);
    if (type == 0x49444154u && p->idat.size() + len > kMaxIdat)
      return fail("png: %s: compressed data larger than any valid raster", path);
    if (want) {
      uint8_t* dst;
      if (type == 0x49444154u) {
        const size_t at = p->idat.size();
        p->idat.resize(at + len);
        dst = p->idat.data() + at;
      } else {
        buf.resize(len);
        dst = buf.data();
      }
      if (len && fread(dst, 1, len, f) != len) return fail("png: %s: truncated chunk", path);
      if (fseek(f, 4, SEEK_CUR) != 0) return fail("png: %s: truncated chunk", path);  // CRC
    } else {
      if (type == 0x49454E44u /*IEND*/) {
        have_iend = true;
        break;
      }
      if (!full && type == 0x49444154u) break;  // the header chunks precede IDAT
      if (fseek(f, (long)len + 4, SEEK_CUR) != 0) return fail("png: %s: truncated chunk", path);
      continue;
    }
    if (type == 0x49484452u) {
      if (have_ihdr || len != 13) return fail("png: %s: bad IHDR", path);
      have_ihdr = true;
      p->w = be32(buf.data());
      p->h = be32(buf.data() + 4);
      p->depth = buf[8];
      p->ctype = buf[9];
      p->interlace = buf[12];
      if (buf[10] != 0 || buf[11] != 0 || p->interlace > 1) return fail("png: %s: bad IHDR", path);
      if (p->w <= 0 || p->h <= 0 || p->w > kMaxSide || p->h > kMaxSide ||
          3 * p->w * p->h > kMaxRaster)
        return fail("png: %s: %lldx%lld is out of range", path, (long long)p->w, (long long)p->h);
    } else if (type == 0x504C5445u) {
      if (len % 3 || len > 768) return fail("png: %s: bad PLTE", path);
      p->npal = (int)(len / 3);
      memcpy(p->pal, buf.data(), len);
    } else if (type == 0x74524E53u) {
      p->trns = true;
      if (p->ctype == 0 && len >= 2) p->trns_gray = (uint16_t)(buf[0] << 8 | buf[1]);
    }
  }
  if (!have_ihdr) return fail("png: %s: no IHDR", path);
  if (full && !have_iend && p->idat.empty()) return fail("png: %s: no image data", path);
  // the pixel format FFmpeg's decoder reports (see the header comment)
  const int d = p->depth, c = p->ctype;
  switch (c) {
    case 0:
      p->channels = 1;
      if (d == 1) p->fmt = UPHIP_FMT_MONOBLACK;
      else if (d == 2 || d == 4) p->fmt = UPHIP_FMT_GRAY8;
      else if (d == 8) p->fmt = p->trns ? UPHIP_FMT_Y400A : UPHIP_FMT_GRAY8;
      break;
    case 2:
      p->channels = 3;
      if (d == 8 && !p->trns) p->fmt = UPHIP_FMT_RGB24;
      break;
    case 3:
      p->channels = 1;
      if (d == 1 || d == 2 || d == 4 || d == 8) p->fmt = UPHIP_FMT_RGB24;
      break;
    case 4:
      p->channels = 2;
      if (d == 8) p->fmt = UPHIP_FMT_Y400A;
      break;
    case 6:
      p->channels = 4;
      break;
    default:
      return fail("png: %s: bad color type %d", path, c);
  }
  if (p->fmt == UPHIP_FMT_NONE)
    return fail("png: %s: unsupported pixel format (color type %d, %d-bit%s)", path, c, d,
                p->trns ? ", tRNS" : "");
  p->bpp = (p->channels * d + 7) / 8;
  return true;
}

// PNG filter reconstruction of one row in place (prev = the unfiltered row
// above, all zero for a pass's first row).
bool unfilter(uint8_t* row, const uint8_t* prev, int64_t n, int bpp, int type) {
  switch (type) {
    case 0:
      return true;
    case 1:
      for (int64_t i = bpp; i < n; i++) row[i] = (uint8_t)(row[i] + row[i - bpp]);
      return true;
    case 2:
      for (int64_t i = 0; i < n; i++) row[i] = (uint8_t)(row[i] + prev[i]);
      return true;
    case 3:
      for (int64_t i = 0; i < n; i++) {
        const int left = i >= bpp ? row[i - bpp] : 0;
        row[i] = (uint8_t)(row[i] + ((left + prev[i]) >> 1));
      }
      return true;
    case 4:
      for (int64_t i = 0; i < n; i++) {
        const int a = i >= bpp ? row[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
        const int pa = abs(b - c), pb = abs(a - c), pc = abs(a + b - 2 * c);
        const int pr = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
        row[i] = (uint8_t)(row[i] + pr);
      }
      return true;
    default:
      return false;
  }
}

// sample x (0-based) of an unfiltered row of `depth`-bit samples
inline int sample(const uint8_t* row, int64_t x, int depth) {
  if (depth == 8) return row[x];
  const int64_t bit = x * depth;
  return (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
}

// Convert pixels [0, n) of one unfiltered file row into the output row at
// output pixels x0, x0 + dx, ... (dx > 1 for Adam7 passes).
void emit(const Png& p, const uint8_t* src, int64_t n, uint8_t* out, int64_t x0, int64_t dx) {
  switch (p.fmt) {
    case UPHIP_FMT_MONOBLACK:
      if (dx == 1 && x0 == 0) {
        memcpy(out, src, (size_t)((n + 7) / 8));
      } else {
        for (int64_t i = 0; i < n; i++) {
          const int64_t x = x0 + i * dx;
          const uint8_t m = (uint8_t)(0x80 >> (x & 7));
          if ((src[i >> 3] >> (7 - (i & 7))) & 1) out[x >> 3] |= m;
          else out[x >> 3] &= (uint8_t)~m;
        }
      }
      return;
    case UPHIP_FMT_GRAY8: {
      const int scale = p.depth == 2 ? 0x55 : p.depth == 4 ? 0x11 : 1;
      if (p.depth == 8 && dx == 1) memcpy(out + x0, src, (size_t)n);
      else
        for (int64_t i = 0; i < n; i++) out[x0 + i * dx] = (uint8_t)(sample(src, i, p.depth) * scale);
      return;
    }
    case UPHIP_FMT_Y400A:
      for (int64_t i = 0; i < n; i++) {
        uint8_t* o = out + 2 * (x0 + i * dx);
        if (p.ctype == 4) {
          o[0] = src[2 * i];
          o[1] = src[2 * i + 1];
        } else {
          o[0] = src[i];
          o[1] = src[i] == p.trns_gray ? 0 : 255;
        }
      }
      return;
    case UPHIP_FMT_RGB24:
      if (p.ctype == 2) {
        if (dx == 1) memcpy(out + 3 * x0, src, (size_t)(3 * n));
        else
          for (int64_t i = 0; i < n; i++) memcpy(out + 3 * (x0 + i * dx), src + 3 * i, 3);
      } else {
        for (int64_t i = 0; i < n; i++) {
          const int k = sample(src, i, p.depth);
          memcpy(out + 3 * (x0 + i * dx), p.pal[k], 3);  // zero past PLTE: black
        }
      }
      return;
  }
}

struct Inflater {
  z_stream z{};
  bool open = false;
  explicit Inflater(std::vector<uint8_t>& in) {
    z.next_in = in.data();
    z.avail_in = (uInt)in.size();
    open = inflateInit(&z) == Z_OK;
  }
  ~Inflater() {
    if (open) inflateEnd(&z);
  }
  // exactly n bytes of the stream into dst
  bool read(uint8_t* dst, int64_t n) {
    while (n > 0) {
      z.next_out = dst;
      z.avail_out = (uInt)(n > (1 << 30) ? (1 << 30) : n);
      const uInt want = z.avail_out;
      const int r = inflate(&z, Z_SYNC_FLUSH);
      const int64_t got = want - z.avail_out;
      dst += got;
      n -= got;
      if (n > 0 && (r == Z_STREAM_END || (r != Z_OK && r != Z_BUF_ERROR) || got == 0)) return false;
    }
    return true;
  }
  // after the last row: the stream must end here (zlib checks the Adler-32
  // at its end), with no image data left over
  bool finish() {
    uint8_t extra;
    z.next_out = &extra;
    z.avail_out = 1;
    return inflate(&z, Z_FINISH) == Z_STREAM_END && z.avail_out == 1;
  }
};

bool decode(Png& p, uint8_t* out, int64_t linesize, const char* path) {
  if (p.idat.size() > 0xFFFFFFFFull) return fail("png: %s: image data too large", path);
  Inflater in(p.idat);
  if (!in.open) return fail("png: %s: zlib init failed", path);
  const int64_t rb = file_row_bytes(p, p.w);
  std::vector<uint8_t> rows(2 * (size_t)(rb + 1));
  uint8_t* cur = rows.data();
  uint8_t* prev = cur + rb + 1;
  if (!p.interlace) {
    memset(prev, 0, (size_t)(rb + 1));
    for (int64_t y = 0; y < p.h; y++) {
      if (!in.read(cur, rb + 1)) return fail("png: %s: truncated or corrupt image data", path);
      if (!unfilter(cur + 1, prev + 1, rb, p.bpp, cur[0])) return fail("png: %s: bad filter type", path);
      emit(p, cur + 1, p.w, out + y * linesize, 0, 1);
      std::swap(cur, prev);
    }
    return in.finish() || fail("png: %s: corrupt image data (stream end, checksum)", path);
  }
  // Adam7: seven reduced images, each row unfiltered against the pass's own
  // previous row, scattered into the output
  static const int x0s[7] = {0, 4, 0, 2, 0, 1, 0}, y0s[7] = {0, 0, 4, 0, 2, 0, 1};
  static const int dxs[7] = {8, 8, 4, 4, 2, 2, 1}, dys[7] = {8, 8, 8, 4, 4, 2, 2};
  for (int k = 0; k < 7; k++) {
    const int64_t pw = p.w > x0s[k] ? (p.w - x0s[k] + dxs[k] - 1) / dxs[k] : 0;
    const int64_t ph = p.h > y0s[k] ? (p.h - y0s[k] + dys[k] - 1) / dys[k] : 0;
    if (pw == 0 || ph == 0) continue;
    const int64_t prb = file_row_bytes(p, pw);
    memset(prev, 0, (size_t)(prb + 1));
    for (int64_t j = 0; j < ph; j++) {
      if (!in.read(cur, prb + 1)) return fail("png: %s: truncated or corrupt image data", path);
      if (!unfilter(cur + 1, prev + 1, prb, p.bpp, cur[0])) return fail("png: %s: bad filter type", path);
      emit(p, cur + 1, pw, out + (y0s[k] + j * dys[k]) * linesize, x0s[k], dxs[k]);
      std::swap(cur, prev);
    }
  }
  return in.finish() || fail("png: %s: corrupt image data (stream end, checksum)", path);
}

// the file's signature: 1 PNG, 2 JPEG (SOI + a marker), 3 JPEG 2000 (the JP2
// signature box or SOC + SIZ), 4 PDF (whole documents: uphip_source_pdf),
// 0 anything else (PNM)
int sniff(FILE* f) {
  uint8_t sig[12];
  const size_t n = fread(sig, 1, 12, f);
  rewind(f);
  static const uint8_t kJp2[12] = {0, 0, 0, 12, 0x6A, 0x50, 0x20, 0x20, 0x0D, 0x0A, 0x87, 0x0A};
  if (n >= 8 && memcmp(sig, kSig, 8) == 0) return 1;
  if (n >= 3 && sig[0] == 0xFF && sig[1] == 0xD8 && sig[2] == 0xFF) return 2;
  if ((n == 12 && memcmp(sig, kJp2, 12) == 0) ||
      (n >= 4 && sig[0] == 0xFF && sig[1] == 0x4F && sig[2] == 0xFF && sig[3] == 0x51))
    return 3;
  if (n >= 5 && memcmp(sig, "%PDF-", 5) == 0) return 4;
  return 0;
}

}  // namespace
}  // namespace uph

using namespace uph;

extern "C" {

int uphip_png_probe(const char* path, UphipPnmInfo* info) {
  if (!path || !info) return fail("png_probe: null argument"), -1;
  FILE* f = fopen(path, "rb");
  if (!f) return fail("png: cannot open %s: %s", path, strerror(errno)), -1;
  Png p;
  bool ok;
  try {
    ok = parse(f, &p, false, path);
  } catch (const std::bad_alloc&) {
    ok = fail("png: %s: out of memory", path);
  }
  fclose(f);
  if (!ok) return -1;
  info->width = (int32_t)p.w;
  info->height = (int32_t)p.h;
  info->format = p.fmt;
  return 0;
}

int uphip_png_read(const char* path, void* dst, int64_t linesize, const UphipPnmInfo* expect) {
  if (!path || !dst) return fail("png_read: null argument"), -1;
  FILE* f = fopen(path, "rb");
  if (!f) return fail("png: cannot open %s: %s", path, strerror(errno)), -1;
  Png p;
  bool ok;
  try {
    ok = parse(f, &p, true, path);
  } catch (const std::bad_alloc&) {
    ok = fail("png: %s: out of memory", path);
  }
  fclose(f);
  if (!ok) return -1;
  if (expect && (expect->width != p.w || expect->height != p.h || expect->format != p.fmt))
    return fail("png: %s is %lldx%lld format %d, expected %dx%d format %d", path, (long long)p.w,
                (long long)p.h, p.fmt, expect->width, expect->height, expect->format),
           -1;
  if (linesize < row_bytes((int32_t)p.w, p.fmt)) return fail("png_read: linesize too small"), -1;
  try {
    return decode(p, (uint8_t*)dst, linesize, path) ? 0 : -1;
  } catch (const std::bad_alloc&) {
    return fail("png: %s: out of memory", path), -1;
  }
}

// loadImage's peer over the codecs: the file's signature picks PNG, JPEG
// (entropy-decoded on the host, pixels made on the current device: jpeg.cpp),
// JPEG 2000 (j2k.cpp, likewise split) or PNM.
int uphip_image_probe(const char* path, UphipPnmInfo* info) {
  if (!path || !info) return fail("image_probe: null argument"), -1;
  FILE* f = fopen(path, "rb");
  if (!f) return fail("image: cannot open %s: %s", path, strerror(errno)), -1;
  const int kind = sniff(f);
  fclose(f);
  if (kind == 4)
    return fail("image: %s is a PDF document: read its pages with uphip_source_pdf / uphip_pdf_read_page", path),
           -1;
  return kind == 1 ? uphip_png_probe(path, info)
       : kind == 2 ? uphip_jpeg_probe(path, info)
       : kind == 3 ? uphip_jp2_probe(path, info)
                   : uphip_pnm_probe(path, info);
}

int uphip_image_read(const char* path, void* dst, int64_t linesize, const UphipPnmInfo* expect) {
  if (!path || !dst) return fail("image_read: null argument"), -1;
  FILE* f = fopen(path, "rb");
  if (!f) return fail("image: cannot open %s: %s", path, strerror(errno)), -1;
  const int kind = sniff(f);
  fclose(f);
  if (kind == 4)
    return fail("image: %s is a PDF document: read its pages with uphip_source_pdf / uphip_pdf_read_page", path),
           -1;
  return kind == 1 ? uphip_png_read(path, dst, linesize, expect)
       : kind == 2 ? uphip_jpeg_read(path, dst, linesize, expect)
       : kind == 3 ? uphip_jp2_read(path, dst, linesize, expect)
                   : uphip_pnm_read(path, dst, linesize, expect);
}

}  // extern "C"
