// jpeg_enc.cpp — host half of the JPEG encode peer (jpeg_enc.h): geometry,
// quantisation / Huffman tables, the file header, device buffers, and the
// single-image entry point uphip_jpeg_encode (nvimgcodec_encode_jpeg's peer,
// imageprocess/nvimgcodec.c:1139-1148).
//
// Tables and header follow libjpeg-turbo's compressor with its defaults and
// jpeg_set_quality(quality, force_baseline = TRUE) (jcparam.c; T.81 Annex K
// tables), so that the files equal PIL's byte for byte (tests/test_jpeg_encode.py).
#include "jpeg_enc.h"

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "runtime.h"

namespace uph {

namespace {

// T.81 K.1 (jcparam.c std_luminance_quant_tbl / std_chrominance_quant_tbl),
// natural order
constexpr uint16_t kStdQ[2][64] = {
    {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
     14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
     18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
     49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99},
    {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
     24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
     99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99}};

// T.81 K.3 (jstdhuff.c): code-length counts 1..16 and symbols
constexpr uint8_t kBitsDc[2][16] = {{0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0},
                                    {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0}};
constexpr uint8_t kBitsAc[2][16] = {{0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d},
                                    {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77}};
// AC symbols (run << 4 | size) in order of code length (K.5, K.6)
constexpr uint8_t kValsAc[2][162] = {
    {0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
     0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
     0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
     0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
     0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
     0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
     0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
     0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
     0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
     0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
     0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa},
    {0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
     0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
     0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
     0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
     0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
     0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
     0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
     0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
     0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
     0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
     0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa}};

// zigzag -> natural (jutils.c jpeg_natural_order)
constexpr uint8_t kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18,
                                  11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                                  13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43,
                                  36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                                  38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

int nvals(const uint8_t* bits) {
  int n = 0;
  for (int i = 0; i < 16; i++) n += bits[i];
  return n;
}

const uint8_t* dc_vals() {
  static const uint8_t v[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
  return v;
}

// jchuff.c jpeg_make_c_derived_tbl: canonical codes, len << 16 | code by symbol
void derive(const uint8_t* bits, const uint8_t* vals, uint32_t* tab, int ntab) {
  std::fill(tab, tab + ntab, 0u);
  uint32_t code = 0;
  int k = 0;
  for (int len = 1; len <= 16; len++) {
    for (int i = 0; i < bits[len - 1]; i++, k++, code++)
      if (vals[k] < ntab) tab[vals[k]] = (uint32_t)len << 16 | code;
    code <<= 1;
  }
}

// jcparam.c jpeg_quality_scaling + jpeg_add_quant_table(force_baseline)
void quant_tables(int quality, uint16_t q[2][64]) {
  quality = std::min(std::max(quality, 1), 100);
  const long scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int t = 0; t < 2; t++)
    for (int i = 0; i < 64; i++) {
      long v = ((long)kStdQ[t][i] * scale + 50L) / 100L;
      q[t][i] = (uint16_t)std::min(std::max(v, 1L), 255L);
    }
}

struct Out {
  uint8_t* p;
  int cap, n = 0;
  void b(int v) {
    if (n < cap) p[n] = (uint8_t)v;
    n++;
  }
  void marker(int m, int len) {
    b(0xFF);
    b(m);
    b(len >> 8);
    b(len & 0xFF);
  }
};

}  // namespace

bool jenc_geometry(int32_t w, int32_t h, int32_t fmt, int32_t sampling, JencGeom* g) {
  if (w <= 0 || h <= 0 || w > 65535 || h > 65535)
    return fail("jpeg encode: %dx%d is outside 1..65535", w, h);
  if (fmt != UPHIP_FMT_GRAY8 && fmt != UPHIP_FMT_RGB24)
    return fail("jpeg encode: format %d is neither GRAY8 nor RGB24", fmt);
  if (sampling < UPHIP_JPEG_444 || sampling > UPHIP_JPEG_420)
    return fail("jpeg encode: unknown sampling %d", sampling);
  memset(g, 0, sizeof(*g));
  g->w = w;
  g->h = h;
  g->ncomp = fmt == UPHIP_FMT_GRAY8 ? 1 : 3;
  g->mode = g->ncomp == 1 ? JENC_GRAY : sampling == UPHIP_JPEG_444 ? JENC_444
                                       : sampling == UPHIP_JPEG_422 ? JENC_422
                                                                    : JENC_420;
  const int hmax = g->mode == JENC_422 || g->mode == JENC_420 ? 2 : 1;
  const int vmax = g->mode == JENC_420 ? 2 : 1;
  g->bpm = g->mode == JENC_GRAY ? 1 : g->mode == JENC_444 ? 3 : g->mode == JENC_422 ? 4 : 6;
  g->mcux = (w + 8 * hmax - 1) / (8 * hmax);
  g->mcuy = (h + 8 * vmax - 1) / (8 * vmax);
  for (int c = 0; c < g->ncomp; c++) {  // jcmaster.c initial_setup
    const int hs = c == 0 ? hmax : 1, vs = c == 0 ? vmax : 1;
    const int cw = (w * hs + hmax - 1) / hmax;
    g->ch[c] = (h * vs + vmax - 1) / vmax;
    g->wb[c] = (cw + 7) / 8;
    g->hb[c] = (g->ch[c] + 7) / 8;
  }
  const int64_t nmcu = (int64_t)g->mcux * g->mcuy;
  g->tiles = (int32_t)((nmcu + kJencTileMcus - 1) / kJencTileMcus);
  return true;
}

void jenc_tables(int32_t quality, JencTables* t) {
  memset(t, 0, sizeof(*t));
  uint16_t q[2][64];
  quant_tables(quality, q);
  for (int k = 0; k < 2; k++)
    for (int i = 0; i < 64; i++) {
      // jcdctmgr.c compute_reciprocal, 16-bit DCTELEM; divisor = q << 3 (islow)
      const uint32_t d = (uint32_t)q[k][i] << 3;
      int b = 0;
      while ((1u << (b + 1)) <= d) b++;
      int r = 16 + b;
      uint64_t fq = (1ull << r) / d;
      const uint64_t fr = (1ull << r) % d;
      uint32_t c = d / 2;
      if (fr == 0) {
        fq >>= 1;
        r--;
      } else if (fr <= d / 2u) {
        c++;
      } else {
        fq++;
      }
      t->recip[k][i] = (uint16_t)fq;
      t->corr[k][i] = (uint16_t)c;
      t->shift[k][i] = (uint8_t)(r - 16);
    }
  for (int k = 0; k < 2; k++) {
    derive(kBitsDc[k], dc_vals(), t->dc[k], 16);
    derive(kBitsAc[k], kValsAc[k], t->ac[k], 256);
  }
}

// jcmarker.c write_file_header + write_frame_header + write_scan_header
int jenc_header(const JencGeom& g, int32_t quality, uint8_t* out, int cap) {
  Out o{out, cap};
  uint16_t q[2][64];
  quant_tables(quality, q);
  o.b(0xFF);
  o.b(0xD8);
  o.marker(0xE0, 16);  // JFIF 1.01, no density unit, 1:1
  static const uint8_t jfif[14] = {'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
  for (uint8_t v : jfif) o.b(v);
  const int ntab = g.ncomp == 1 ? 1 : 2;
  for (int t = 0; t < ntab; t++) {
    o.marker(0xDB, 67);
    o.b(t);
    for (int i = 0; i < 64; i++) o.b(q[t][kNatural[i]]);
  }
  const int hs = g.mode == JENC_422 || g.mode == JENC_420 ? 2 : 1, vs = g.mode == JENC_420 ? 2 : 1;
  o.marker(0xC0, 8 + 3 * g.ncomp);
  o.b(8);
  o.b(g.h >> 8);
  o.b(g.h & 0xFF);
  o.b(g.w >> 8);
  o.b(g.w & 0xFF);
  o.b(g.ncomp);
  for (int c = 0; c < g.ncomp; c++) {
    o.b(c + 1);
    o.b(c == 0 ? (hs << 4 | vs) : 0x11);
    o.b(c == 0 ? 0 : 1);
  }
  for (int t = 0; t < ntab; t++)
    for (int ac = 0; ac < 2; ac++) {
      const uint8_t* bits = ac ? kBitsAc[t] : kBitsDc[t];
      const uint8_t* vals = ac ? kValsAc[t] : dc_vals();
      const int nv = nvals(bits);
      o.marker(0xC4, 2 + 17 + nv);
      o.b(ac << 4 | t);
      for (int i = 0; i < 16; i++) o.b(bits[i]);
      for (int i = 0; i < nv; i++) o.b(vals[i]);
    }
  o.marker(0xDA, 6 + 2 * g.ncomp);
  o.b(g.ncomp);
  for (int c = 0; c < g.ncomp; c++) {
    o.b(c + 1);
    o.b(c == 0 ? 0x00 : 0x11);
  }
  o.b(0);
  o.b(63);
  o.b(0);
  return o.n;
}

namespace {
size_t a16(size_t v) { return (v + 15) & ~(size_t)15; }
}  // namespace

size_t jenc_meta_bytes(const JencGeom& g, int n) {
  const size_t T = (size_t)g.tiles * n;
  return a16(sizeof(JencImage) * n) + a16(4 * T) + a16(12 * T) + a16(8 * (T + n)) + a16(8 * T) +
         a16(4 * T) + a16(8 * T) + a16(16 * (size_t)n);
}

void jenc_carve(const JencGeom& g, int n, uint8_t* meta, JencBuffers* b) {
  const size_t T = (size_t)g.tiles * n;
  uint8_t* p = meta;
  auto take = [&](size_t bytes) {
    uint8_t* r = p;
    p += a16(bytes);
    return r;
  };
  b->images = (JencImage*)take(sizeof(JencImage) * n);
  b->tile_bits = (uint32_t*)take(4 * T);
  b->tile_dc = (int16_t*)take(12 * T);
  b->tile_off = (uint64_t*)take(8 * (T + n));
  b->edges = (uint32_t*)take(8 * T);
  b->tile_ff = (uint32_t*)take(4 * T);
  b->tile_out = (uint64_t*)take(8 * T);
  b->sizes = (int64_t*)take(16 * (size_t)n);
  b->offs = b->sizes + n;
}

// ---------------------------------------------------------------------------
// JencContext: the device buffers of one encoder (a batch's, or a thread's
// for uphip_jpeg_encode), grown on demand and reused.
// ---------------------------------------------------------------------------
JencContext::~JencContext() { release(); }

void JencContext::release() {
  if (device >= 0) hipSetDevice(device);
  for (void* p : {(void*)tables, (void*)header, (void*)meta, (void*)bits, (void*)out})
    if (p) hipFree(p);
  if (host_sizes) hipHostFree(host_sizes);
  tables = nullptr;
  header = meta = out = nullptr;
  bits = nullptr;
  host_sizes = nullptr;
  meta_cap = bits_cap = out_cap = 0;
  sizes_cap = 0;
  quality = -1;
}

bool JencContext::setup(int32_t w, int32_t h, int32_t fmt, int32_t sampling, int32_t q, int nimg,
                        int64_t cap_words, int64_t out_bytes, hipStream_t st) {
  JencGeom ng;
  if (!jenc_geometry(w, h, fmt, sampling, &ng)) return false;
  if (q < 1 || q > 100) return fail("jpeg encode: quality %d outside 1..100", q);
  device = current_device();
  const size_t meta_need = jenc_meta_bytes(ng, nimg);
  const size_t bits_need = (size_t)cap_words * 4 * nimg;
  const bool grow = meta_need > meta_cap || bits_need > bits_cap || (size_t)out_bytes > out_cap ||
                    nimg > sizes_cap || !tables;
  const bool retab = q != quality || ng.w != g.w || ng.h != g.h || ng.mode != g.mode;
  if (grow || retab) {
    // the stream's earlier encodes are the only readers of the old buffers
    if (!UPH_HIP(hipStreamSynchronize(st))) return false;
  }
  auto regrow = [](auto** p, size_t* cap, size_t need) -> bool {
    if (need <= *cap && *p) return true;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (!UPH_HIP(hipMalloc((void**)p, std::max<size_t>(need, 256)))) return false;
    *cap = std::max<size_t>(need, 256);
    return true;
  };
  if (!regrow(&meta, &meta_cap, meta_need) || !regrow(&bits, &bits_cap, bits_need) ||
      !regrow(&out, &out_cap, (size_t)out_bytes))
    return false;
  if (!tables) {
    if (!UPH_HIP(hipMalloc((void**)&tables, sizeof(JencTables))) ||
        !UPH_HIP(hipMalloc((void**)&header, 1024)))
      return false;
  }
  if (nimg > sizes_cap) {
    if (host_sizes) hipHostFree(host_sizes);
    host_sizes = nullptr;
    sizes_cap = 0;
    if (!UPH_HIP(hipHostMalloc((void**)&host_sizes, 16 * (size_t)nimg, hipHostMallocDefault)))
      return false;
    sizes_cap = nimg;
  }
  if (retab) {
    JencTables ht;
    jenc_tables(q, &ht);
    uint8_t hdr[1024];
    const int hb = jenc_header(ng, q, hdr, (int)sizeof(hdr));
    if (hb > (int)sizeof(hdr)) return fail("jpeg encode: header too long");
    ng.header_bytes = hb;
    if (!UPH_HIP(hipMemcpy(tables, &ht, sizeof(ht), hipMemcpyHostToDevice)) ||
        !UPH_HIP(hipMemcpy(header, hdr, (size_t)hb, hipMemcpyHostToDevice)))
      return false;
    quality = q;
  } else {
    ng.header_bytes = g.header_bytes;
  }
  ng.cap_words = cap_words;
  ng.out_cap = out_bytes;
  g = ng;
  n = nimg;
  B = JencBuffers{};
  jenc_carve(g, n, meta, &B);
  B.bits = bits;
  B.out = out;
  B.header = header;
  B.tables = tables;
  return true;
}

bool JencContext::encode_async(hipStream_t st) {
  return jenc_launch(g, B, n, st) &&
         UPH_HIP(hipMemcpyAsync(host_sizes, B.sizes, 16 * (size_t)n, hipMemcpyDeviceToHost, st));
}

}  // namespace uph

using namespace uph;

extern "C" {

int64_t uphip_jpeg_encode(const void* device_src, int64_t pitch, int32_t width, int32_t height,
                          int32_t format, int32_t quality, int32_t sampling, void* out,
                          int64_t capacity) {
  if (!device_src) return fail("jpeg_encode: null source"), -1;
  if (!runtime_ready()) return fail("jpeg_encode: no HIP device"), -1;
  if (quality == 0) quality = UPHIP_JPEG_DEFAULT_QUALITY;
  const int bpp = format == UPHIP_FMT_RGB24 ? 3 : 1;
  if (pitch < (int64_t)width * bpp) return fail("jpeg_encode: pitch too small"), -1;
  // one context per thread and device (uphip_jpeg_encode is synchronous)
  static thread_local JencContext* ctx[64] = {};
  const int dev = current_device();
  if (dev < 0 || dev >= 64) return fail("jpeg_encode: device %d out of range", dev), -1;
  if (!ctx[dev]) ctx[dev] = new JencContext();
  JencContext& c = *ctx[dev];
  hipStream_t st = current_stream();
  // bit buffer: the raw pixel bytes (+64 KiB) suffice for any quality short
  // of noise at q > 95; an overflow re-runs with the exact size
  int64_t cap_words = ((int64_t)width * height * bpp + (64 << 10)) / 4;
  for (int attempt = 0; attempt < 2; attempt++) {
    const int64_t out_bytes = cap_words * 4 * 2 + 4096;  // stuffing at most doubles
    if (!c.setup(width, height, format, sampling, quality, 1, cap_words, out_bytes, st)) return -1;
    const JencImage im{(const uint8_t*)device_src, pitch};
    if (!UPH_HIP(hipMemcpyAsync(c.B.images, &im, sizeof(im), hipMemcpyHostToDevice, st)) ||
        !c.encode_async(st) || !UPH_HIP(hipStreamSynchronize(st)))
      return -1;
    const int64_t size = c.host_sizes[0];
    if (size == -1) {  // bit stream larger than guessed: its exact length
      uint64_t total = 0;
      if (!UPH_HIP(hipMemcpy(&total, c.B.tile_off + c.g.tiles, 8, hipMemcpyDeviceToHost))) return -1;
      cap_words = (int64_t)(total / 32) + 16;
      continue;
    }
    if (size < 0) return fail("jpeg_encode: output buffer overflow"), -1;
    if (out && capacity >= size &&
        !UPH_HIP(hipMemcpy(out, c.out + c.host_sizes[1], (size_t)size, hipMemcpyDeviceToHost)))
      return -1;
    return size;
  }
  return fail("jpeg_encode: bit stream overflow"), -1;
}

}  // extern "C"
