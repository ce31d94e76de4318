/*
 * jpeg_enc.c — CPU restatement of the JPEG encode the reference's GPU output
 * branch performs (TEST INFRASTRUCTURE, part of the oracle; see oracle.h).
 *
 * The reference encodes a finished device sheet with nvImageCodec
 * (src/core/sheet_stages.c:554-581 -> lib/encode_queue.c:860-990 ->
 * imageprocess/nvimgcodec.c:1007-1212, quality from --jpeg-quality,
 * src/cli/cli_options.c:1068-1071, default 85 per lib/options.h:42 and
 * nvimgcodec.c:451).  nvImageCodec is a third-party library absent here (and
 * NVIDIA-only), so its output is "parity unpinned"; what this file restates is
 * the baseline JPEG encoder of libjpeg-turbo (the IJG algorithm, T.81 Annex
 * K tables), which PIL links here: tests/test_jpeg_encode.py pins this
 * restatement byte for byte against PIL's encoder output (quality 1..100,
 * gray / 4:4:4 / 4:2:2 / 4:2:0, odd sizes), and the device encoder
 * (csrc/kernels_jpeg_enc.hip) against this restatement.
 *
 * Followed, function by function (libjpeg-turbo 2.x/3.x file names):
 *   jcparam.c   jpeg_quality_scaling, jpeg_add_quant_table, std tables (K.1)
 *   jchuff.c    jpeg_make_c_derived_tbl, encode_one_block (F.1.2)
 *   jstdhuff.c  the Annex K.3 Huffman tables
 *   jccolor.c   rgb_ycc_convert (16-bit fixed point, rounding fudge)
 *   jcsample.c  h2v1_downsample / h2v2_downsample (alternating bias),
 *               expand_right_edge
 *   jcprepct.c  expand_bottom_edge (row group and iMCU row padding)
 *   jfdctint.c  jpeg_fdct_islow (LL&M, CONST_BITS 13, PASS1_BITS 2)
 *   jcdctmgr.c  compute_reciprocal + quantize (16-bit DCTELEM, the SIMD
 *               build's arithmetic)
 *   jccoefct.c  compress_data's dummy blocks (zero AC, previous DC)
 *   jcmarker.c  SOI, APP0 JFIF 1.01, DQT, SOF0, DHT, SOS, EOI
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* jcparam.c std_luminance_quant_tbl / std_chrominance_quant_tbl (natural order) */
static const unsigned o_std_lum_q[64] = {
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const unsigned o_std_chr_q[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

/* jstdhuff.c (T.81 K.3): counts of code lengths 1..16, then the symbols */
static const uint8_t o_bits_dc_lum[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t o_bits_dc_chr[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t o_vals_dc[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t o_bits_ac_lum[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t o_vals_ac_lum[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
static const uint8_t o_bits_ac_chr[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t o_vals_ac_chr[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

/* jutils.c jpeg_natural_order: zigzag index -> natural index */
static const uint8_t o_natural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

typedef struct {
  unsigned code[256];
  uint8_t size[256];
} OHuff;

/* jchuff.c jpeg_make_c_derived_tbl: canonical codes in symbol order */
static void o_derive(OHuff *t, const uint8_t *bits, const uint8_t *vals) {
  memset(t, 0, sizeof(*t));
  unsigned code = 0;
  int k = 0;
  for (int len = 1; len <= 16; len++) {
    for (int i = 0; i < bits[len - 1]; i++, k++, code++) {
      t->code[vals[k]] = code;
      t->size[vals[k]] = (uint8_t)len;
    }
    code <<= 1;
  }
}

/* jcparam.c jpeg_quality_scaling + jpeg_add_quant_table(force_baseline) */
void o_jpeg_quant_tables(int quality, uint16_t qtab[2][64]) {
  if (quality <= 0) quality = 1;
  if (quality > 100) quality = 100;
  const long scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int t = 0; t < 2; t++)
    for (int i = 0; i < 64; i++) {
      long v = ((long)(t ? o_std_chr_q : o_std_lum_q)[i] * scale + 50L) / 100L;
      if (v <= 0) v = 1;
      if (v > 32767) v = 32767;
      if (v > 255) v = 255; /* force_baseline */
      qtab[t][i] = (uint16_t)v;
    }
}

/* jcdctmgr.c compute_reciprocal with a 16-bit DCTELEM (the SIMD build):
 * q = ((|x| + corr) * recip) >> (16 + shift) */
static void o_reciprocal(unsigned divisor, unsigned *recip, unsigned *corr, int *shift) {
  int b = 0;
  while ((1u << (b + 1)) <= divisor) b++; /* flss(divisor) - 1 */
  int r = 16 + b;
  uint32_t fq = (uint32_t)((1ull << r) / divisor);
  const uint32_t fr = (uint32_t)((1ull << r) % divisor);
  unsigned c = divisor / 2;
  if (fr == 0) {
    fq >>= 1;
    r--;
  } else if (fr <= divisor / 2u) {
    c++;
  } else {
    fq++;
  }
  *recip = fq & 0xFFFF;
  *corr = c & 0xFFFF;
  *shift = r - 16;
}

/* jfdctint.c jpeg_fdct_islow on d[64] (natural order, samples - 128) */
static void o_fdct_islow(int32_t *d) {
  enum { CB = 13, P1 = 2 };
  const int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373,
                F1175 = 9633, F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819,
                F2562 = 20995, F3072 = 25172;
#define O_DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))
  for (int pass = 0; pass < 2; pass++) {
    for (int k = 0; k < 8; k++) {
      const int st = pass ? 8 : 1; /* pass 0: rows, pass 1: columns */
      int32_t *p = pass ? d + k : d + 8 * k;
      const int32_t t0 = p[0 * st] + p[7 * st], t7 = p[0 * st] - p[7 * st];
      const int32_t t1 = p[1 * st] + p[6 * st], t6 = p[1 * st] - p[6 * st];
      const int32_t t2 = p[2 * st] + p[5 * st], t5 = p[2 * st] - p[5 * st];
      const int32_t t3 = p[3 * st] + p[4 * st], t4 = p[3 * st] - p[4 * st];
      const int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
      const int n = pass ? CB + P1 : CB - P1;
      if (pass) {
        p[0] = O_DESCALE(t10 + t11, P1);
        p[4 * st] = O_DESCALE(t10 - t11, P1);
      } else {
        p[0] = (t10 + t11) * (1 << P1);
        p[4] = (t10 - t11) * (1 << P1);
      }
      int32_t z1 = (t12 + t13) * F0541;
      p[2 * st] = O_DESCALE(z1 + t13 * F0765, n);
      p[6 * st] = O_DESCALE(z1 + t12 * -F1847, n);
      z1 = t4 + t7;
      int32_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
      const int32_t z5 = (z3 + z4) * F1175;
      const int32_t a4 = t4 * F0298, a5 = t5 * F2053, a6 = t6 * F3072, a7 = t7 * F1501;
      z1 *= -F0899;
      z2 *= -F2562;
      z3 *= -F1961;
      z4 *= -F0390;
      z3 += z5;
      z4 += z5;
      p[7 * st] = O_DESCALE(a4 + z1 + z3, n);
      p[5 * st] = O_DESCALE(a5 + z2 + z4, n);
      p[3 * st] = O_DESCALE(a6 + z2 + z3, n);
      p[1 * st] = O_DESCALE(a7 + z1 + z4, n);
    }
  }
#undef O_DESCALE
}

typedef struct {
  uint8_t *out;
  int64_t cap, n;
  uint32_t acc; /* pending bits, left-aligned count in nacc */
  int nacc;
} OBits;

static void o_byte(OBits *b, unsigned v) {
  if (b->n < b->cap) b->out[b->n] = (uint8_t)v;
  b->n++;
}

/* jchuff.c emit_bits: MSB first, 0xFF stuffed with 0x00 */
static void o_emit(OBits *b, unsigned code, int size) {
  for (int i = size - 1; i >= 0; i--) {
    b->acc = (b->acc << 1) | ((code >> i) & 1u);
    if (++b->nacc == 8) {
      o_byte(b, b->acc & 0xFF);
      if ((b->acc & 0xFF) == 0xFF) o_byte(b, 0);
      b->acc = 0;
      b->nacc = 0;
    }
  }
}

static void o_marker16(OBits *b, unsigned m, unsigned len) {
  o_byte(b, 0xFF);
  o_byte(b, m);
  o_byte(b, len >> 8);
  o_byte(b, len & 0xFF);
}

static int o_nbits(int v) {
  int n = 0;
  for (unsigned a = (unsigned)(v < 0 ? -v : v); a; a >>= 1) n++;
  return n;
}

/* jchuff.c encode_one_block */
static void o_encode_block(OBits *b, const int16_t *blk /*natural*/, int *last_dc,
                           const OHuff *dc, const OHuff *ac) {
  int diff = blk[0] - *last_dc;
  *last_dc = blk[0];
  int nb = o_nbits(diff);
  o_emit(b, dc->code[nb], dc->size[nb]);
  if (nb) o_emit(b, (unsigned)(diff < 0 ? diff - 1 : diff) & ((1u << nb) - 1u), nb);
  int r = 0;
  for (int k = 1; k < 64; k++) {
    const int v = blk[o_natural[k]];
    if (!v) {
      r++;
      continue;
    }
    while (r > 15) {
      o_emit(b, ac->code[0xF0], ac->size[0xF0]);
      r -= 16;
    }
    nb = o_nbits(v);
    o_emit(b, ac->code[(r << 4) + nb], ac->size[(r << 4) + nb]);
    o_emit(b, (unsigned)(v < 0 ? v - 1 : v) & ((1u << nb) - 1u), nb);
    r = 0;
  }
  if (r > 0) o_emit(b, ac->code[0], ac->size[0]);
}

/* the file header libjpeg writes for these parameters (jcmarker.c) */
int64_t o_jpeg_header(int w, int h, int ncomp, int sampling, int quality, uint8_t *out,
                      int64_t cap) {
  OBits b = {out, cap, 0, 0, 0};
  uint16_t q[2][64];
  o_jpeg_quant_tables(quality, q);
  o_byte(&b, 0xFF);
  o_byte(&b, 0xD8);
  /* APP0 JFIF 1.01, density 1:1 (write_jfif_app0) */
  o_marker16(&b, 0xE0, 16);
  static const uint8_t jfif[14] = {'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
  for (int i = 0; i < 14; i++) o_byte(&b, jfif[i]);
  for (int t = 0; t < (ncomp == 1 ? 1 : 2); t++) { /* emit_dqt, 8-bit */
    o_marker16(&b, 0xDB, 67);
    o_byte(&b, (unsigned)t);
    for (int i = 0; i < 64; i++) o_byte(&b, q[t][o_natural[i]]);
  }
  const int hs = sampling == 0 ? 1 : 2, vs = sampling == 2 ? 2 : 1;
  o_marker16(&b, 0xC0, (unsigned)(8 + 3 * ncomp)); /* emit_sof, baseline */
  o_byte(&b, 8);
  o_byte(&b, (unsigned)h >> 8);
  o_byte(&b, (unsigned)h & 0xFF);
  o_byte(&b, (unsigned)w >> 8);
  o_byte(&b, (unsigned)w & 0xFF);
  o_byte(&b, (unsigned)ncomp);
  for (int c = 0; c < ncomp; c++) {
    o_byte(&b, (unsigned)c + 1);
    o_byte(&b, c == 0 && ncomp == 3 ? (unsigned)(hs << 4 | vs) : 0x11);
    o_byte(&b, c == 0 ? 0 : 1);
  }
  for (int t = 0; t < (ncomp == 1 ? 1 : 2); t++) /* emit_dht: DC t, AC t */
    for (int isac = 0; isac < 2; isac++) {
      const uint8_t *bits = isac ? (t ? o_bits_ac_chr : o_bits_ac_lum) : (t ? o_bits_dc_chr : o_bits_dc_lum);
      const uint8_t *vals = isac ? (t ? o_vals_ac_chr : o_vals_ac_lum) : o_vals_dc;
      int nv = 0;
      for (int i = 0; i < 16; i++) nv += bits[i];
      o_marker16(&b, 0xC4, (unsigned)(2 + 17 + nv));
      o_byte(&b, (unsigned)(isac << 4 | t));
      for (int i = 0; i < 16; i++) o_byte(&b, bits[i]);
      for (int i = 0; i < nv; i++) o_byte(&b, vals[i]);
    }
  o_marker16(&b, 0xDA, (unsigned)(6 + 2 * ncomp)); /* emit_sos */
  o_byte(&b, (unsigned)ncomp);
  for (int c = 0; c < ncomp; c++) {
    o_byte(&b, (unsigned)c + 1);
    o_byte(&b, c == 0 ? 0x00 : 0x11);
  }
  o_byte(&b, 0);
  o_byte(&b, 63);
  o_byte(&b, 0);
  return b.n;
}

/* Encodes a GRAY8 (1 component) or RGB24 (YCbCr, sampling 0 = 4:4:4,
 * 1 = 4:2:2, 2 = 4:2:0) image as libjpeg-turbo does with its defaults and
 * jpeg_set_quality(quality, TRUE).  Returns the file size (bytes written up
 * to cap), or -1 on bad arguments. */
int64_t o_jpeg_encode(const uint8_t *src, int64_t linesize, int w, int h, int fmt,
                      int quality, int sampling, uint8_t *out, int64_t cap) {
  if (!src || w <= 0 || h <= 0 || w > 65535 || h > 65535 ||
      (fmt != UPHIP_FMT_GRAY8 && fmt != UPHIP_FMT_RGB24) || sampling < 0 || sampling > 2)
    return -1;
  const int ncomp = fmt == UPHIP_FMT_GRAY8 ? 1 : 3;
  const int hmax = ncomp == 3 && sampling ? 2 : 1, vmax = ncomp == 3 && sampling == 2 ? 2 : 1;
  OBits b = {out, cap, 0, 0, 0};
  b.n = o_jpeg_header(w, h, ncomp, sampling, quality, out, cap);
  uint16_t q[2][64];
  o_jpeg_quant_tables(quality, q);
  unsigned recip[2][64], corr[2][64];
  int shift[2][64];
  for (int t = 0; t < 2; t++)
    for (int i = 0; i < 64; i++) o_reciprocal(q[t][i] * 8u, &recip[t][i], &corr[t][i], &shift[t][i]);
  OHuff dct[2], act[2];
  o_derive(&dct[0], o_bits_dc_lum, o_vals_dc);
  o_derive(&act[0], o_bits_ac_lum, o_vals_ac_lum);
  o_derive(&dct[1], o_bits_dc_chr, o_vals_dc);
  o_derive(&act[1], o_bits_ac_chr, o_vals_ac_chr);
  /* full-resolution component planes (jccolor.c), then downsampled planes
   * padded to whole iMCU rows / blocks (jcsample.c, jcprepct.c) */
  const int mcux = (w + 8 * hmax - 1) / (8 * hmax), mcuy = (h + 8 * vmax - 1) / (8 * vmax);
  int cw[3], chh[3], wb[3], hb[3], pw[3], ph[3], hsf[3], vsf[3];
  uint8_t *plane[3] = {0, 0, 0};
  uint8_t *full = (uint8_t *)malloc((size_t)w * h * ncomp);
  if (!full) return -1;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const uint8_t *p = src + (int64_t)y * linesize + (int64_t)x * ncomp;
      if (ncomp == 1) {
        full[(int64_t)y * w + x] = p[0];
        continue;
      }
      const int64_t SC = 16, HALF = 1 << 15, OFF = (int64_t)128 << 16;
#define O_FIX(v) ((int64_t)((v) * (1L << SC) + 0.5))
      const int64_t r = p[0], g = p[1], bb = p[2];
      const int64_t Y = (O_FIX(0.29900) * r + O_FIX(0.58700) * g + O_FIX(0.11400) * bb + HALF) >> SC;
      const int64_t Cb = (-O_FIX(0.16874) * r - O_FIX(0.33126) * g + O_FIX(0.50000) * bb + OFF + HALF - 1) >> SC;
      const int64_t Cr = (O_FIX(0.50000) * r - O_FIX(0.41869) * g - O_FIX(0.08131) * bb + OFF + HALF - 1) >> SC;
#undef O_FIX
      const int64_t i = (int64_t)y * w + x;
      full[i] = (uint8_t)Y;
      full[(int64_t)w * h + i] = (uint8_t)Cb;
      full[2 * (int64_t)w * h + i] = (uint8_t)Cr;
    }
  for (int c = 0; c < ncomp; c++) {
    hsf[c] = c == 0 ? hmax : 1;
    vsf[c] = c == 0 ? vmax : 1;
    cw[c] = (w * hsf[c] + hmax - 1) / hmax;
    chh[c] = (h * vsf[c] + vmax - 1) / vmax;
    wb[c] = (cw[c] + 7) / 8;
    hb[c] = (chh[c] + 7) / 8;
    pw[c] = wb[c] * 8;
    ph[c] = mcuy * vsf[c] * 8;
    plane[c] = (uint8_t *)malloc((size_t)pw[c] * ph[c]);
    const uint8_t *f = full + (int64_t)c * w * h;
    const int rh = hmax / hsf[c], rv = vmax / vsf[c];
    for (int y = 0; y < ph[c]; y++) {
      const int yy = y < chh[c] ? y : chh[c] - 1; /* rows past the component: last row */
      for (int x = 0; x < pw[c]; x++) {
        int v;
        /* input columns past the image repeat the last one (expand_right_edge) */
#define O_IN(xx, rr) f[(int64_t)(rr) * w + ((xx) < w ? (xx) : w - 1)]
        if (rh == 1 && rv == 1) {
          v = O_IN(x, yy < h ? yy : h - 1);
        } else if (rv == 1) { /* h2v1_downsample: bias 0, 1, 0, 1 ... */
          v = (O_IN(2 * x, yy) + O_IN(2 * x + 1, yy) + (x & 1)) >> 1;
        } else { /* h2v2_downsample: bias 1, 2, 1, 2 ...; odd last row repeated */
          const int r0 = 2 * yy, r1 = 2 * yy + 1 < h ? 2 * yy + 1 : h - 1;
          v = (O_IN(2 * x, r0) + O_IN(2 * x + 1, r0) + O_IN(2 * x, r1) + O_IN(2 * x + 1, r1) +
               1 + (x & 1)) >> 2;
        }
#undef O_IN
        plane[c][(int64_t)y * pw[c] + x] = (uint8_t)v;
      }
    }
  }
  free(full);
  /* jccoefct.c compress_data: MCUs in raster order, each component's
   * hsf x vsf blocks; dummy blocks (past width_in_blocks / height_in_blocks)
   * get zero AC and the previous block's DC */
  int last_dc[3] = {0, 0, 0};
  int16_t blk[64];
  for (int my = 0; my < mcuy; my++)
    for (int mx = 0; mx < mcux; mx++)
      for (int c = 0; c < ncomp; c++) {
        const int nbx = ncomp == 1 ? 1 : hsf[c], nby = ncomp == 1 ? 1 : vsf[c];
        int prev_dc = last_dc[c];
        for (int by = 0; by < nby; by++)
          for (int bx = 0; bx < nbx; bx++) {
            const int gbx = mx * nbx + bx, gby = my * nby + by;
            memset(blk, 0, sizeof blk);
            if (gbx < wb[c] && gby < hb[c]) {
              int32_t d[64];
              for (int i = 0; i < 8; i++)
                for (int j = 0; j < 8; j++)
                  d[i * 8 + j] = (int32_t)plane[c][(int64_t)(gby * 8 + i) * pw[c] + gbx * 8 + j] - 128;
              o_fdct_islow(d);
              const int t = c ? 1 : 0;
              for (int i = 0; i < 64; i++) {
                const int32_t x = d[i];
                const uint32_t a = (uint32_t)(x < 0 ? -x : x);
                const uint32_t qv = (uint32_t)(((uint64_t)(a + corr[t][i]) * recip[t][i]) >> (16 + shift[t][i]));
                blk[i] = (int16_t)(x < 0 ? -(int32_t)qv : (int32_t)qv);
              }
            } else {
              blk[0] = (int16_t)prev_dc;
            }
            prev_dc = blk[0];
            const int t = c ? 1 : 0;
            o_encode_block(&b, blk, &last_dc[c], &dct[t], &act[t]);
          }
      }
  for (int c = 0; c < ncomp; c++) free(plane[c]);
  if (b.nacc) o_emit(&b, 0x7F, 8 - b.nacc); /* flush_bits: pad with ones */
  o_byte(&b, 0xFF);
  o_byte(&b, 0xD9);
  return b.n;
}
