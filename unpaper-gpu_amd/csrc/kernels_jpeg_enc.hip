// kernels_jpeg_enc.hip — device half of the JPEG encode peer (jpeg_enc.h):
// a batch of same-geometry images (a batch's finished sheets) -> baseline
// JPEG file images packed one after another, libjpeg-turbo's bytes exactly.
//
// Work decomposition: a tile is 256 MCUs of one image, one workgroup of 256
// lanes; it walks its MCUs in 8 rounds of 32, 8 lanes per MCU.  Lane j of an
// MCU's group produces row j of every block of the MCU (colour conversion
// and chroma downsampling in registers), runs the row pass of the islow DCT,
// and, after an LDS transpose, the column pass of column j; the quantised
// coefficients go to LDS in zigzag order, where lane j takes zigzag
// positions 8j..8j+7 of each block for the Huffman stage: its nonzero
// coefficients' run lengths come from a prefix-max of the last nonzero index
// over the 8 lanes.  Lane 0 codes the DC difference (the predictor runs
// through the MCUs of the round via LDS, across rounds in registers and
// across tiles through pass B's scan), lane 7 the end of block.
//
// Reference arithmetic (the libjpeg-turbo files named): jccolor.c
// rgb_ycc_convert, jcsample.c h2v1/h2v2_downsample + expand_right_edge,
// jcprepct.c expand_bottom_edge, jfdctint.c jpeg_fdct_islow, jcdctmgr.c
// quantize (reciprocal with correction), jccoefct.c compress_data (dummy
// blocks: zero AC, the previous block's DC), jchuff.c encode_one_block
// (F.1.2.1-2) and flush_bits (pad with ones).
//
// HBM per image: the sheet read twice (passes A and C), the bit stream
// written once and read twice (passes D, F), the file written once, a few
// words per tile.  A text page's stream is a few % of its pixels.
#include "jpeg_enc.h"
#include "runtime.h"

namespace uph {

namespace {

// natural index -> zigzag position (inverse of jpeg_natural_order)
__constant__ uint8_t kZig[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                 3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

template <int M>
struct JMode;
template <>
struct JMode<JENC_GRAY> {
  static constexpr int NB = 1;
};
template <>
struct JMode<JENC_444> {
  static constexpr int NB = 3;
};
template <>
struct JMode<JENC_422> {
  static constexpr int NB = 4;
};
template <>
struct JMode<JENC_420> {
  static constexpr int NB = 6;
};

// component of block b of an MCU (blocks in T.81 order: each component's
// h x v blocks row-major, Y first)
template <int M>
__device__ __forceinline__ constexpr int comp_of(int b) {
  return M == JENC_GRAY ? 0 : M == JENC_444 ? b : M == JENC_422 ? (b < 2 ? 0 : b - 1) : (b < 4 ? 0 : b - 3);
}
template <int M>
__device__ __forceinline__ constexpr bool first_of_comp(int b) {
  return b == 0 || comp_of<M>(b) != comp_of<M>(b - 1);
}

// jfdctint.c jpeg_fdct_islow, one 8-point pass (rows: kCol false, outputs
// scaled by 2^PASS1_BITS; columns: kCol true, PASS1_BITS removed)
template <bool kCol>
__device__ __forceinline__ void fdct8(const int32_t* in, int32_t* out) {
  constexpr int n = kCol ? 15 : 11;  // CONST_BITS +/- PASS1_BITS
  constexpr int32_t half = 1 << (n - 1);
  const int32_t t0 = in[0] + in[7], t7 = in[0] - in[7];
  const int32_t t1 = in[1] + in[6], t6 = in[1] - in[6];
  const int32_t t2 = in[2] + in[5], t5 = in[2] - in[5];
  const int32_t t3 = in[3] + in[4], t4 = in[3] - in[4];
  const int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
  if (kCol) {
    out[0] = (t10 + t11 + 2) >> 2;
    out[4] = (t10 - t11 + 2) >> 2;
  } else {
    out[0] = (t10 + t11) * 4;
    out[4] = (t10 - t11) * 4;
  }
  const int32_t z1 = (t12 + t13) * 4433;
  out[2] = (z1 + t13 * 6270 + half) >> n;
  out[6] = (z1 + t12 * -15137 + half) >> n;
  int32_t a1 = t4 + t7, a2 = t5 + t6, a3 = t4 + t6, a4 = t5 + t7;
  const int32_t z5 = (a3 + a4) * 9633;
  const int32_t b4 = t4 * 2446, b5 = t5 * 16819, b6 = t6 * 25172, b7 = t7 * 12299;
  a1 *= -7373;
  a2 *= -20995;
  a3 = a3 * -16069 + z5;
  a4 = a4 * -3196 + z5;
  out[7] = (b4 + a1 + a3 + half) >> n;
  out[5] = (b5 + a2 + a4 + half) >> n;
  out[3] = (b6 + a2 + a3 + half) >> n;
  out[1] = (b7 + a1 + a4 + half) >> n;
}

// jcdctmgr.c quantize: ((|x| + corr) * recip) >> (16 + shift), sign restored
__device__ __forceinline__ int32_t quant(int32_t x, const JencTables& T, int t, int i) {
  const uint32_t a = (uint32_t)(x < 0 ? -x : x);
  const uint32_t q = ((a + T.corr[t][i]) * (uint32_t)T.recip[t][i]) >> (16 + T.shift[t][i]);
  return x < 0 ? -(int32_t)q : (int32_t)q;
}

__device__ __forceinline__ int nbits(int32_t v) {
  const uint32_t a = (uint32_t)(v < 0 ? -v : v);
  return a ? 32 - __clz(a) : 0;
}

// jccolor.c rgb_ycc_convert (SCALEBITS 16, FIX(x) = x * 65536 + 0.5)
__device__ __forceinline__ void ycc(int r, int g, int b, int* y, int* cb, int* cr) {
  *y = (19595 * r + 38470 * g + 7471 * b + 32768) >> 16;
  *cb = (-11059 * r - 21709 * g + 32768 * b + (128 << 16) + 32767) >> 16;
  *cr = (32768 * r - 27439 * g - 5329 * b + (128 << 16) + 32767) >> 16;
}

// the three components of pixel (x, y) of an RGB24 image, x clamped to the
// last column (expand_right_edge replicates it before downsampling)
__device__ __forceinline__ void px_ycc(const uint8_t* row, int x, int w, int* y, int* cb, int* cr) {
  const uint8_t* p = row + 3 * (int64_t)(x < w ? x : w - 1);
  ycc(p[0], p[1], p[2], y, cb, cr);
}

// Row j of every block of MCU (mx, my), samples - 128, into s[NB][8].
template <int M>
__device__ __forceinline__ void mcu_rows(const JencGeom& G, const JencImage& I, int mx, int my,
                                         int j, int32_t (*s)[8]) {
  const int w = G.w, h = G.h;
  if (M == JENC_GRAY) {
    const int y = min(my * 8 + j, h - 1);
    const uint8_t* row = I.src + (int64_t)y * I.pitch;
    const int x0 = mx * 8;
    if (x0 + 8 <= w && (((uintptr_t)(row + x0)) & 7) == 0) {
      const uint2 v = *(const uint2*)(row + x0);
      for (int k = 0; k < 4; k++) {
        s[0][k] = (int32_t)((v.x >> (8 * k)) & 0xFF) - 128;
        s[0][k + 4] = (int32_t)((v.y >> (8 * k)) & 0xFF) - 128;
      }
    } else {
      for (int k = 0; k < 8; k++) s[0][k] = (int32_t)row[min(x0 + k, w - 1)] - 128;
    }
  } else if (M == JENC_444) {
    const int y = min(my * 8 + j, h - 1);
    const uint8_t* row = I.src + (int64_t)y * I.pitch;
    for (int k = 0; k < 8; k++) {
      int Y, Cb, Cr;
      px_ycc(row, mx * 8 + k, w, &Y, &Cb, &Cr);
      s[0][k] = Y - 128;
      s[1][k] = Cb - 128;
      s[2][k] = Cr - 128;
    }
  } else if (M == JENC_422) {
    const int y = min(my * 8 + j, h - 1);
    const uint8_t* row = I.src + (int64_t)y * I.pitch;
    for (int k = 0; k < 8; k++) {
      int Y0, Cb0, Cr0, Y1, Cb1, Cr1;
      px_ycc(row, mx * 16 + 2 * k, w, &Y0, &Cb0, &Cr0);
      px_ycc(row, mx * 16 + 2 * k + 1, w, &Y1, &Cb1, &Cr1);
      s[(2 * k) >> 3][(2 * k) & 7] = Y0 - 128;
      s[(2 * k + 1) >> 3][(2 * k + 1) & 7] = Y1 - 128;
      // h2v1_downsample: bias 0, 1, 0, 1, ... along the output row
      s[2][k] = ((Cb0 + Cb1 + (k & 1)) >> 1) - 128;
      s[3][k] = ((Cr0 + Cr1 + (k & 1)) >> 1) - 128;
    }
  } else {  // 4:2:0
    for (int half = 0; half < 2; half++) {  // Y blocks 0,1 (rows j) and 2,3 (rows 8 + j)
      const int y = min(my * 16 + 8 * half + j, h - 1);
      const uint8_t* row = I.src + (int64_t)y * I.pitch;
      for (int k = 0; k < 16; k++) {
        const uint8_t* p = row + 3 * (int64_t)min(mx * 16 + k, w - 1);
        s[2 * half + (k >> 3)][k & 7] = ((19595 * p[0] + 38470 * p[1] + 7471 * p[2] + 32768) >> 16) - 128;
      }
    }
    // chroma row my*8 + j from input rows 2cy, 2cy+1 (the last row repeated
    // for an odd height; rows past the component repeat its last row)
    const int cy = min(my * 8 + j, G.ch[1] - 1);
    const int r0 = 2 * cy, r1 = min(r0 + 1, h - 1);
    const uint8_t* row0 = I.src + (int64_t)r0 * I.pitch;
    const uint8_t* row1 = I.src + (int64_t)r1 * I.pitch;
    for (int k = 0; k < 8; k++) {
      int Y, a0, a1, b0, b1, c0, c1, d0, d1;
      px_ycc(row0, mx * 16 + 2 * k, w, &Y, &a0, &a1);
      px_ycc(row0, mx * 16 + 2 * k + 1, w, &Y, &b0, &b1);
      px_ycc(row1, mx * 16 + 2 * k, w, &Y, &c0, &c1);
      px_ycc(row1, mx * 16 + 2 * k + 1, w, &Y, &d0, &d1);
      // h2v2_downsample: bias 1, 2, 1, 2, ...
      s[4][k] = ((a0 + b0 + c0 + d0 + 1 + (k & 1)) >> 2) - 128;
      s[5][k] = ((a1 + b1 + c1 + d1 + 1 + (k & 1)) >> 2) - 128;
    }
  }
}

// A Y block of a 4:2:x MCU past width_in_blocks / height_in_blocks is a
// dummy block (jccoefct.c compress_data): zero AC, the previous block's DC
template <int M>
__device__ __forceinline__ bool dummy_block(const JencGeom& G, int mx, int my, int b) {
  if (M != JENC_422 && M != JENC_420) return false;
  if (comp_of<M>(b) != 0) return false;
  const int bx = mx * 2 + (b & 1), by = M == JENC_420 ? my * 2 + (b >> 1) : my;
  return bx >= G.wb[0] || by >= G.hb[0];
}

__device__ __forceinline__ uint32_t piece_len(uint32_t e) { return e >> 16; }

// OR n bits (value v) at stream bit p into the LDS window of words
// [base, base + kJencWinWords)
__device__ __forceinline__ void win_or(uint32_t* win, int64_t base, uint64_t p, uint32_t v, int n) {
  const int64_t w0 = (int64_t)(p >> 5);
  const int o = (int)(p & 31);
  if (o + n <= 32) {
    const int64_t i = w0 - base;
    if (i >= 0 && i < kJencWinWords) atomicOr(&win[i], v << (32 - o - n));
  } else {
    const int k = o + n - 32;  // bits in the next word
    const int64_t i = w0 - base;
    if (i >= 0 && i < kJencWinWords) atomicOr(&win[i], v >> k);
    if (i + 1 >= 0 && i + 1 < kJencWinWords) atomicOr(&win[i + 1], v << (32 - k));
  }
}

// The pieces lane j codes for one block, in stream order: the DC difference
// (lane 0), each nonzero AC coefficient of zigzag positions 8j..8j+7 with the
// ZRL codes before it, the end of block (lane 7).  put(value, length).
template <class F>
__device__ __forceinline__ void walk_block(int j, const int32_t* q, uint32_t mask, int prev,
                                           bool eob, int dc_diff, bool dc_on, const JencTables& T,
                                           int t, F&& put) {
  if (j == 0 && dc_on) {
    const int nb = nbits(dc_diff);
    const uint32_t e = T.dc[t][nb];
    const uint32_t mag = (uint32_t)(dc_diff < 0 ? dc_diff - 1 : dc_diff) & ((1u << nb) - 1u);
    put(((e & 0xFFFF) << nb) | mag, (int)piece_len(e) + nb);
  }
  while (mask) {
    const int k = __ffs(mask) - 1;
    mask &= mask - 1;
    const int z = 8 * j + k;
    int r = z - prev - 1;
    prev = z;
    while (r > 15) {
      const uint32_t e = T.ac[t][0xF0];
      put(e & 0xFFFF, (int)piece_len(e));
      r -= 16;
    }
    const int32_t v = q[k];
    const int nb = nbits(v);
    const uint32_t e = T.ac[t][(r << 4) + nb];
    const uint32_t mag = (uint32_t)(v < 0 ? v - 1 : v) & ((1u << nb) - 1u);
    put(((e & 0xFFFF) << nb) | mag, (int)piece_len(e) + nb);
  }
  if (j == 7 && eob) {
    const uint32_t e = T.ac[t][0];
    put(e & 0xFFFF, (int)piece_len(e));
  }
}

}  // namespace

// Passes A (kEmit false) and C (kEmit true), grid (tiles, images).
template <int M, bool kEmit>
__global__ void __launch_bounds__(256) k_jenc_tile(const JencGeom G, const JencBuffers B) {
  constexpr int NB = JMode<M>::NB;
  __shared__ __attribute__((aligned(16))) int16_t tile[kJencRoundMcus][NB][64];
  __shared__ uint32_t win[kEmit ? kJencWinWords : 1];
  __shared__ int16_t mfirst[kJencRoundMcus][3], mlast[kJencRoundMcus][3];
  __shared__ uint32_t gsum[kJencRoundMcus];
  __shared__ uint32_t edge_s[2];
  __shared__ uint32_t red[4];
  const int img = blockIdx.y, t = blockIdx.x;
  const int tid = threadIdx.x, g = tid >> 3, j = tid & 7;
  if (kEmit && B.sizes[img] < 0) return;  // bit buffer overflow (pass B)
  const JencTables& T = *B.tables;
  const JencImage I = B.images[img];
  const int64_t nmcu = (int64_t)G.mcux * G.mcuy;
  const int64_t tb = (int64_t)img * G.tiles + t;
  // DC predictors entering the round, per component
  int carry[3] = {0, 0, 0};
  uint64_t pos = 0, tile_end = 0;
  int64_t fw = 0, lw = 0, base_word = 0;
  if (kEmit) {
    const uint64_t* off = B.tile_off + (int64_t)img * (G.tiles + 1);
    pos = off[t];
    tile_end = off[t + 1];
    fw = (int64_t)(pos >> 5);
    lw = (int64_t)((tile_end - 1) >> 5);
    base_word = fw;
    if (t > 0)
      for (int c = 0; c < G.ncomp; c++) carry[c] = B.tile_dc[(tb - 1) * 6 + 3 + c];
    for (int i = tid; i < kJencWinWords; i += 256) win[i] = 0;
    if (tid < 2) edge_s[tid] = 0;
  }
  uint32_t* bits = B.bits + (int64_t)img * G.cap_words;
  uint32_t lane_bits = 0;  // pass A
  auto route = [&](int64_t w, uint32_t v) {  // a finished word of this tile
    if (w == fw) edge_s[0] = v;
    else if (w == lw) edge_s[1] = v;
    else bits[w] = v;
  };
  for (int r = 0; r < kJencTileRounds; r++) {
    const int64_t m0 = (int64_t)t * kJencTileMcus + (int64_t)r * kJencRoundMcus;
    if (m0 >= nmcu) break;
    const int64_t m = m0 + g;
    const bool live = m < nmcu;
    const int ng = (int)min((int64_t)kJencRoundMcus, nmcu - m0);
    const int mx = live ? (int)(m % G.mcux) : 0, my = live ? (int)(m / G.mcux) : 0;
    // rows: colour, downsampling, row pass of the DCT (uniform blocks skip it)
    bool uni[NB], dum[NB];
    int32_t uval[NB];
    {
      int32_t s[NB][8];
      if (live) mcu_rows<M>(G, I, mx, my, j, s);
      for (int b = 0; b < NB; b++) {
        dum[b] = live && dummy_block<M>(G, mx, my, b);
        int32_t lo = s[b][0], hi = s[b][0];
        for (int k = 1; k < 8; k++) {
          lo = min(lo, s[b][k]);
          hi = max(hi, s[b][k]);
        }
        for (int o = 1; o < 8; o <<= 1) {
          lo = min(lo, __shfl_xor(lo, o, 8));
          hi = max(hi, __shfl_xor(hi, o, 8));
        }
        uni[b] = !live || dum[b] || lo == hi;
        uval[b] = lo;
        if (!uni[b]) {
          int32_t o8[8];
          fdct8<false>(s[b], o8);
          short4 a = make_short4((short)o8[0], (short)o8[1], (short)o8[2], (short)o8[3]);
          short4 c = make_short4((short)o8[4], (short)o8[5], (short)o8[6], (short)o8[7]);
          *(short4*)&tile[g][b][8 * j] = a;
          *(short4*)&tile[g][b][8 * j + 4] = c;
        }
      }
    }
    __syncthreads();
    // columns: column pass, quantisation
    int32_t qv[NB][8];
    for (int b = 0; b < NB; b++) {
      const int tq = comp_of<M>(b) ? 1 : 0;
      if (uni[b]) {
        // a uniform block's islow output is 64 * (v - 128) at DC, 0 elsewhere
        for (int i = 0; i < 8; i++) qv[b][i] = 0;
        if (j == 0 && live && !dum[b]) qv[b][0] = quant(64 * uval[b], T, tq, 0);
      } else {
        int32_t c[8], o8[8];
        for (int i = 0; i < 8; i++) c[i] = tile[g][b][8 * i + j];
        fdct8<true>(c, o8);
        for (int i = 0; i < 8; i++) qv[b][i] = quant(o8[i], T, tq, 8 * i + j);
      }
    }
    __syncthreads();
    for (int b = 0; b < NB; b++)
      for (int i = 0; i < 8; i++) tile[g][b][kZig[8 * i + j]] = (int16_t)qv[b][i];
    __syncthreads();
    // DC values of the MCU (dummies take the previous block's), per component
    // first and last, for the predictors of the next MCU
    int dcs[NB];
    if (j == 0 && live) {
      for (int b = 0; b < NB; b++) dcs[b] = dum[b] ? dcs[b > 0 ? b - 1 : 0] : tile[g][b][0];
      for (int b = 0; b < NB; b++) {
        const int c = comp_of<M>(b);
        if (first_of_comp<M>(b)) mfirst[g][c] = (int16_t)dcs[b];
        mlast[g][c] = (int16_t)dcs[b];
      }
    }
    __syncthreads();
    // per block: this lane's coefficients, run-length context, bit count
    uint32_t nlane[NB];
    int32_t q[NB][8];
    uint32_t mask[NB];
    int prev[NB];
    bool eob[NB];
    int diff[NB];
    bool dc_on[NB];
    for (int b = 0; b < NB; b++) {
      const int c = comp_of<M>(b);
      const short4 a = *(const short4*)&tile[g][b][8 * j];
      const short4 e = *(const short4*)&tile[g][b][8 * j + 4];
      q[b][0] = a.x, q[b][1] = a.y, q[b][2] = a.z, q[b][3] = a.w;
      q[b][4] = e.x, q[b][5] = e.y, q[b][6] = e.z, q[b][7] = e.w;
      uint32_t mk = 0;
      for (int k = 0; k < 8; k++) mk |= (q[b][k] != 0 ? 1u : 0u) << k;
      if (j == 0) mk &= ~1u;  // zigzag 0 is the DC
      if (!live) mk = 0;
      mask[b] = mk;
      int incl = mk ? 8 * j + 31 - __clz(mk) : -1;
      for (int o = 1; o < 8; o <<= 1) {
        const int v = __shfl_up(incl, o, 8);
        if (j >= o) incl = max(incl, v);
      }
      int excl = __shfl_up(incl, 1, 8);
      if (j == 0) excl = -1;
      prev[b] = max(excl, 0);
      eob[b] = incl != 63;
      // DC difference from the previous block of the component
      int pred = 0;
      dc_on[b] = live;
      if (j == 0 && live) {
        if (!first_of_comp<M>(b)) {
          pred = dcs[b - 1];
        } else if (g > 0) {
          pred = mlast[g - 1][c];
        } else if (r > 0 || kEmit) {
          pred = carry[c];
        } else {
          dc_on[b] = false;  // the tile's first block of the component: pass B
        }
        diff[b] = dcs[b] - pred;
      } else {
        diff[b] = 0;
      }
      uint32_t n = 0;
      if (live)
        walk_block(j, q[b], mask[b], prev[b], eob[b], diff[b], dc_on[b], T, c ? 1 : 0,
                   [&](uint32_t, int len) { n += (uint32_t)len; });
      nlane[b] = n;
    }
    // the predictors leaving the round (the last live MCU's last DCs)
    int nc[3];
    for (int c = 0; c < 3; c++) nc[c] = c < G.ncomp ? mlast[ng - 1][c] : 0;
    if (!kEmit) {
      if (r == 0 && tid == 0)
        for (int c = 0; c < G.ncomp; c++) B.tile_dc[tb * 6 + c] = mfirst[0][c];
      for (int b = 0; b < NB; b++) lane_bits += nlane[b];
      for (int c = 0; c < 3; c++) carry[c] = nc[c];
      __syncthreads();  // mfirst / mlast / tile reused by the next round
      continue;
    }
    // pass C: exact offsets.  Order: MCU g, block b, lane j.
    uint32_t lane_off[NB];
    uint32_t gtot = 0;
    for (int b = 0; b < NB; b++) {
      uint32_t incl = nlane[b];
      for (int o = 1; o < 8; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 8);
        if (j >= o) incl += v;
      }
      lane_off[b] = gtot + incl - nlane[b];
      gtot += __shfl(incl, 7, 8);
    }
    if (j == 0) gsum[g] = gtot;
    __syncthreads();
    uint32_t goff = 0, rtot = 0;
    for (int k = 0; k < kJencRoundMcus; k++) {
      const uint32_t v = gsum[k];
      goff += k < g ? v : 0;
      rtot += v;
    }
    const uint64_t re = pos + rtot;
    for (;;) {
      for (int b = 0; b < NB; b++) {
        if (!live) break;
        uint64_t p = pos + goff + lane_off[b];
        walk_block(j, q[b], mask[b], prev[b], eob[b], diff[b], dc_on[b], T,
                   comp_of<M>(b) ? 1 : 0, [&](uint32_t v, int len) {
                     win_or(win, base_word, p, v, len);
                     p += (uint64_t)len;
                   });
      }
      __syncthreads();
      const int64_t cend = (int64_t)(re >> 5);  // words below are complete
      const int64_t wend = base_word + kJencWinWords;
      const int64_t fend = min(wend, cend);
      for (int64_t w = base_word + tid; w < fend; w += 256) route(w, win[w - base_word]);
      const bool done = wend > (int64_t)((re - 1) >> 5);
      uint32_t pend = 0;
      if (done && (re & 31)) pend = win[cend - base_word];
      const int64_t used = min((int64_t)kJencWinWords, (done ? cend : wend) - base_word + 1);
      __syncthreads();
      for (int64_t i = tid; i < used; i += 256) win[i] = 0;
      __syncthreads();
      if (done) {
        if (tid == 0) win[0] = pend;
        base_word = cend;
        break;
      }
      base_word = wend;
    }
    pos = re;
    for (int c = 0; c < 3; c++) carry[c] = nc[c];
    __syncthreads();
  }
  if (!kEmit) {
    // tile bit count, last DCs
    uint32_t v = lane_bits;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    if (tid == 0) {
      B.tile_bits[tb] = red[0] + red[1] + red[2] + red[3];
      for (int c = 0; c < G.ncomp; c++) B.tile_dc[tb * 6 + 3 + c] = (int16_t)carry[c];
    }
    return;
  }
  __syncthreads();
  if (tid == 0) {
    if (tile_end & 31) route((int64_t)(tile_end >> 5), win[0]);
    B.edges[tb * 2] = edge_s[0];
    B.edges[tb * 2 + 1] = edge_s[1];
  }
}

namespace {

// workgroup exclusive scan (blockDim 1024 or 256), returns the total
template <class T>
__device__ T block_scan(T v, T* excl, T* lds /* >= 16 */) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  T incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) lds[wv] = incl;
  __syncthreads();
  T before = 0, total = 0;
  for (int k = 0; k < nw; k++) {
    const T s = lds[k];
    before += k < wv ? s : 0;
    total += s;
  }
  __syncthreads();
  *excl = before + incl - v;
  return total;
}

__device__ __forceinline__ int dc_bits(const JencTables& T, int t, int diff) {
  const int nb = nbits(diff);
  return (int)(T.dc[t][nb] >> 16) + nb;
}

}  // namespace

// Pass B: tile bit offsets per image (grid: images, 1024 threads).
__global__ void __launch_bounds__(1024) k_jenc_scan(const JencGeom G, const JencBuffers B) {
  __shared__ uint64_t lds[16];
  const int img = blockIdx.x;
  const JencTables& T = *B.tables;
  const int64_t t0 = (int64_t)img * G.tiles;
  uint64_t* off = B.tile_off + (int64_t)img * (G.tiles + 1);
  uint64_t carry = 0;
  for (int base = 0; base < G.tiles; base += 1024) {
    const int t = base + (int)threadIdx.x;
    uint64_t v = 0;
    if (t < G.tiles) {
      v = B.tile_bits[t0 + t];
      for (int c = 0; c < G.ncomp; c++) {
        const int first = B.tile_dc[(t0 + t) * 6 + c];
        const int prev = t > 0 ? B.tile_dc[(t0 + t - 1) * 6 + 3 + c] : 0;
        v += (uint64_t)dc_bits(T, c ? 1 : 0, first - prev);
      }
    }
    uint64_t ex;
    const uint64_t tot = block_scan<uint64_t>(v, &ex, lds);
    if (t < G.tiles) off[t] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) {
    off[G.tiles] = carry;
    B.sizes[img] = carry > (uint64_t)G.cap_words * 32 ? -1 : 0;
  }
}

namespace {

struct TileSpan {
  uint64_t off, end;
  int64_t fw, lw;
};

__device__ __forceinline__ TileSpan span_of(const uint64_t* off, int t) {
  TileSpan s;
  s.off = off[t];
  s.end = off[t + 1];
  s.fw = (int64_t)(s.off >> 5);
  s.lw = (int64_t)((s.end - 1) >> 5);
  return s;
}

// the final value of word w, one of tile t's first / last words: the OR of
// the contributions of the tiles that share it (at most t-1, t, t+1: every
// tile but the last holds well over 32 bits)
__device__ uint32_t shared_word(const JencGeom& G, const JencBuffers& B, int img, int t, int64_t w) {
  const uint64_t* off = B.tile_off + (int64_t)img * (G.tiles + 1);
  uint32_t v = 0;
  for (int u = max(t - 1, 0); u <= min(t + 1, G.tiles - 1); u++) {
    const TileSpan s = span_of(off, u);
    const int64_t tb = (int64_t)img * G.tiles + u;
    if (w == s.fw) v |= B.edges[tb * 2];
    if (w == s.lw && s.lw != s.fw) v |= B.edges[tb * 2 + 1];
  }
  return v;
}

__device__ __forceinline__ uint32_t stream_byte(uint32_t word, int64_t k, uint64_t total) {
  uint32_t v = (word >> (24 - 8 * (int)(k & 3))) & 0xFFu;
  // flush_bits: the last partial byte is padded with ones
  if ((uint64_t)k == ((total + 7) >> 3) - 1 && (total & 7)) v |= 0xFFu >> (total & 7);
  return v;
}

}  // namespace

// Pass D: shared words, 0xFF count per tile (grid (tiles, images), 256 threads).
__global__ void __launch_bounds__(256) k_jenc_fix(const JencGeom G, const JencBuffers B) {
  __shared__ uint32_t red[4];
  __shared__ uint32_t sw[2];
  const int img = blockIdx.y, t = blockIdx.x;
  if (B.sizes[img] < 0) return;
  const uint64_t* off = B.tile_off + (int64_t)img * (G.tiles + 1);
  const TileSpan s = span_of(off, t);
  const uint64_t total = off[G.tiles];
  uint32_t* bits = B.bits + (int64_t)img * G.cap_words;
  if (threadIdx.x == 0) {
    sw[0] = shared_word(G, B, img, t, s.fw);
    sw[1] = shared_word(G, B, img, t, s.lw);
    // each word is written by the tile holding its first bit
    if ((s.off & 31) == 0) bits[s.fw] = sw[0];
    if (s.lw != s.fw) bits[s.lw] = sw[1];
  }
  __syncthreads();
  const int64_t b0 = (int64_t)((s.off + 7) >> 3), b1 = (int64_t)((s.end + 7) >> 3);
  uint32_t ff = 0;
  for (int64_t k = b0 + threadIdx.x; k < b1; k += 256) {
    const int64_t w = k >> 2;
    const uint32_t word = w == s.fw ? sw[0] : w == s.lw ? sw[1] : bits[w];
    ff += stream_byte(word, k, total) == 0xFF;
  }
  for (int o = 32; o > 0; o >>= 1) ff += __shfl_xor(ff, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ff;
  __syncthreads();
  if (threadIdx.x == 0)
    B.tile_ff[(int64_t)img * G.tiles + t] = red[0] + red[1] + red[2] + red[3];
}

// Pass E: stuffed offsets of the tiles, file size (grid: images, 1024 threads).
__global__ void __launch_bounds__(1024) k_jenc_layout(const JencGeom G, const JencBuffers B) {
  __shared__ uint64_t lds[16];
  const int img = blockIdx.x;
  if (B.sizes[img] < 0) return;
  const uint64_t* off = B.tile_off + (int64_t)img * (G.tiles + 1);
  uint64_t carry = 0;
  for (int base = 0; base < G.tiles; base += 1024) {
    const int t = base + (int)threadIdx.x;
    uint64_t v = 0;
    if (t < G.tiles)
      v = ((off[t + 1] + 7) >> 3) - ((off[t] + 7) >> 3) + B.tile_ff[(int64_t)img * G.tiles + t];
    uint64_t ex;
    const uint64_t tot = block_scan<uint64_t>(v, &ex, lds);
    if (t < G.tiles) B.tile_out[(int64_t)img * G.tiles + t] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) B.sizes[img] = (int64_t)G.header_bytes + (int64_t)carry + 2;
}

// Image offsets in the packed output; images that do not fit are marked -2.
__global__ void k_jenc_pack(const JencGeom G, const JencBuffers B, int n) {
  if (threadIdx.x != 0) return;
  int64_t o = 0;
  for (int i = 0; i < n; i++) {
    const int64_t s = B.sizes[i];
    B.offs[i] = o;
    if (s < 0) continue;
    if (o + s > G.out_cap) {
      B.sizes[i] = -2;
      continue;
    }
    o += s;
  }
}

// Pass F: the file bytes (grid (tiles, images), 256 threads).
__global__ void __launch_bounds__(256) k_jenc_write(const JencGeom G, const JencBuffers B) {
  __shared__ uint32_t lds[16];
  const int img = blockIdx.y, t = blockIdx.x;
  const int64_t size = B.sizes[img];
  if (size < 0) return;
  uint8_t* dst = B.out + B.offs[img];
  const uint64_t* off = B.tile_off + (int64_t)img * (G.tiles + 1);
  const uint64_t total = off[G.tiles];
  const uint32_t* bits = B.bits + (int64_t)img * G.cap_words;
  if (t == 0)
    for (int i = threadIdx.x; i < G.header_bytes; i += 256) dst[i] = B.header[i];
  if (t == G.tiles - 1 && threadIdx.x == 0) {
    dst[size - 2] = 0xFF;
    dst[size - 1] = 0xD9;
  }
  const int64_t b0 = (int64_t)((off[t] + 7) >> 3), b1 = (int64_t)((off[t + 1] + 7) >> 3);
  const int64_t nb = b1 - b0;
  const int64_t per = (nb + 255) / 256;
  const int64_t k0 = b0 + min((int64_t)threadIdx.x * per, nb), k1 = min(k0 + per, b1);
  uint32_t ff = 0;
  for (int64_t k = k0; k < k1; k++) ff += stream_byte(bits[k >> 2], k, total) == 0xFF;
  uint32_t ex;
  block_scan<uint32_t>(ff, &ex, lds);
  uint8_t* o = dst + G.header_bytes + B.tile_out[(int64_t)img * G.tiles + t] + (k0 - b0) + ex;
  for (int64_t k = k0; k < k1; k++) {
    const uint32_t v = stream_byte(bits[k >> 2], k, total);
    *o++ = (uint8_t)v;
    if (v == 0xFF) *o++ = 0;
  }
}

namespace {

template <int M>
void launch_tiles(const JencGeom& g, const JencBuffers& b, int n, hipStream_t st, bool emit) {
  const dim3 grid((unsigned)g.tiles, (unsigned)n);
  if (emit)
    hipLaunchKernelGGL((k_jenc_tile<M, true>), grid, dim3(256), 0, st, g, b);
  else
    hipLaunchKernelGGL((k_jenc_tile<M, false>), grid, dim3(256), 0, st, g, b);
}

void tiles_pass(const JencGeom& g, const JencBuffers& b, int n, hipStream_t st, bool emit) {
  switch (g.mode) {
    case JENC_GRAY: launch_tiles<JENC_GRAY>(g, b, n, st, emit); break;
    case JENC_444: launch_tiles<JENC_444>(g, b, n, st, emit); break;
    case JENC_422: launch_tiles<JENC_422>(g, b, n, st, emit); break;
    default: launch_tiles<JENC_420>(g, b, n, st, emit); break;
  }
}

}  // namespace

bool jenc_launch(const JencGeom& g, const JencBuffers& b, int n, hipStream_t st) {
  if (n <= 0 || g.tiles <= 0 || n > 65535) return fail("jpeg encode: bad image count");
  const dim3 tiles((unsigned)g.tiles, (unsigned)n);
  tiles_pass(g, b, n, st, false);
  hipLaunchKernelGGL(k_jenc_scan, dim3((unsigned)n), dim3(1024), 0, st, g, b);
  tiles_pass(g, b, n, st, true);
  hipLaunchKernelGGL(k_jenc_fix, tiles, dim3(256), 0, st, g, b);
  hipLaunchKernelGGL(k_jenc_layout, dim3((unsigned)n), dim3(1024), 0, st, g, b);
  hipLaunchKernelGGL(k_jenc_pack, dim3(1), dim3(64), 0, st, g, b, n);
  hipLaunchKernelGGL(k_jenc_write, tiles, dim3(256), 0, st, g, b);
  return UPH_HIP(hipGetLastError());
}

}  // namespace uph
