// kernels_jpeg.hip — device half of the JPEG decode peer (jpeg.h): the
// coefficients the host's Huffman decoder packed (jpeg.cpp) -> pixels in a
// page buffer (GRAY8 or RGB24 rows at any pitch, e.g. a batch input slot).
//
// k_jpeg_idct   one workgroup per group (an MCU row of a scan), 256 lanes =
//               32 blocks x 8 lanes per round: the blocks' coefficient
//               offsets by a wave prefix sum of their counts; lane j of a
//               block dequantises zigzag positions j, j+8, .. into an LDS
//               tile in natural order, then the islow IDCT (libjpeg
//               jidctint.c: LL&M, CONST_BITS 13, PASS1_BITS 2, JLONG = 64-bit
//               products) runs column j (pass 1) and row j (pass 2) of the
//               block; the row's 8 samples are one 8-byte store.  A gray
//               image is written straight into the destination (clipped);
//               colour components go to planes in device scratch.
// k_jpeg_color  one lane per output pixel: libjpeg's fancy upsampling
//               (jdsample.c h2v1/h2v2/h1v2_fancy_upsample, triangle filters
//               with the first/last sample and row replicated at the edges;
//               box replication where libjpeg uses it: downsampled width <= 2)
//               and jdcolor.c ycc_rgb_convert (16-bit fixed point tables,
//               evaluated inline).
//
// HBM: the packed coefficients (a few MB a page, mostly counts and DC terms
// on a text page) are read once; gray output written once; colour planes
// written once and read by the colour pass (1.5x or 3x the output bytes).
#include "jpeg.h"
#include "runtime.h"

namespace uph {

namespace {

constexpr int kJpegBlocksPerRound = 32;  // 256 lanes, 8 per block

// jidctint.c constants (CONST_BITS = 13)
constexpr int64_t F_0_298631336 = 2446, F_0_390180644 = 3196, F_0_541196100 = 4433,
                  F_0_765366865 = 6270, F_0_899976223 = 7373, F_1_175875602 = 9633,
                  F_1_501321110 = 12299, F_1_847759065 = 15137, F_1_961570560 = 16069,
                  F_2_053119869 = 16819, F_2_562915447 = 20995, F_3_072711026 = 25172;

// One 8-point pass of jpeg_idct_islow on in[0..7] (stride already applied).
// shift: CONST_BITS - PASS1_BITS (pass 1) or CONST_BITS + PASS1_BITS + 3
// (pass 2); results DESCALEd (round half up, arithmetic shift).
__device__ __forceinline__ void idct8(const int64_t* in, int64_t* out, int shift) {
  // even part
  int64_t z2 = in[2], z3 = in[6];
  int64_t z1 = (z2 + z3) * F_0_541196100;
  int64_t tmp2 = z1 + z3 * (-F_1_847759065);
  int64_t tmp3 = z1 + z2 * F_0_765366865;
  z2 = in[0];
  z3 = in[4];
  int64_t tmp0 = (z2 + z3) * 8192;  // LEFT_SHIFT(.., CONST_BITS)
  int64_t tmp1 = (z2 - z3) * 8192;
  const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
  const int64_t tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
  // odd part
  tmp0 = in[7];
  tmp1 = in[5];
  tmp2 = in[3];
  tmp3 = in[1];
  z1 = tmp0 + tmp3;
  z2 = tmp1 + tmp2;
  z3 = tmp0 + tmp2;
  int64_t z4 = tmp1 + tmp3;
  const int64_t z5 = (z3 + z4) * F_1_175875602;
  tmp0 = tmp0 * F_0_298631336;
  tmp1 = tmp1 * F_2_053119869;
  tmp2 = tmp2 * F_3_072711026;
  tmp3 = tmp3 * F_1_501321110;
  z1 = z1 * (-F_0_899976223);
  z2 = z2 * (-F_2_562915447);
  z3 = z3 * (-F_1_961570560);
  z4 = z4 * (-F_0_390180644);
  z3 += z5;
  z4 += z5;
  tmp0 += z1 + z3;
  tmp1 += z2 + z4;
  tmp2 += z2 + z3;
  tmp3 += z1 + z4;
  const int64_t half = (int64_t)1 << (shift - 1);
  out[0] = (tmp10 + tmp3 + half) >> shift;
  out[7] = (tmp10 - tmp3 + half) >> shift;
  out[1] = (tmp11 + tmp2 + half) >> shift;
  out[6] = (tmp11 - tmp2 + half) >> shift;
  out[2] = (tmp12 + tmp1 + half) >> shift;
  out[5] = (tmp12 - tmp1 + half) >> shift;
  out[3] = (tmp13 + tmp0 + half) >> shift;
  out[4] = (tmp13 - tmp0 + half) >> shift;
}

// jdmaster.c prepare_range_limit_table as used by the IDCT: the descaled
// value masked to 10 bits, read as signed, +128 and clamped
__device__ __forceinline__ uint32_t idct_limit(int64_t v) {
  int32_t s = (int32_t)(v & 1023);
  if (s >= 512) s -= 1024;
  s += 128;
  return (uint32_t)(s < 0 ? 0 : s > 255 ? 255 : s);
}

__device__ __forceinline__ int scan_of(const JpegHeader& h, int g) {
  int s = 0;
  for (int k = 1; k < h.nscans; k++)
    if (g >= h.scan[k].first_group) s = k;
  return s;
}

}  // namespace

template <bool kGray>
__global__ void __launch_bounds__(256) k_jpeg_idct(const JpegHeader h, const uint8_t* packed,
                                                   uint8_t* dst, int64_t dpitch,
                                                   uint8_t* scratch) {
  __shared__ int32_t tile[kJpegBlocksPerRound][64];
  __shared__ int32_t offs[kJpegBlocksPerRound];
  __shared__ int32_t total_s;
  const int g = blockIdx.x;
  const int t = threadIdx.x, b = t >> 3, j = t & 7;
  const int sc = scan_of(h, g);
  const JpegScan& S = h.scan[sc];
  const int64_t gl = g - S.first_group;               // MCU row within the scan
  const int64_t nblk = (int64_t)S.mcus_x * S.blocks_per_mcu;
  const uint8_t* counts = packed + h.counts_off + S.first_block + gl * nblk;
  const uint32_t* groups = (const uint32_t*)(packed + h.groups_off);
  const int16_t* coefs = (const int16_t*)(packed + h.coefs_off);
  int64_t carry = groups[g];
  for (int64_t base = 0; base < nblk; base += kJpegBlocksPerRound) {
    // coefficient offsets of this round's blocks (exclusive prefix of counts)
    if (t < 64) {
      const int c = (t < kJpegBlocksPerRound && base + t < nblk) ? counts[base + t] : 0;
      int pre = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(pre, o, 64);
        if (t >= o) pre += v;
      }
      if (t < kJpegBlocksPerRound) offs[t] = pre - c;
      if (t == 63) total_s = pre;
    }
    __syncthreads();
    const int64_t lb = base + b;  // block within the group
    const bool live = lb < nblk;
    // which component and block position
    int comp = S.comp[0];
    int64_t bx = 0, by = 0;
    if (live) {
      const int64_t l = gl * nblk + lb;  // block within the scan
      const int64_t mcu = l / S.blocks_per_mcu;
      int k = (int)(l - mcu * S.blocks_per_mcu);
      const int64_t mx = mcu % S.mcus_x, my = mcu / S.mcus_x;
      if (S.ncomp == 1) {
        bx = mx;
        by = my;
      } else {
        for (int i = 0; i < S.ncomp; i++) {
          const JpegComp& c = h.comp[S.comp[i]];
          const int nb = c.h * c.v;
          if (k < nb) {
            comp = S.comp[i];
            bx = mx * c.h + k % c.h;
            by = my * c.v + k / c.h;
            break;
          }
          k -= nb;
        }
      }
      // dequantise into natural order (every position written once)
      const int cnt = counts[lb];
      const int16_t* cf = coefs + carry + offs[b];
      const uint16_t* q = h.comp[comp].qzz;
      for (int z = j; z < 64; z += 8)
        tile[b][kJpegNatural[z]] = z < cnt ? (int32_t)cf[z] * (int32_t)q[z] : 0;
    }
    __syncthreads();
    if (live) {  // pass 1: column j
      int64_t in[8], out[8];
      for (int i = 0; i < 8; i++) in[i] = tile[b][i * 8 + j];
      idct8(in, out, 13 - 2);
      for (int i = 0; i < 8; i++) tile[b][i * 8 + j] = (int32_t)out[i];
    }
    __syncthreads();
    if (live) {  // pass 2: row j
      int64_t in[8], out[8];
      for (int i = 0; i < 8; i++) in[i] = tile[b][j * 8 + i];
      idct8(in, out, 13 + 2 + 3);
      uint32_t lo = 0, hi = 0;
      for (int i = 0; i < 4; i++) {
        lo |= idct_limit(out[i]) << (8 * i);
        hi |= idct_limit(out[i + 4]) << (8 * i);
      }
      const int64_t y = by * 8 + j, x0 = bx * 8;
      if (kGray) {
        if (y < h.height && x0 < h.width) {
          uint8_t* p = dst + y * dpitch + x0;
          if (x0 + 8 <= h.width && ((uintptr_t)p & 7) == 0) {
            *(uint2*)p = make_uint2(lo, hi);
          } else {
            const int n = (int)(h.width - x0 < 8 ? h.width - x0 : 8);
            for (int i = 0; i < n; i++) p[i] = (uint8_t)((i < 4 ? lo >> (8 * i) : hi >> (8 * (i - 4))));
          }
        }
      } else {
        const JpegComp& c = h.comp[comp];
        *(uint2*)(scratch + c.plane_off + y * c.pitch + x0) = make_uint2(lo, hi);
      }
    }
    if (t == 0) offs[0] = 0;  // keep the compiler from caching across the barrier
    carry += total_s;
    __syncthreads();
  }
}

namespace {

// libjpeg's upsampled sample of component c at output (x, y) (jdsample.c)
__device__ __forceinline__ int upsampled(const JpegHeader& h, const uint8_t* scratch, int c,
                                         int x, int y) {
  const JpegComp& C = h.comp[c];
  const uint8_t* P = scratch + C.plane_off;
  const int rh = h.hmax / C.h, rv = h.vmax / C.v;
  auto at = [&](int sy, int sx) -> int { return P[(int64_t)sy * C.pitch + sx]; };
  if (rh == 1 && rv == 1) return at(y, x);
  if (rh == 2 && rv == 1) {
    const int cx = x >> 1;
    if (C.dw <= 2) return at(y, cx);  // h2v1_upsample (box)
    const int v3 = 3 * at(y, cx);
    if ((x & 1) == 0) return cx == 0 ? at(y, 0) : (v3 + at(y, cx - 1) + 1) >> 2;
    return cx == C.dw - 1 ? at(y, cx) : (v3 + at(y, cx + 1) + 2) >> 2;
  }
  const int cy = y >> 1;
  if (rh == 1) {  // rv == 2: h1v2_fancy_upsample
    const int ny = (y & 1) ? (cy + 1 < C.dh ? cy + 1 : cy) : (cy > 0 ? cy - 1 : 0);
    return (3 * at(cy, x) + at(ny, x) + ((y & 1) ? 2 : 1)) >> 2;
  }
  // rh == rv == 2
  const int cx = x >> 1;
  if (C.dw <= 2) return at(cy, cx);  // h2v2_upsample (box)
  const int ny = (y & 1) ? (cy + 1 < C.dh ? cy + 1 : cy) : (cy > 0 ? cy - 1 : 0);
  auto colsum = [&](int sx) { return 3 * at(cy, sx) + at(ny, sx); };
  const int cs = colsum(cx);
  if ((x & 1) == 0) return cx == 0 ? (cs * 4 + 8) >> 4 : (cs * 3 + colsum(cx - 1) + 8) >> 4;
  return cx == C.dw - 1 ? (cs * 4 + 7) >> 4 : (cs * 3 + colsum(cx + 1) + 7) >> 4;
}

__device__ __forceinline__ uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

}  // namespace

__global__ void __launch_bounds__(256) k_jpeg_color(const JpegHeader h, const uint8_t* scratch,
                                                    uint8_t* dst, int64_t dpitch) {
  const int y = blockIdx.y;
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= h.width) return;
  const int c0 = upsampled(h, scratch, 0, x, y);
  const int c1 = upsampled(h, scratch, 1, x, y);
  const int c2 = upsampled(h, scratch, 2, x, y);
  uint8_t* p = dst + (int64_t)y * dpitch + 3 * (int64_t)x;
  if (h.color == 2) {
    p[0] = (uint8_t)c0;
    p[1] = (uint8_t)c1;
    p[2] = (uint8_t)c2;
    return;
  }
  // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert, SCALEBITS 16
  const int64_t cb = c1 - 128, cr = c2 - 128;
  const int r_off = (int)((91881 * cr + 32768) >> 16);   // FIX(1.40200)
  const int b_off = (int)((116130 * cb + 32768) >> 16);  // FIX(1.77200)
  const int g_off = (int)((-22554 * cb + 32768 + -46802 * cr) >> 16);  // FIX(0.34414), FIX(0.71414)
  p[0] = clamp255(c0 + r_off);
  p[1] = clamp255(c0 + g_off);
  p[2] = clamp255(c0 + b_off);
}

// Decodes one packed image (device copy `dpacked`, host copy of its header
// `h`) into dst (rows dpitch apart) on stream st.  scratch: h.scratch_bytes.
bool jpeg_launch(const JpegHeader& h, const uint8_t* dpacked, uint8_t* scratch, uint8_t* dst,
                 int64_t dpitch, hipStream_t st) {
  if (h.ngroups <= 0 || h.ngroups > 0x7fffffff) return fail("jpeg: bad group count");
  for (int c = 0; c < h.ncomp; c++) {
    const int rh = h.hmax / h.comp[c].h, rv = h.vmax / h.comp[c].v;
    if (h.hmax % h.comp[c].h || h.vmax % h.comp[c].v || rh > 2 || rv > 2)
      return fail("jpeg: sampling factors %dx%d of %dx%d are not supported", h.comp[c].h,
                  h.comp[c].v, h.hmax, h.vmax);
  }
  if (h.ncomp == 1) {
    hipLaunchKernelGGL(k_jpeg_idct<true>, dim3((unsigned)h.ngroups), dim3(256), 0, st, h, dpacked,
                       dst, dpitch, (uint8_t*)nullptr);
  } else {
    if (!scratch) return fail("jpeg: no scratch for the colour planes");
    hipLaunchKernelGGL(k_jpeg_idct<false>, dim3((unsigned)h.ngroups), dim3(256), 0, st, h,
                       dpacked, (uint8_t*)nullptr, (int64_t)0, scratch);
    hipLaunchKernelGGL(k_jpeg_color, dim3((h.width + 255) / 256, h.height), dim3(256), 0, st, h,
                       (const uint8_t*)scratch, dst, dpitch);
  }
  return UPH_HIP(hipGetLastError());
}

}  // namespace uph
