// kernels_jpeg_huff.hip — device entropy decoding of a sequential JPEG scan
// (jpeg.h JdecHeader): the host hands over the unstuffed entropy-coded data,
// the device decodes the Huffman codes and writes the packed coefficient
// layout (per-block counts, per-MCU-row offsets, zigzag prefixes) that
// k_jpeg_idct turns into pixels.  Peer of the GPU decode in
// imageprocess/nvimgcodec.c:679-1007 (nvImageCodec / nvJPEG's GPU Huffman).
//
// The stream is cut into subsequences of kJdecSubBits bits (restart segments
// are cut separately; a segment's first subsequence starts in a known state).
// A decoder state is (bit position, block of the MCU, next zigzag index).
//   k_jdec_sync  pass 0: every macro (kJdecMacro subsequences) decodes from
//                its first bit as if a block started there, recording the
//                state at the first code boundary at or past the end of each
//                of its subsequences (their exits).  Pass t > 0: every macro
//                starts from the exit its predecessor had in pass t-1 (only
//                macros whose entry changed decode again).  A
//                decoder that starts off the true code boundaries falls into
//                step after a few codes (Huffman codes self-synchronise, and
//                an end of block realigns the block state), so exits stop
//                changing after a pass or two; a pass in which none changes
//                is the fixed point, and its exits are exact (by induction
//                from the segment starts).  Later passes see the fixed point
//                and return at once.
//   k_jdec_settle  per image: the pass that converged, or (no convergence in
//                the passes launched) the exact exits by one lane walking the
//                subsequences in order -- correct for any stream, slow only
//                for pathological ones.
//                A macro also counts, per subsequence, the blocks whose DC
//                code starts in its bits (their number, coefficients, DC
//                difference sums): the counts of a macro's last decode are
//                those of its exact entry.
//   k_jdec_scan  per image: block / coefficient offsets, DC predictors
//                (restarting at each segment), consistency checks
//   k_jdec_zero  clears the coefficient prefixes
//   k_jdec_emit  per subsequence (one lane each, kJdecMacro x the sync
//                passes' parallelism): decode again from its exact entry,
//                write counts, non-zero coefficients (absolute DCs), MCU-row
//                offsets
// Codes come from a 10-bit lookahead table in LDS (lengths 11..16 by the
// canonical maxcode walk); one 32-bit peek serves a code and its magnitude
// bits.  Every kernel takes all the images of a chunk (grid.y = image).
#include "jpeg.h"
#include "jpeg_huff_core.h"
#include "runtime.h"

namespace uph {

using namespace jdec;

namespace {

// the image's decode tables in LDS: DC tables of the scan components, then
// their AC tables
struct TabLds {
  JdecTable t[6];
};

__device__ Dec load_dec(const JdecHeader& H, TabLds* t) {
  const int ns = H.h.scan[0].ncomp;
  for (int i = 0; i < ns; i++) {
    const uint32_t* s0 = (const uint32_t*)&H.dc[H.tdc[i]];
    const uint32_t* s1 = (const uint32_t*)&H.ac[H.tac[i]];
    uint32_t* d0 = (uint32_t*)&t->t[i];
    uint32_t* d1 = (uint32_t*)&t->t[3 + i];
    for (int j = threadIdx.x; j < (int)(sizeof(JdecTable) / 4); j += blockDim.x) {
      d0[j] = s0[j];
      d1[j] = s1[j];
    }
  }
  __syncthreads();
  const uint8_t* base = (const uint8_t*)&H;
  Dec d;
  d.tab = (const JD_LDS JdecTable*)t->t;
  d.bpm = H.h.scan[0].blocks_per_mcu;
  d.bmap = block_map(H.bcomp, d.bpm);
  d.nseg = H.nseg;
  d.seg = (const JD_GLB int32_t*)(base + H.seg_off);
  d.segsub = (const JD_GLB int32_t*)(base + H.segsub_off);
  d.segmac = (const JD_GLB int32_t*)(base + H.segmac_off);
  d.data = (const JD_GLB uint32_t*)(base + H.data_off);
  return d;
}

__device__ __forceinline__ JdecScratch scratch_of(const JdecJob& J, const JdecHeader& H) {
  return carve(J.scratch, H.nsub, H.nmac);
}

}  // namespace

// Clears the pass flags of every image.  Grid: (1, images).
__global__ void k_jdec_init(const JdecJob* jobs) {
  const JdecJob J = jobs[blockIdx.y];
  const JdecHeader& H = *(const JdecHeader*)J.stream;
  const JdecScratch S = scratch_of(J, H);
  if (threadIdx.x < kSyncPasses + 2) S.changed[threadIdx.x] = 0;
}

// Sync pass `pass` (0: from the macro starts).  Grid: (macros / 256, images).
#ifndef UPH_JDEC_WAVES
// > 0: k_jdec_sync's register budget in waves a SIMD (JPEG runner A/B: 6
// waves 3,404 vs 3,399 pages/s, 8 waves 3,326: kept at the compiler's 5)
#define UPH_JDEC_WAVES 0
#endif
#if UPH_JDEC_WAVES > 0
#define UPH_JDEC_ATTR __attribute__((amdgpu_waves_per_eu(UPH_JDEC_WAVES)))
#else
#define UPH_JDEC_ATTR
#endif
__global__ void __launch_bounds__(256) UPH_JDEC_ATTR k_jdec_sync(const JdecJob* jobs, int pass) {
  const JdecJob J = jobs[blockIdx.y];
  const JdecHeader& H = *(const JdecHeader*)J.stream;
  if ((int64_t)blockIdx.x * blockDim.x >= H.nmac) return;
  const JdecScratch S = scratch_of(J, H);
  for (int p = 1; p < pass; p++)
    if (S.changed[p] == 0) return;  // converged earlier
  __shared__ TabLds tl;
  const Dec d = load_dec(H, &tl);
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m < H.nmac) sync_macro(d, S, m, pass);
}

// Which buffer holds the exact exits; without convergence, one lane walks the
// stream in order.  Grid: (1, images).
__global__ void __launch_bounds__(256) k_jdec_settle(const JdecJob* jobs) {
  const JdecJob J = jobs[blockIdx.y];
  const JdecHeader& H = *(const JdecHeader*)J.stream;
  const JdecScratch S = scratch_of(J, H);
  __shared__ TabLds tl;
  const Dec d = load_dec(H, &tl);
  if (threadIdx.x != 0) return;
  for (int p = 1; p <= kSyncPasses; p++)
    if (S.changed[p] == 0) {
      *S.final_buf = p & 1;
      return;
    }
  settle_serial(d, S, kSyncPasses & 1);
  *S.final_buf = kSyncPasses & 1;
}

namespace {

template <class T>
__device__ T scan_block(T v, T* excl, T* lds) {
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

}  // namespace

// Offsets and DC predictors.  Grid: (1, images), 1024 threads.
__global__ void __launch_bounds__(1024) k_jdec_scan(const JdecJob* jobs) {
  __shared__ long long lds[16];
  const JdecJob J = jobs[blockIdx.y];
  const JdecHeader& H = *(const JdecHeader*)J.stream;
  const JdecScratch S = scratch_of(J, H);
  const uint8_t* base = J.stream;
  const JD_GLB int32_t* segsub = (const JD_GLB int32_t*)(base + H.segsub_off);
  long long cb = 0, cc = 0, cd[3] = {0, 0, 0};
  for (int64_t b0 = 0; b0 < H.nsub; b0 += 1024) {
    const int64_t i = b0 + threadIdx.x;
    const bool live = i < H.nsub;
    long long ex;
    const long long tb = scan_block<long long>(live ? S.nblk[i] : 0, &ex, lds);
    if (live) S.blkoff[i] = cb + ex;
    cb += tb;
    const long long tc = scan_block<long long>(live ? S.ncoef[i] : 0, &ex, lds);
    if (live) S.coefoff[i] = cc + ex;
    cc += tc;
    for (int k = 0; k < 3; k++) {
      const long long td = scan_block<long long>(live ? S.dcsum[3 * i + k] : 0, &ex, lds);
      if (live) S.dcpre[3 * i + k] = (int32_t)(cd[k] + ex);
      cd[k] += td;
    }
  }
  __syncthreads();
  // predictors restart at each segment; the blocks before a segment are whole
  // restart intervals
  const int bpm = H.h.scan[0].blocks_per_mcu;
  for (int64_t i = threadIdx.x; i < H.nsub; i += 1024) {
    const int g = seg_search(segsub, H.nseg, i);
    const int64_t f = segsub[g];
    if (i == f && H.restart && S.blkoff[i] != (int64_t)g * H.restart * bpm) atomicOr(J.status, 2);
    if (i != f)
      for (int k = 0; k < 3; k++) S.dcpre[3 * i + k] -= S.dcpre[3 * f + k];
  }
  __syncthreads();
  if (H.nseg > 1)
    for (int64_t i = threadIdx.x; i < H.nsub; i += 1024)
      if (i == segsub[seg_search(segsub, H.nseg, i)])
        for (int k = 0; k < 3; k++) S.dcpre[3 * i + k] = 0;
  if (threadIdx.x == 0) {
    if (cb != H.h.nblocks) atomicOr(J.status, 4);
    ((uint32_t*)(J.packed + H.h.groups_off))[H.h.ngroups] = (uint32_t)cc;
    if (cc > 0xF0000000ll) atomicOr(J.status, 8);
  }
}

// Zeroes each image's coefficient prefixes (the write pass stores only the
// non-zero coefficients).  Grid: (blocks, images).
__global__ void __launch_bounds__(256) k_jdec_zero(const JdecJob* jobs) {
  const JdecJob J = jobs[blockIdx.y];
  const JdecHeader& H = *(const JdecHeader*)J.stream;
  const int64_t ncoef = *(const uint32_t*)(J.packed + H.h.groups_off + 4 * H.h.ngroups);
  const int64_t cap = (H.h.total_bytes - H.h.coefs_off) >> 4;
  int64_t n16 = (2 * ncoef + 15) >> 4;  // coefs_off is 16-aligned
  n16 = n16 < cap ? n16 : cap;          // (a corrupt total is caught by the scan)
  uint4* dst = (uint4*)(J.packed + H.h.coefs_off);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = make_uint4(0, 0, 0, 0);
}

// Writes counts, zigzag prefixes (absolute DCs; the zeros are in place) and
// MCU-row offsets.
__global__ void __launch_bounds__(256) k_jdec_emit(const JdecJob* jobs) {
  const JdecJob J = jobs[blockIdx.y];
  const JdecHeader& H = *(const JdecHeader*)J.stream;
  if ((int64_t)blockIdx.x * blockDim.x >= H.nsub) return;
  const JdecScratch S = scratch_of(J, H);
  __shared__ TabLds tl;
  const Dec d = load_dec(H, &tl);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H.nsub) return;
  JD_GLB uint8_t* counts = (JD_GLB uint8_t*)(J.packed + H.h.counts_off);
  JD_GLB uint32_t* groups = (JD_GLB uint32_t*)(J.packed + H.h.groups_off);
  JD_GLB int16_t* coefs = (JD_GLB int16_t*)(J.packed + H.h.coefs_off);
  int64_t blk = S.blkoff[i], co = S.coefoff[i];
  int p0 = S.dcpre[3 * i], p1 = S.dcpre[3 * i + 1], p2 = S.dcpre[3 * i + 2];
  const int64_t row_blocks = (int64_t)H.h.scan[0].mcus_x * H.h.scan[0].blocks_per_mcu;
  const int64_t nblocks = H.h.nblocks;
  int64_t next_row = (blk + row_blocks - 1) / row_blocks * row_blocks;  // next row start
  const bool ok = walk_owned(
      d, S, i,
      [&](int c, int zz, int val) {
        if (blk >= nblocks) return;
        int v = val;
        if (zz == 0) {
          if (blk == next_row) groups[blk / row_blocks] = (uint32_t)co;
          p0 += c == 0 ? val : 0;
          p1 += c == 1 ? val : 0;
          p2 += c == 2 ? val : 0;
          v = c == 0 ? p0 : c == 1 ? p1 : p2;
        }
        coefs[co + zz] = (int16_t)v;
      },
      [&](int last) {
        if (blk < nblocks) counts[blk] = (uint8_t)(last + 1);
        next_row += blk == next_row ? row_blocks : 0;
        blk++;
        co += last + 1;
      });
  if (!ok) atomicOr(J.status, 16);
}

size_t jdec_scratch_bytes(const JdecHeader& hd) {
  return scratch_bytes(hd.nsub > 0 ? hd.nsub : 1, hd.nmac > 0 ? hd.nmac : 1);
}

bool jdec_launch_batch(const JdecJob* djobs, int n, int64_t max_nsub, int64_t max_nmac,
                       hipStream_t st) {
  if (n <= 0 || n > 65535 || max_nsub <= 0 || max_nmac <= 0 || max_nsub > 0x7fffffffll)
    return fail("jpeg: bad device decode batch");
  const dim3 gm((unsigned)((max_nmac + 255) / 256), (unsigned)n);
  const dim3 gs((unsigned)((max_nsub + 255) / 256), (unsigned)n);
  hipLaunchKernelGGL(k_jdec_init, dim3(1, (unsigned)n), dim3(64), 0, st, djobs);
  for (int p = 0; p <= kSyncPasses; p++)
    hipLaunchKernelGGL(k_jdec_sync, gm, dim3(256), 0, st, djobs, p);
  hipLaunchKernelGGL(k_jdec_settle, dim3(1, (unsigned)n), dim3(256), 0, st, djobs);
  hipLaunchKernelGGL(k_jdec_scan, dim3(1, (unsigned)n), dim3(1024), 0, st, djobs);
  hipLaunchKernelGGL(k_jdec_zero, dim3(256, (unsigned)n), dim3(256), 0, st, djobs);
  hipLaunchKernelGGL(k_jdec_emit, gs, dim3(256), 0, st, djobs);
  return UPH_HIP(hipGetLastError());
}

// One image; the job record goes to the end of its scratch.
bool jdec_launch(const JdecHeader& hd, const uint8_t* dstream, uint8_t* dpacked, uint8_t* scratch,
                 int32_t* dstatus, hipStream_t st) {
  if (hd.h.nscans != 1) return fail("jpeg: device decode takes one scan");
  JdecJob* dj = (JdecJob*)(scratch + jdec_scratch_bytes(hd));
  const JdecJob j{dstream, dpacked, scratch, dstatus};
  return UPH_HIP(hipMemcpyAsync(dj, &j, sizeof(j), hipMemcpyHostToDevice, st)) &&
         UPH_HIP(hipStreamSynchronize(st)) &&  // the job record is on this frame
         jdec_launch_batch(dj, 1, hd.nsub, hd.nmac, st);
}

}  // namespace uph
