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
//   k_jdec_sync  pass 0: every subsequence decodes from its first bit as if a
//                block started there, up to the first code boundary at or past
//                its end: its exit state.  Pass t > 0: every subsequence
//                starts from the exit its predecessor had in pass t-1.  A
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
//   k_jdec_count a subsequence owns the blocks whose DC code starts in it:
//                their number, coefficient count, DC difference sums
//   k_jdec_scan  per image: block / coefficient offsets, DC predictors
//                (restarting at each segment), consistency checks
//   k_jdec_emit  decode again, write counts, zigzag prefixes (absolute DCs),
//                MCU-row offsets
// Codes come from a 10-bit lookahead table (lengths 11..16 by the canonical
// maxcode walk); one 32-bit peek serves a code and its magnitude bits.
#include "jpeg.h"
#include "jpeg_huff_core.h"
#include "runtime.h"

namespace uph {

using namespace jdec;

namespace {
// the decode tables of the scan's components in LDS
struct TabLds {
  JdecTable dc[3], ac[3];
};

__device__ void load_tables(const JdecHeader& H, TabLds* t) {
  const int ns = H.h.scan[0].ncomp;
  for (int i = 0; i < ns; i++) {
    const uint32_t* s0 = (const uint32_t*)&H.dc[H.tdc[i]];
    const uint32_t* s1 = (const uint32_t*)&H.ac[H.tac[i]];
    uint32_t* d0 = (uint32_t*)&t->dc[i];
    uint32_t* d1 = (uint32_t*)&t->ac[i];
    for (int j = threadIdx.x; j < (int)(sizeof(JdecTable) / 4); j += blockDim.x) {
      d0[j] = s0[j];
      d1[j] = s1[j];
    }
  }
  __syncthreads();
}

}  // namespace

// Sync pass `pass` (0: from the subsequence starts).  Grid: ceil(nsub/256).
__global__ void __launch_bounds__(256) k_jdec_sync(const uint8_t* stream, uint8_t* scratch, int pass) {
  const Ctx c = ctx_of(stream);
  const JdecHeader& H = *c.hd;
  const JdecScratch S = carve(scratch, H.nsub);
  if (pass > 0)
    for (int p = 1; p < pass; p++)
      if (S.changed[p] == 0) return;  // converged earlier
  __shared__ TabLds tl;
  load_tables(H, &tl);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H.nsub) return;
  sync_sub(c, tl.dc, tl.ac, S, i, pass);
}

// Which buffer holds the exact exits; without convergence, one lane walks the
// subsequences in order (exact for any stream).  Grid: 1 block.
__global__ void __launch_bounds__(256) k_jdec_settle(const uint8_t* stream, uint8_t* scratch) {
  const Ctx c = ctx_of(stream);
  const JdecHeader& H = *c.hd;
  const JdecScratch S = carve(scratch, H.nsub);
  __shared__ TabLds tl;
  load_tables(H, &tl);
  if (threadIdx.x != 0) return;
  for (int p = 1; p <= kSyncPasses; p++)
    if (S.changed[p] == 0) {
      *S.final_buf = p & 1;
      return;
    }
  const int fb = kSyncPasses & 1;
  JdecState prev{0, 0};
  for (int64_t i = 0; i < H.nsub; i++) {
    const Sub s = sub_of(c, i);
    const JdecState st = s.first ? JdecState{s.start, 0} : prev;
    prev = run_to(c, tl.dc, tl.ac, st, s.stop, s.seg_end);
    S.xpos[fb][i] = prev.pos;
    S.xbk[fb][i] = prev.bk;
  }
  *S.final_buf = fb;
}

// Owned blocks, coefficients and DC difference sums per subsequence.
__global__ void __launch_bounds__(256) k_jdec_count(const uint8_t* stream, uint8_t* scratch,
                                                    int32_t* status) {
  const Ctx c = ctx_of(stream);
  const JdecHeader& H = *c.hd;
  const JdecScratch S = carve(scratch, H.nsub);
  __shared__ TabLds tl;
  load_tables(H, &tl);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H.nsub) return;
  int32_t nb = 0, dc[3] = {0, 0, 0}, diff = 0;
  int64_t nc = 0;
  const bool ok = walk_owned(
      c, tl.dc, tl.ac, S, i, [&](int, int zz, int val, int) { if (zz == 0) diff = val; },
      [&](int b, int last) {
        nb++;
        nc += last + 1;
        dc[H.bcomp[b]] += diff;
      });
  if (!ok) atomicOr(status, 1);
  S.nblk[i] = nb;
  S.ncoef[i] = nc;
  for (int k = 0; k < 3; k++) S.dcsum[3 * i + k] = dc[k];
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

// Offsets and DC predictors (grid: 1 block of 1024).
__global__ void __launch_bounds__(1024) k_jdec_scan(const uint8_t* stream, uint8_t* scratch,
                                                    uint8_t* packed, int32_t* status) {
  __shared__ long long lds[16];
  const Ctx c = ctx_of(stream);
  const JdecHeader& H = *c.hd;
  const JdecScratch S = carve(scratch, H.nsub);
  long long cb = 0, cc = 0, cd[3] = {0, 0, 0};
  for (int64_t base = 0; base < H.nsub; base += 1024) {
    const int64_t i = base + threadIdx.x;
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
    const int g = seg_of(c, i);
    const int64_t f = c.segsub[g];
    if (i == f && H.restart && S.blkoff[i] != (int64_t)g * H.restart * bpm) atomicOr(status, 2);
    if (i != f)
      for (int k = 0; k < 3; k++) S.dcpre[3 * i + k] -= S.dcpre[3 * f + k];
  }
  __syncthreads();
  if (H.nseg > 1)
    for (int64_t i = threadIdx.x; i < H.nsub; i += 1024) {
      const int64_t f = c.segsub[seg_of(c, i)];
      if (i == f)
        for (int k = 0; k < 3; k++) S.dcpre[3 * i + k] = 0;
    }
  if (threadIdx.x == 0) {
    if (cb != H.h.nblocks) atomicOr(status, 4);
    ((uint32_t*)(packed + H.h.groups_off))[H.h.ngroups] = (uint32_t)cc;
    if (cc > 0xF0000000ll) atomicOr(status, 8);
  }
}

// Writes counts, zigzag prefixes (absolute DCs) and MCU-row offsets.
__global__ void __launch_bounds__(256) k_jdec_emit(const uint8_t* stream, uint8_t* scratch,
                                                   uint8_t* packed, int32_t* status) {
  const Ctx c = ctx_of(stream);
  const JdecHeader& H = *c.hd;
  const JdecScratch S = carve(scratch, H.nsub);
  __shared__ TabLds tl;
  load_tables(H, &tl);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H.nsub) return;
  uint8_t* counts = packed + H.h.counts_off;
  uint32_t* groups = (uint32_t*)(packed + H.h.groups_off);
  int16_t* coefs = (int16_t*)(packed + H.h.coefs_off);
  int64_t blk = S.blkoff[i], co = S.coefoff[i];
  int pred[3] = {S.dcpre[3 * i], S.dcpre[3 * i + 1], S.dcpre[3 * i + 2]};
  const int64_t row_blocks = (int64_t)H.h.scan[0].mcus_x * H.h.scan[0].blocks_per_mcu;
  const int64_t nblocks = H.h.nblocks;
  const bool ok = walk_owned(
      c, tl.dc, tl.ac, S, i,
      [&](int cb, int zz, int val, int last) {
        if (blk >= nblocks) return;
        if (zz == 0) {
          if (blk % row_blocks == 0) groups[blk / row_blocks] = (uint32_t)co;
          int& p = pred[H.bcomp[cb]];
          p += val;
          coefs[co] = (int16_t)p;
          return;
        }
        for (int z = last + 1; z < zz; z++) coefs[co + z] = 0;  // the run's zeros
        coefs[co + zz] = (int16_t)val;
      },
      [&](int, int last) {
        if (blk < nblocks) counts[blk] = (uint8_t)(last + 1);
        blk++;
        co += last + 1;
      });
  if (!ok) atomicOr(status, 16);
}

size_t jdec_scratch_bytes(const JdecHeader& hd) {
  const size_t n = (size_t)(hd.nsub > 0 ? hd.nsub : 1);
  return a256(8 * n) * 2 + a256(4 * n) * 2 + a256(n) * 2 + a256(4 * (kSyncPasses + 2)) +
         a256(4 * n) + a256(8 * n) + a256(12 * n) + a256(8 * n) * 2 + a256(12 * n);
}

bool jdec_launch(const JdecHeader& hd, const uint8_t* dstream, uint8_t* dpacked, uint8_t* scratch,
                 int32_t* dstatus, hipStream_t st) {
  if (hd.nsub <= 0 || hd.nsub > 0x7fffffffll) return fail("jpeg: bad subsequence count");
  if (hd.h.nscans != 1) return fail("jpeg: device decode takes one scan");
  const JdecScratch S = carve(scratch, hd.nsub);
  if (!UPH_HIP(hipMemsetAsync(S.changed, 0, 4 * (kSyncPasses + 2), st))) return false;
  const dim3 grid((unsigned)((hd.nsub + 255) / 256));
  for (int p = 0; p <= kSyncPasses; p++)
    hipLaunchKernelGGL(k_jdec_sync, grid, dim3(256), 0, st, dstream, scratch, p);
  hipLaunchKernelGGL(k_jdec_settle, dim3(1), dim3(256), 0, st, dstream, scratch);
  hipLaunchKernelGGL(k_jdec_count, grid, dim3(256), 0, st, dstream, scratch, dstatus);
  hipLaunchKernelGGL(k_jdec_scan, dim3(1), dim3(1024), 0, st, dstream, scratch, dpacked, dstatus);
  hipLaunchKernelGGL(k_jdec_emit, grid, dim3(256), 0, st, dstream, scratch, dpacked, dstatus);
  return UPH_HIP(hipGetLastError());
}

}  // namespace uph
