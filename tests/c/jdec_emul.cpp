// jdec_emul.cpp — TEST INFRASTRUCTURE: the device Huffman decoder's phases
// (csrc/kernels_jpeg_huff.hip) replayed on the CPU with the same building
// blocks (csrc/jpeg_huff_core.h), so that the CPU suite checks the
// algorithm -- subsequence synchronisation, block ownership, offsets, DC
// predictors, the packed layout -- against PIL without a GPU.  Every
// "thread" of a pass reads only what the previous pass wrote, as on the
// device.  Built by `make jdec_emul` into tests/c/_build/libjdec_emul.so.
#include <cstdint>
#include <cstring>
#include <vector>

#include "jpeg.h"
#include "jpeg_huff_core.h"

using namespace uph;
using namespace uph::jdec;

extern "C" {

// Decodes `file` into the packed layout (jpeg.h) as the device would.
// Returns the layout's size (written when cap suffices), -1 on a host error
// (uphip_last_error), -2 for a file the device path does not take
// (progressive / several scans), -3 + status bits << 8 for corrupt data;
// *passes = the sync pass that converged (0 = settled serially).
int64_t jdec_emulate(const uint8_t* file, size_t n, uint8_t* out, int64_t cap, int32_t* passes) {
  JdecStreamHost S;
  const int r = jpeg_stream_prepare(file, n, "<emul>", &S);
  if (r < 0) return -1;
  if (r == 0) return -2;
  std::vector<uint8_t> stream((size_t)S.hd.total_bytes + 16);
  jpeg_stream_pack(S, stream.data());
  const JdecHeader& hd = S.hd;
  std::vector<uint8_t> scratch(jdec_scratch_bytes(hd) + 256);
  const JdecScratch X = carve(scratch.data(), hd.nsub, hd.nmac);
  JdecTable tab[6];
  for (int i = 0; i < hd.h.scan[0].ncomp; i++) {
    tab[i] = hd.dc[hd.tdc[i]];
    tab[3 + i] = hd.ac[hd.tac[i]];
  }
  const uint8_t* base = stream.data();
  Dec d;
  d.tab = tab;
  d.bpm = hd.h.scan[0].blocks_per_mcu;
  d.bmap = block_map(hd.bcomp, d.bpm);
  d.nseg = hd.nseg;
  d.seg = (const int32_t*)(base + hd.seg_off);
  d.segsub = (const int32_t*)(base + hd.segsub_off);
  d.segmac = (const int32_t*)(base + hd.segmac_off);
  d.data = (const uint32_t*)(base + hd.data_off);
  int32_t status = 0;
  // k_jdec_sync
  memset(X.changed, 0, 4 * (kSyncPasses + 2));
  for (int pass = 0; pass <= kSyncPasses; pass++) {
    bool skip = false;
    for (int p = 1; p < pass; p++)
      if (X.changed[p] == 0) skip = true;
    if (skip) continue;
    for (int64_t m = 0; m < hd.nmac; m++) sync_macro(d, X, m, pass);
  }
  // k_jdec_settle
  *passes = 0;
  bool conv = false;
  for (int p = 1; p <= kSyncPasses && !conv; p++)
    if (X.changed[p] == 0) {
      *X.final_buf = p & 1;
      *passes = p;
      conv = true;
    }
  if (!conv) {
    settle_serial(d, X, kSyncPasses & 1);
    *X.final_buf = kSyncPasses & 1;
  }
  // k_jdec_scan
  std::vector<uint8_t> packed((size_t)hd.h.total_bytes, 0);
  memcpy(packed.data(), &hd.h, sizeof(JpegHeader));
  {
    int64_t cb = 0, cc = 0, cd[3] = {0, 0, 0};
    for (int64_t i = 0; i < hd.nsub; i++) {
      X.blkoff[i] = cb;
      X.coefoff[i] = cc;
      cb += X.nblk[i];
      cc += X.ncoef[i];
      for (int k = 0; k < 3; k++) {
        X.dcpre[3 * i + k] = (int32_t)cd[k];
        cd[k] += X.dcsum[3 * i + k];
      }
    }
    const int bpm = hd.h.scan[0].blocks_per_mcu;
    std::vector<int32_t> pre(X.dcpre, X.dcpre + 3 * hd.nsub);
    for (int64_t i = 0; i < hd.nsub; i++) {
      const int g = seg_search(d.segsub, d.nseg, i);
      const int64_t f = d.segsub[g];
      if (i == f && hd.restart && X.blkoff[i] != (int64_t)g * hd.restart * bpm) status |= 2;
      for (int k = 0; k < 3; k++) X.dcpre[3 * i + k] = pre[3 * i + k] - pre[3 * f + k];
    }
    if (cb != hd.h.nblocks) status |= 4;
    ((uint32_t*)(packed.data() + hd.h.groups_off))[hd.h.ngroups] = (uint32_t)cc;
  }
  // k_jdec_zero: the vector above starts zeroed; k_jdec_emit
  uint8_t* counts = packed.data() + hd.h.counts_off;
  uint32_t* groups = (uint32_t*)(packed.data() + hd.h.groups_off);
  int16_t* coefs = (int16_t*)(packed.data() + hd.h.coefs_off);
  const int64_t row_blocks = (int64_t)hd.h.scan[0].mcus_x * hd.h.scan[0].blocks_per_mcu;
  for (int64_t i = 0; i < hd.nsub; i++) {
    int64_t blk = X.blkoff[i], co = X.coefoff[i];
    int pred[3] = {X.dcpre[3 * i], X.dcpre[3 * i + 1], X.dcpre[3 * i + 2]};
    int64_t next_row = (blk + row_blocks - 1) / row_blocks * row_blocks;
    const bool ok = walk_owned(
        d, X, i,
        [&](int c, int zz, int val) {
          if (blk >= hd.h.nblocks) return;
          if (zz == 0) {
            if (blk == next_row) groups[blk / row_blocks] = (uint32_t)co;
            pred[c] += val;
            val = pred[c];
          }
          coefs[co + zz] = (int16_t)val;
        },
        [&](int last) {
          if (blk < hd.h.nblocks) counts[blk] = (uint8_t)(last + 1);
          next_row += blk == next_row ? row_blocks : 0;
          blk++;
          co += last + 1;
        });
    if (!ok) status |= 16;
  }
  if (status) return -3 - ((int64_t)status << 8);
  if (out && cap >= (int64_t)packed.size()) memcpy(out, packed.data(), packed.size());
  return (int64_t)packed.size();
}

}  // extern "C"
