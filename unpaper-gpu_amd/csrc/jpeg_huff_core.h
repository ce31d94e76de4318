// jpeg_huff_core.h — the device Huffman decoder's building blocks
// (kernels_jpeg_huff.hip), callable from host code as well so that
// tests/c/jdec_emul.cpp can replay the kernels' phases on the CPU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg.h"

#define JD_HD __host__ __device__

namespace uph {
namespace jdec {


constexpr int kSyncPasses = 8;  // k_jdec_sync launches after pass 0

struct JdecState {
  int64_t pos;
  int32_t bk;  // block of the MCU << 8 | next zigzag index (0 = the DC)
};

struct JdecScratch {
  int64_t* xpos[2];   // exits of the sync passes (double-buffered)
  int32_t* xbk[2];
  uint8_t* chg[2];    // per subsequence: its exit changed in the pass (alternating)
  int32_t* changed;   // [kSyncPasses + 1]
  int32_t* final_buf; // which buffer holds the exact exits
  int32_t* nblk;      // per subsequence: owned blocks
  int64_t* ncoef;     // coefficients written
  int32_t* dcsum;     // [3] per subsequence
  int64_t* blkoff;
  int64_t* coefoff;
  int32_t* dcpre;     // [3] per subsequence
};

JD_HD inline size_t a256(size_t v) { return (v + 255) & ~(size_t)255; }

JD_HD inline JdecScratch carve(uint8_t* p, int64_t nsub) {
  JdecScratch s;
  const size_t n = (size_t)nsub;
  auto take = [&](size_t bytes) {
    uint8_t* r = p;
    p += a256(bytes);
    return r;
  };
  s.xpos[0] = (int64_t*)take(8 * n);
  s.xpos[1] = (int64_t*)take(8 * n);
  s.xbk[0] = (int32_t*)take(4 * n);
  s.xbk[1] = (int32_t*)take(4 * n);
  s.chg[0] = take(n);
  s.chg[1] = take(n);
  s.changed = (int32_t*)take(4 * (kSyncPasses + 2));
  s.final_buf = s.changed + kSyncPasses + 1;
  s.nblk = (int32_t*)take(4 * n);
  s.ncoef = (int64_t*)take(8 * n);
  s.dcsum = (int32_t*)take(12 * n);
  s.blkoff = (int64_t*)take(8 * n);
  s.coefoff = (int64_t*)take(8 * n);
  s.dcpre = (int32_t*)take(12 * n);
  return s;
}

// 32 bits of the stream from bit `pos` (MSB first); the data is 4-aligned
// and has 16 bytes of slack
struct BitPeek {
  const uint32_t* w;
  int64_t cw = -2;
  uint64_t v = 0;
  JD_HD inline uint32_t at(int64_t pos) {
    const int64_t wi = pos >> 5;
    if (wi != cw) {
      if (wi == cw + 1)
        v = (v << 32) | __builtin_bswap32(w[wi + 1]);
      else
        v = ((uint64_t)__builtin_bswap32(w[wi]) << 32) | __builtin_bswap32(w[wi + 1]);
      cw = wi;
    }
    const int off = (int)(pos & 31);
    return (uint32_t)(v >> (32 - off));
  }
};

// one Huffman code at the top of `bits`: symbol, or -1 (no such code)
JD_HD inline int huff(const JdecTable& t, uint32_t bits, int* len) {
  const uint32_t e = t.look[bits >> (32 - kJdecLook)];
  if (e) {
    *len = (int)(e >> 8);
    return (int)(e & 0xFF);
  }
  for (int l = kJdecLook + 1; l <= 16; l++) {
    const int32_t code = (int32_t)(bits >> (32 - l));
    if (code <= t.maxcode[l]) {
      *len = l;
      return t.vals[(code + t.valoff[l]) & 0xFF];
    }
  }
  *len = 16;
  return -1;
}

JD_HD inline int extend(uint32_t v, int s) {
  return v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

struct Ctx {
  const JdecHeader* hd;
  const int64_t* seg;
  const int32_t* segsub;
  const uint32_t* data;
};

JD_HD inline Ctx ctx_of(const uint8_t* stream) {
  Ctx c;
  c.hd = (const JdecHeader*)stream;
  c.seg = (const int64_t*)(stream + c.hd->seg_off);
  c.segsub = (const int32_t*)(stream + c.hd->segsub_off);
  c.data = (const uint32_t*)(stream + c.hd->data_off);
  return c;
}

// segment of subsequence i (binary search over the prefix of subsequences)
JD_HD inline int seg_of(const Ctx& c, int64_t i) {
  int lo = 0, hi = c.hd->nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (c.segsub[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

struct Sub {
  int64_t start, stop, seg_end;
  bool first;  // the segment's first subsequence: starts in a known state
};

JD_HD inline Sub sub_of(const Ctx& c, int64_t i) {
  const int g = seg_of(c, i);
  Sub s;
  const int64_t k = i - c.segsub[g];
  s.seg_end = c.seg[g + 1];
  s.start = c.seg[g] + k * kJdecSubBits;
  s.stop = s.start + kJdecSubBits < s.seg_end ? s.start + kJdecSubBits : s.seg_end;
  s.first = k == 0;
  return s;
}

// Decodes one code (plus magnitude bits) from state (pos, b, k).  Returns
// false on an invalid code / coefficient index (the state then moves to the
// next block, so a decoder off the code boundaries always advances).
// blockend: the code finished a block.  val/zz: a coefficient written
// (zz 0 = the DC difference), zz = -1 none.
JD_HD inline bool jdec_step(const JdecHeader& H, const JdecTable* dct,
                                          const JdecTable* act, BitPeek& br, int64_t& pos, int& b,
                                          int& k, int bpm, int* zz, int* val, bool* blockend) {
  const uint32_t w = br.at(pos);
  const int c = H.bcomp[b];
  int len;
  bool ok = true;
  *zz = -1;
  if (k == 0) {
    const int t = huff(dct[c], w, &len);
    if (t < 0 || t > 11) {
      ok = false;
      pos += len;
      k = 64;
    } else {
      *zz = 0;
      *val = t ? extend((w << len) >> (32 - t), t) : 0;
      pos += len + t;
      k = 1;
    }
  } else {
    const int rs = huff(act[c], w, &len);
    if (rs < 0) {
      ok = false;
      pos += len;
      k = 64;
    } else {
      const int r = rs >> 4, sz = rs & 15;
      if (sz) {
        k += r;
        if (k > 63 || sz > 10) {
          ok = false;
          pos += len;
          k = 64;
        } else {
          *zz = k;
          *val = extend((w << len) >> (32 - sz), sz);
          pos += len + sz;
          k++;
        }
      } else if (r == 15) {
        k += 16;
        pos += len;
        if (k > 63) {  // a zero run must be followed by a coefficient
          ok = false;
          k = 64;
        }
      } else {
        pos += len;  // end of block
        k = 64;
      }
    }
  }
  *blockend = k >= 64;
  if (*blockend) {
    k = 0;
    b = b + 1 == bpm ? 0 : b + 1;
  }
  return ok;
}

// At an MCU boundary within the last byte of a segment whose remaining bits
// are the encoder's 1-padding: the segment is done.
JD_HD inline bool padding_end(BitPeek& br, int64_t pos, int b, int k,
                                            int64_t seg_end) {
  const int64_t left = seg_end - pos;
  if (b != 0 || k != 0 || left <= 0 || left >= 8) return false;
  const uint32_t w = br.at(pos) >> (32 - (int)left);
  return w == (1u << left) - 1u;
}

// Runs the decoder from `st` to the first code boundary at or past `stop`.
JD_HD inline JdecState run_to(const Ctx& c, const JdecTable* dct, const JdecTable* act, JdecState st,
                            int64_t stop, int64_t seg_end) {
  const JdecHeader& H = *c.hd;
  const int bpm = H.h.scan[0].blocks_per_mcu;
  BitPeek br{c.data};
  int64_t pos = st.pos;
  int b = st.bk >> 8, k = st.bk & 255;
  while (pos < stop) {
    if (padding_end(br, pos, b, k, seg_end)) {
      pos = seg_end;
      break;
    }
    int zz, val;
    bool be;
    jdec_step(H, dct, act, br, pos, b, k, bpm, &zz, &val, &be);
  }
  return JdecState{pos, b << 8 | k};
}

// Walks subsequence i's blocks (those whose DC code starts in it) with the
// exact entry state; on_block(b, coefs written ..) per block via callbacks.
template <class FCoef, class FBlock>
JD_HD inline bool walk_owned(const Ctx& c, const JdecTable* dct, const JdecTable* act,
                          const JdecScratch& S, int64_t i, FCoef&& on_coef, FBlock&& on_block) {
  const JdecHeader& H = *c.hd;
  const int bpm = H.h.scan[0].blocks_per_mcu;
  const Sub s = sub_of(c, i);
  const int fb = *S.final_buf;
  JdecState st = s.first ? JdecState{s.start, 0} : JdecState{S.xpos[fb][i - 1], S.xbk[fb][i - 1]};
  const int64_t own_end = S.xpos[fb][i];  // blocks starting before this are ours
  BitPeek br{c.data};
  int64_t pos = st.pos;
  int b = st.bk >> 8, k = st.bk & 255;
  bool ok = true;
  // the block in progress at the entry belongs to the previous subsequence
  while (k != 0 && pos < s.seg_end) {
    int zz, val;
    bool be;
    jdec_step(H, dct, act, br, pos, b, k, bpm, &zz, &val, &be);
  }
  while (pos < own_end) {
    if (padding_end(br, pos, b, k, s.seg_end)) break;
    const int cb = b;
    int last = 0;
    for (;;) {  // one block
      if (pos >= s.seg_end) {  // the data ended inside a block
        ok = false;
        break;
      }
      int zz, val;
      bool be;
      ok &= jdec_step(H, dct, act, br, pos, b, k, bpm, &zz, &val, &be);
      if (zz >= 0) {
        on_coef(cb, zz, val, last);
        if (zz > 0) last = zz;
      }
      if (be) break;
    }
    on_block(cb, last);
    if (!ok) break;
  }
  return ok;
}


// One subsequence of sync pass `pass`: its exit from its predecessor's exit of
// the previous pass (pass 0: from its first bit, as if a block started there).
// From pass 2 on, a subsequence whose entry did not change keeps its exit.
JD_HD inline void sync_sub(const Ctx& c, const JdecTable* dct, const JdecTable* act,
                           const JdecScratch& X, int64_t i, int pass) {
  const Sub s = sub_of(c, i);
  const int cur = pass & 1, prv = cur ^ 1;
  if (pass > 0 && (s.first || (pass >= 2 && !X.chg[prv][i - 1]))) {
    X.xpos[cur][i] = X.xpos[prv][i];
    X.xbk[cur][i] = X.xbk[prv][i];
    X.chg[cur][i] = 0;
    return;
  }
  const JdecState st = (s.first || pass == 0) ? JdecState{s.start, 0}
                                              : JdecState{X.xpos[prv][i - 1], X.xbk[prv][i - 1]};
  const JdecState x = run_to(c, dct, act, st, s.stop, s.seg_end);
  const bool ch = pass > 0 && (x.pos != X.xpos[prv][i] || x.bk != X.xbk[prv][i]);
  X.xpos[cur][i] = x.pos;
  X.xbk[cur][i] = x.bk;
  X.chg[cur][i] = ch ? 1 : 0;
  if (ch) X.changed[pass] = 1;
}

}  // namespace jdec
}  // namespace uph
