// jpeg_huff_core.h — the device Huffman decoder's building blocks
// (kernels_jpeg_huff.hip), callable from host code as well so that
// tests/c/jdec_emul.cpp can replay the kernels' phases on the CPU.
//
// Units: a subsequence is kJdecSubBits bits of one restart segment (the
// count and write passes give each its own lane); a macro is kJdecMacro
// consecutive subsequences of a segment (a synchronisation pass decodes a
// macro in one lane, recording the exit state of each of its subsequences).
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

// Scratch of one image.  Arrays indexed [buf * n + i] are double-buffered
// across the synchronisation passes.
struct JdecScratch {
  int64_t n, nm;      // subsequences, macros
  int64_t* xpos;      // [2][n] subsequence exits
  int32_t* xbk;       // [2][n]
  uint8_t* chg;       // [2][nm] the macro's exit changed in the pass
  int32_t* changed;   // [kSyncPasses + 1] any macro exit changed in the pass
  int32_t* final_buf; // which buffer holds the exact exits
  int32_t* nblk;      // per subsequence: owned blocks
  int64_t* ncoef;     // coefficients written
  int32_t* dcsum;     // [3] per subsequence
  int64_t* blkoff;
  int64_t* coefoff;
  int32_t* dcpre;     // [3] per subsequence
};

JD_HD inline size_t a256(size_t v) { return (v + 255) & ~(size_t)255; }

JD_HD inline JdecScratch carve(uint8_t* p, int64_t nsub, int64_t nmac) {
  JdecScratch s;
  s.n = nsub;
  s.nm = nmac;
  const size_t n = (size_t)nsub, nm = (size_t)nmac;
  s.xpos = (int64_t*)p;
  p += a256(16 * n);
  s.xbk = (int32_t*)p;
  p += a256(8 * n);
  s.chg = p;
  p += a256(2 * nm);
  s.changed = (int32_t*)p;
  s.final_buf = s.changed + kSyncPasses + 1;
  p += a256(4 * (kSyncPasses + 2));
  s.nblk = (int32_t*)p;
  p += a256(4 * n);
  s.ncoef = (int64_t*)p;
  p += a256(8 * n);
  s.dcsum = (int32_t*)p;
  p += a256(12 * n);
  s.blkoff = (int64_t*)p;
  p += a256(8 * n);
  s.coefoff = (int64_t*)p;
  p += a256(8 * n);
  s.dcpre = (int32_t*)p;
  return s;
}

JD_HD inline size_t scratch_bytes(int64_t nsub, int64_t nmac) {
  const size_t n = (size_t)nsub, nm = (size_t)nmac;
  return a256(16 * n) + a256(8 * n) + a256(2 * nm) + a256(4 * (kSyncPasses + 2)) + a256(4 * n) +
         a256(8 * n) + a256(12 * n) + a256(8 * n) * 2 + a256(12 * n);
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

// What a decoding lane needs: the stream's tables (in LDS on the device),
// the block -> scan component map, the segment tables and the data.
struct Dec {
  const JdecTable* dct;  // per scan component
  const JdecTable* act;
  const int8_t* bcomp;   // scan component of each block of an MCU
  int bpm;               // blocks per MCU
  int nseg;
  const int64_t* seg;
  const int32_t* segsub;
  const int32_t* segmac;
  const uint32_t* data;
};

// segment of subsequence i / macro m (binary search over a prefix)
JD_HD inline int seg_search(const int32_t* pre, int nseg, int64_t i) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

struct Sub {
  int64_t start, stop, seg_end;
  bool first;  // the segment's first subsequence: starts in a known state
};

JD_HD inline Sub sub_of(const Dec& d, int64_t i) {
  const int g = seg_search(d.segsub, d.nseg, i);
  Sub s;
  const int64_t k = i - d.segsub[g];
  s.seg_end = d.seg[g + 1];
  s.start = d.seg[g] + k * kJdecSubBits;
  s.stop = s.start + kJdecSubBits < s.seg_end ? s.start + kJdecSubBits : s.seg_end;
  s.first = k == 0;
  return s;
}

// Decodes one code (plus magnitude bits) from state (pos, b, k).  Returns
// false on an invalid code / coefficient index (the state then moves to the
// next block, so a decoder off the code boundaries always advances).
// blockend: the code finished a block.  val/zz: a coefficient written
// (zz 0 = the DC difference), zz = -1 none.
JD_HD inline bool jdec_step(const Dec& d, BitPeek& br, int64_t& pos, int& b, int& k, int* zz,
                            int* val, bool* blockend) {
  const uint32_t w = br.at(pos);
  const int c = d.bcomp[b];
  int len;
  bool ok = true;
  *zz = -1;
  if (k == 0) {
    const int t = huff(d.dct[c], w, &len);
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
    const int rs = huff(d.act[c], w, &len);
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
    b = b + 1 == d.bpm ? 0 : b + 1;
  }
  return ok;
}

// At an MCU boundary within the last byte of a segment whose remaining bits
// are the encoder's 1-padding: the segment is done.
JD_HD inline bool padding_end(BitPeek& br, int64_t pos, int b, int k, int64_t seg_end) {
  const int64_t left = seg_end - pos;
  if (b != 0 || k != 0 || left <= 0 || left >= 8) return false;
  const uint32_t w = br.at(pos) >> (32 - (int)left);
  return w == (1u << left) - 1u;
}

// Runs the decoder from (pos, b, k) to the first code boundary at or past
// `stop`.
JD_HD inline void run_to(const Dec& d, BitPeek& br, int64_t& pos, int& b, int& k, int64_t stop,
                         int64_t seg_end) {
  while (pos < stop) {
    if (padding_end(br, pos, b, k, seg_end)) {
      pos = seg_end;
      break;
    }
    int zz, val;
    bool be;
    jdec_step(d, br, pos, b, k, &zz, &val, &be);
  }
}

// Macro m of sync pass `pass`: from its predecessor's exit of the previous
// pass (pass 0: from its first bit, as if a block started there) through its
// subsequences, recording each one's exit.  From pass 2 on, a macro whose
// entry did not change keeps its exits.
JD_HD inline void sync_macro(const Dec& d, const JdecScratch& X, int64_t m, int pass) {
  const int g = seg_search(d.segmac, d.nseg, m);
  const int64_t first = d.segsub[g] + (m - d.segmac[g]) * kJdecMacro;
  const int64_t lim = d.segsub[g + 1] < first + kJdecMacro ? d.segsub[g + 1] : first + kJdecMacro;
  const bool seg_first = m == d.segmac[g];
  const int cur = pass & 1, prv = cur ^ 1;
  int64_t* xp = X.xpos + cur * X.n;
  int32_t* xb = X.xbk + cur * X.n;
  const int64_t* pp = X.xpos + prv * X.n;
  const int32_t* pb = X.xbk + prv * X.n;
  if (pass > 0 && (seg_first || (pass >= 2 && !X.chg[prv * X.nm + m - 1]))) {
    for (int64_t i = first; i < lim; i++) {
      xp[i] = pp[i];
      xb[i] = pb[i];
    }
    X.chg[cur * X.nm + m] = 0;
    return;
  }
  const int64_t seg_end = d.seg[g + 1];
  int64_t pos;
  int b = 0, k = 0;
  if (seg_first || pass == 0) {
    pos = d.seg[g] + (first - d.segsub[g]) * kJdecSubBits;
  } else {
    pos = pp[first - 1];
    b = pb[first - 1] >> 8;
    k = pb[first - 1] & 255;
  }
  BitPeek br{d.data};
  for (int64_t i = first; i < lim; i++) {
    const int64_t start = d.seg[g] + (i - d.segsub[g]) * kJdecSubBits;
    const int64_t stop = start + kJdecSubBits < seg_end ? start + kJdecSubBits : seg_end;
    run_to(d, br, pos, b, k, stop, seg_end);
    xp[i] = pos;
    xb[i] = b << 8 | k;
  }
  const bool ch = pass > 0 && (xp[lim - 1] != pp[lim - 1] || xb[lim - 1] != pb[lim - 1]);
  X.chg[cur * X.nm + m] = ch ? 1 : 0;
  if (ch) X.changed[pass] = 1;
}

// Exact exits without convergence: the macros in order from the known
// segment starts (one lane; correct for any stream).
JD_HD inline void settle_serial(const Dec& d, const JdecScratch& X, int buf) {
  int64_t* xp = X.xpos + buf * X.n;
  int32_t* xb = X.xbk + buf * X.n;
  BitPeek br{d.data};
  int64_t pos = 0;
  int b = 0, k = 0;
  for (int64_t i = 0; i < X.n; i++) {
    const Sub s = sub_of(d, i);
    if (s.first) {
      pos = s.start;
      b = k = 0;
    }
    run_to(d, br, pos, b, k, s.stop, s.seg_end);
    xp[i] = pos;
    xb[i] = b << 8 | k;
  }
}

// Walks subsequence i's blocks (those whose DC code starts in it) from its
// exact entry; on_coef(block, zz, value, last zz so far) per coefficient,
// on_block(block, last zz) per block.  False: corrupt data.
template <class FCoef, class FBlock>
JD_HD inline bool walk_owned(const Dec& d, const JdecScratch& S, int64_t i, FCoef&& on_coef,
                             FBlock&& on_block) {
  const Sub s = sub_of(d, i);
  const int fb = *S.final_buf;
  const int64_t* xp = S.xpos + fb * S.n;
  const int32_t* xb = S.xbk + fb * S.n;
  int64_t pos = s.first ? s.start : xp[i - 1];
  int b = s.first ? 0 : xb[i - 1] >> 8, k = s.first ? 0 : xb[i - 1] & 255;
  const int64_t own_end = xp[i];  // blocks starting before this are ours
  BitPeek br{d.data};
  bool ok = true;
  // the block in progress at the entry belongs to the previous subsequence
  while (k != 0 && pos < s.seg_end) {
    int zz, val;
    bool be;
    jdec_step(d, br, pos, b, k, &zz, &val, &be);
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
      ok &= jdec_step(d, br, pos, b, k, &zz, &val, &be);
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

}  // namespace jdec
}  // namespace uph
