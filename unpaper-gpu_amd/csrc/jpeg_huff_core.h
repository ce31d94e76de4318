// jpeg_huff_core.h — the device Huffman decoder's building blocks
// (kernels_jpeg_huff.hip), callable from host code as well so that
// tests/c/jdec_emul.cpp can replay the kernels' phases on the CPU.
//
// Units: a subsequence is kJdecSubBits bits of one restart segment (the
// write pass gives each its own lane); a macro is kJdecMacro consecutive
// subsequences of a segment (a synchronisation pass decodes a macro in one
// lane, recording the exit state of each of its subsequences and counting
// the blocks each owns).  Bit positions are int32 (the stream's data is
// below 2^31 bits, jpeg_stream_prepare).
//
// The decoding loops are written for a wave whose lanes sit at different
// points of their blocks: one path for DC and AC codes, selects instead of
// branches where both sides are cheap, and one rarely taken branch for
// subsequence ends and the end of a segment.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg.h"

#define JD_HD __host__ __device__

// Device code reads the tables through LDS pointers and everything else
// through global ones, so that the compiler emits ds_ / global_ accesses
// (flat accesses count against both wait counters: a table lookup would
// wait for every store in flight).
#if defined(__HIP_DEVICE_COMPILE__)
#define JD_LDS __attribute__((address_space(3)))
#define JD_GLB __attribute__((address_space(1)))
#else
#define JD_LDS
#define JD_GLB
#endif

namespace uph {
namespace jdec {

constexpr int kSyncPasses = 8;  // k_jdec_sync launches after pass 0

struct JdecState {
  int32_t pos;
  int32_t bk;  // block of the MCU << 8 | next zigzag index (0 = the DC)
};

// Scratch of one image.  Arrays indexed [buf * n + i] are double-buffered
// across the synchronisation passes.
struct JdecScratch {
  int64_t n, nm;               // subsequences, macros
  JD_GLB int32_t* xpos;        // [2][n] subsequence exits
  JD_GLB int32_t* xbk;         // [2][n]
  JD_GLB uint8_t* chg;         // [2][nm] the macro's exit changed in the pass
  JD_GLB int32_t* epos;        // [nm] pass 0: state at the first code boundary at or
  JD_GLB int32_t* ebk;         //      past the macro's start, decoding from a subsequence earlier
  JD_GLB int32_t* changed;     // [kSyncPasses + 1] any macro exit changed in the pass
  JD_GLB int32_t* final_buf;   // which buffer holds the exact exits
  JD_GLB int32_t* nblk;        // per subsequence: owned blocks
  JD_GLB int32_t* ncoef;       // coefficients written
  JD_GLB int32_t* dcsum;       // [3] per subsequence
  JD_GLB int64_t* blkoff;
  JD_GLB int64_t* coefoff;
  JD_GLB int32_t* dcpre;       // [3] per subsequence
};

JD_HD inline size_t a256(size_t v) { return (v + 255) & ~(size_t)255; }

JD_HD inline JdecScratch carve(uint8_t* p, int64_t nsub, int64_t nmac) {
  JdecScratch s;
  s.n = nsub;
  s.nm = nmac;
  const size_t n = (size_t)nsub, nm = (size_t)nmac;
  s.xpos = (JD_GLB int32_t*)p;
  p += a256(8 * n);
  s.xbk = (JD_GLB int32_t*)p;
  p += a256(8 * n);
  s.chg = (JD_GLB uint8_t*)p;
  p += a256(2 * nm);
  s.epos = (JD_GLB int32_t*)p;
  p += a256(4 * nm);
  s.ebk = (JD_GLB int32_t*)p;
  p += a256(4 * nm);
  s.changed = (JD_GLB int32_t*)p;
  s.final_buf = s.changed + kSyncPasses + 1;
  p += a256(4 * (kSyncPasses + 2));
  s.nblk = (JD_GLB int32_t*)p;
  p += a256(4 * n);
  s.ncoef = (JD_GLB int32_t*)p;
  p += a256(4 * n);
  s.dcsum = (JD_GLB int32_t*)p;
  p += a256(12 * n);
  s.blkoff = (JD_GLB int64_t*)p;
  p += a256(8 * n);
  s.coefoff = (JD_GLB int64_t*)p;
  p += a256(8 * n);
  s.dcpre = (JD_GLB int32_t*)p;
  return s;
}

JD_HD inline size_t scratch_bytes(int64_t nsub, int64_t nmac) {
  const size_t n = (size_t)nsub, nm = (size_t)nmac;
  return a256(8 * n) * 2 + a256(2 * nm) + a256(4 * nm) * 2 + a256(4 * (kSyncPasses + 2)) +
         a256(4 * n) * 2 + a256(12 * n) + a256(8 * n) * 2 + a256(12 * n);
}

// 32 bits of the stream from bit `pos` (MSB first).  A window of 64 bits
// (v, from bit `base`, a multiple of 64) and the 64 after it (nx, fetched
// when the window last moved, so that its load is in flight while the
// window's bits are decoded).  The data is 16-aligned with 48 bytes of slack.
struct BitPeek {
  const JD_GLB uint32_t* w;
  int32_t base = -128;  // any pos >= 0 is outside: the first peek loads
  uint64_t v = 0, nx = 0;
  JD_HD inline uint64_t pair(int32_t wi) const {
    const uint64_t x = *(const JD_GLB uint64_t*)(w + wi);  // words wi, wi + 1
    return (uint64_t)__builtin_bswap32((uint32_t)x) << 32 | __builtin_bswap32((uint32_t)(x >> 32));
  }
  JD_HD inline uint32_t at(int32_t pos) {
    int32_t off = pos - base;
    if ((uint32_t)off >= 64u) {
      if ((uint32_t)(off - 64) < 64u) {
        base += 64;
        v = nx;
      } else {
        base = pos & ~63;
        v = pair(base >> 5);
      }
      nx = pair((base >> 5) + 2);
      off = pos - base;
    }
    const uint64_t hi = off < 32 ? v : (v << 32) | (nx >> 32);
    return (uint32_t)((hi << (off & 31)) >> 32);
  }
};

// one Huffman code at the top of `bits`: symbol, or -1 (no such code; len 16)
JD_HD inline int huff(const JD_LDS JdecTable* t, uint32_t bits, int* len) {
  const uint32_t e = t->look[bits >> (32 - kJdecLook)];
  if (e) {
    *len = (int)(e >> 8);
    return (int)(e & 0xFF);
  }
  // canonical codes: the length is the shortest l whose code <= maxcode[l]
  int l = 0;
#pragma unroll
  for (int q = 16; q > kJdecLook; q--) l = (int32_t)(bits >> (32 - q)) <= t->maxcode[q] ? q : l;
  if (l == 0) {
    *len = 16;
    return -1;
  }
  *len = l;
  return t->vals[((int32_t)(bits >> (32 - l)) + t->valoff[l]) & 0xFF];
}

JD_HD inline int extend(uint32_t v, int s) {
  return v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

// What a decoding lane needs: the stream's tables (in LDS on the device:
// tab[c] the DC table of scan component c, tab[3 + c] its AC table), the
// block -> scan component map (2 bits a block), the segment tables and the
// data.
struct Dec {
  const JD_LDS JdecTable* tab;
  uint32_t bmap;
  int bpm;  // blocks per MCU
  int nseg;
  const JD_GLB int32_t* seg;
  const JD_GLB int32_t* segsub;
  const JD_GLB int32_t* segmac;
  const JD_GLB uint32_t* data;
};

JD_HD inline uint32_t block_map(const int32_t* bcomp, int bpm) {
  uint32_t m = 0;
  for (int i = 0; i < bpm; i++) m |= (uint32_t)(bcomp[i] & 3) << (2 * i);
  return m;
}

JD_HD inline int comp_of(const Dec& d, int b) { return (int)(d.bmap >> (2 * b)) & 3; }

// segment of subsequence i / macro m (binary search over a prefix)
JD_HD inline int seg_search(const JD_GLB int32_t* pre, int nseg, int64_t i) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

struct Sub {
  int32_t start, stop, seg_end;
  bool first;  // the segment's first subsequence: starts in a known state
};

JD_HD inline Sub sub_of(const Dec& d, int64_t i) {
  const int g = seg_search(d.segsub, d.nseg, i);
  Sub s;
  const int32_t k = (int32_t)(i - d.segsub[g]);
  s.seg_end = d.seg[g + 1];
  s.start = d.seg[g] + k * kJdecSubBits;
  s.stop = s.start + kJdecSubBits < s.seg_end ? s.start + kJdecSubBits : s.seg_end;
  s.first = k == 0;
  return s;
}

// Decodes one code (plus magnitude bits) from state (pos, b, k); c is block
// b's scan component.  Returns false on an invalid code / coefficient index
// (the state then moves to the next block, so a decoder off the code
// boundaries always advances).  blockend: the code finished a block.
// val/zz: a coefficient written (zz 0 = the DC difference), zz = -1 none.
JD_HD inline bool jdec_step(const Dec& d, BitPeek& br, int c, int32_t& pos, int& b, int& k,
                            int* zz, int* val, bool* blockend) {
  const uint32_t w = br.at(pos);
  const bool dc = k == 0;
  int len;
  const int sym = huff(d.tab + (dc ? c : 3 + c), w, &len);
  const int r = dc ? 0 : (sym >> 4) & 15, sz = dc ? sym : sym & 15;
  const bool zrl = !dc && sz == 0 && r == 15;
  const bool eob = !dc && sz == 0 && r != 15;
  const int ci = k + r;  // the coefficient's zigzag index (0 for a DC)
  const bool ok = sym >= 0 && (dc ? sz <= 11 : eob || (zrl ? k + 16 <= 63 : ci <= 63 && sz <= 10));
  const bool coef = ok && (dc || sz > 0);
  *val = coef && sz > 0 ? extend((w << len) >> (32 - sz), sz) : 0;
  *zz = coef ? ci : -1;
  pos += len + (coef ? sz : 0);
  k = !ok || eob ? 64 : zrl ? k + 16 : ci + 1;
  *blockend = k >= 64;
  if (*blockend) {
    k = 0;
    b = b + 1 == d.bpm ? 0 : b + 1;
  }
  return ok;
}

// At an MCU boundary within the last byte of a segment whose remaining bits
// are the encoder's 1-padding: the segment is done.
JD_HD inline bool padding_end(BitPeek& br, int32_t pos, int b, int k, int32_t seg_end) {
  const int32_t left = seg_end - pos;
  if (b != 0 || k != 0 || left <= 0 || left >= 8) return false;
  const uint32_t w = br.at(pos) >> (32 - left);
  return w == (1u << left) - 1u;
}

// Runs the decoder from (pos, b, k) to the first code boundary at or past
// `stop`.
JD_HD inline void run_to(const Dec& d, BitPeek& br, int32_t& pos, int& b, int& k, int32_t stop,
                         int32_t seg_end) {
  while (pos < stop) {
    if (pos >= seg_end - 7 && padding_end(br, pos, b, k, seg_end)) {
      pos = seg_end;
      break;
    }
    int zz, val;
    bool be;
    jdec_step(d, br, comp_of(d, b), pos, b, k, &zz, &val, &be);
  }
}

// Decodes macro [first, lim) (subsequences of segment g) from (pos, b, k), a
// point at or before the macro's start: records each subsequence's exit
// (the state at the first code boundary at or past its end) into xp / xb,
// and counts, per subsequence, the blocks whose DC code starts in its bits
// -- their number, coefficients (last zigzag index + 1) and DC differences
// per component -- finishing the last block past the macro's end.  *entry:
// the state at the first code boundary at or past the macro's start.
JD_HD inline void decode_macro(const Dec& d, const JdecScratch& X, int g, int64_t first,
                               int64_t lim, int32_t pos, int b, int k, JD_GLB int32_t* xp,
                               JD_GLB int32_t* xb, JdecState* entry) {
  const int32_t seg0 = d.seg[g], seg_end = d.seg[g + 1];
  const int64_t s0 = d.segsub[g];
  BitPeek br{d.data};
  const int32_t mstart = seg0 + (int32_t)(first - s0) * kJdecSubBits;
  run_to(d, br, pos, b, k, mstart, seg_end);  // the look-back, when there is one
  entry->pos = pos;
  entry->bk = b << 8 | k;
  for (int64_t i = first; i < lim; i++) {
    X.nblk[i] = 0;
    X.ncoef[i] = 0;
    X.dcsum[3 * i] = X.dcsum[3 * i + 1] = X.dcsum[3 * i + 2] = 0;
  }
  // from here on every code starts at or past the macro's start
  int64_t j = first;  // the subsequence the decoder is in
  const int32_t pad = seg_end - 7;  // past this the segment may end in padding
  int32_t stop = mstart + kJdecSubBits < seg_end ? mstart + kJdecSubBits : seg_end;
  int32_t gate = stop < pad ? stop : pad;  // the rare branch below runs from here
  int64_t owner = -1;  // subsequence owning the block in progress (-1: not counted)
  int64_t cur = -1;    // subsequence whose counts are being summed
  int cc = 0, last = 0, diff = 0;
  int32_t nb = 0, nc = 0, d0 = 0, d1 = 0, d2 = 0;
  for (;;) {
    if (pos >= gate) {
      while (j < lim && pos >= stop) {  // crossed subsequence j's end
        xp[j] = pos;
        xb[j] = b << 8 | k;
        if (++j < lim) stop = stop + kJdecSubBits < seg_end ? stop + kJdecSubBits : seg_end;
      }
      if (j >= lim && k == 0) break;  // every exit recorded, no block open
      if (padding_end(br, pos, b, k, seg_end) || pos >= seg_end) {
        // the segment ends (inside a block: corrupt; the scan checks it)
        const int32_t e = pos >= seg_end ? pos : seg_end;
        const int32_t ebk = pos >= seg_end ? (b << 8 | k) : 0;
        for (; j < lim; j++) {
          xp[j] = e;
          xb[j] = ebk;
        }
        break;
      }
      // past the last exit: stay in this branch until the block ends
      gate = j >= lim ? pos : (stop < pad ? stop : pad);
    }
    const int c = comp_of(d, b);
    int zz, val;
    bool be;
    jdec_step(d, br, c, pos, b, k, &zz, &val, &be);
    const bool dcz = zz == 0;  // a block starts: owned by j (none past the macro)
    owner = dcz ? (j < lim ? j : -1) : owner;
    cc = dcz ? c : cc;
    diff = dcz ? val : diff;
    last = dcz ? 0 : zz > 0 ? zz : last;
    const bool done = be && owner >= 0;
    if (done && owner != cur) {  // the first block of another subsequence
      if (cur >= 0) {
        X.nblk[cur] = nb;
        X.ncoef[cur] = nc;
        X.dcsum[3 * cur] = d0;
        X.dcsum[3 * cur + 1] = d1;
        X.dcsum[3 * cur + 2] = d2;
      }
      nb = nc = d0 = d1 = d2 = 0;
      cur = owner;
    }
    nb += done ? 1 : 0;
    nc += done ? last + 1 : 0;
    d0 += done && cc == 0 ? diff : 0;
    d1 += done && cc == 1 ? diff : 0;
    d2 += done && cc == 2 ? diff : 0;
    owner = be ? -1 : owner;
  }
  if (cur >= 0) {
    X.nblk[cur] = nb;
    X.ncoef[cur] = nc;
    X.dcsum[3 * cur] = d0;
    X.dcsum[3 * cur + 1] = d1;
    X.dcsum[3 * cur + 2] = d2;
  }
}

// Macro m of sync pass `pass`.  Pass 0 decodes from one subsequence before
// the macro (its segment's start for a segment's first macro) and keeps the
// state it crosses the macro's start in.  Pass 1 decodes again, from the
// predecessor's pass-0 exit, only the macros whose crossing state differs
// from that exit (the others already decoded from the true state); later
// passes only those whose predecessor's exit changed in the pass before.
JD_HD inline void sync_macro(const Dec& d, const JdecScratch& X, int64_t m, int pass) {
  const int g = seg_search(d.segmac, d.nseg, m);
  const int64_t first = d.segsub[g] + (m - d.segmac[g]) * kJdecMacro;
  const int64_t lim = d.segsub[g + 1] < first + kJdecMacro ? d.segsub[g + 1] : first + kJdecMacro;
  const bool seg_first = m == d.segmac[g];
  const int cur = pass & 1, prv = cur ^ 1;
  JD_GLB int32_t* xp = X.xpos + cur * X.n;
  JD_GLB int32_t* xb = X.xbk + cur * X.n;
  const JD_GLB int32_t* pp = X.xpos + prv * X.n;
  const JD_GLB int32_t* pb = X.xbk + prv * X.n;
  bool redo = pass == 0;
  if (pass == 1)
    redo = !seg_first && (X.epos[m] != pp[first - 1] || X.ebk[m] != pb[first - 1]);
  else if (pass >= 2)
    redo = !seg_first && X.chg[prv * X.nm + m - 1];
  if (!redo) {
    for (int64_t i = first; i < lim; i++) {
      xp[i] = pp[i];
      xb[i] = pb[i];
    }
    X.chg[cur * X.nm + m] = 0;
    return;
  }
  const int32_t seg0 = d.seg[g];
  int32_t pos;
  int b = 0, k = 0;
  if (pass == 0) {
    pos = seg_first ? seg0 : seg0 + (int32_t)(first - 1 - d.segsub[g]) * kJdecSubBits;
  } else {
    pos = pp[first - 1];
    b = pb[first - 1] >> 8;
    k = pb[first - 1] & 255;
  }
  JdecState e;
  decode_macro(d, X, g, first, lim, pos, b, k, xp, xb, &e);
  if (pass == 0) {
    X.epos[m] = e.pos;
    X.ebk[m] = e.bk;
  }
  const bool ch = pass > 0 && (xp[lim - 1] != pp[lim - 1] || xb[lim - 1] != pb[lim - 1]);
  X.chg[cur * X.nm + m] = ch ? 1 : 0;
  if (ch) X.changed[pass] = 1;
}

// Exact exits (and counts) without convergence: the macros in order from
// the known segment starts (one lane; correct for any stream).
JD_HD inline void settle_serial(const Dec& d, const JdecScratch& X, int buf) {
  JD_GLB int32_t* xp = X.xpos + buf * X.n;
  JD_GLB int32_t* xb = X.xbk + buf * X.n;
  for (int g = 0; g < d.nseg; g++) {
    int32_t pos = d.seg[g];
    int b = 0, k = 0;
    for (int64_t m = d.segmac[g]; m < d.segmac[g + 1]; m++) {
      const int64_t first = d.segsub[g] + (m - d.segmac[g]) * kJdecMacro;
      const int64_t lim =
          d.segsub[g + 1] < first + kJdecMacro ? d.segsub[g + 1] : first + kJdecMacro;
      JdecState e;
      decode_macro(d, X, g, first, lim, pos, b, k, xp, xb, &e);
      pos = xp[lim - 1];
      b = xb[lim - 1] >> 8;
      k = xb[lim - 1] & 255;
    }
  }
}

// Walks subsequence i's blocks (those whose DC code starts in it) from its
// exact entry; on_coef(block's component, zz, value) per coefficient,
// on_block(last zz) per block.  False: corrupt data.
template <class FCoef, class FBlock>
JD_HD inline bool walk_owned(const Dec& d, const JdecScratch& S, int64_t i, FCoef&& on_coef,
                             FBlock&& on_block) {
  const Sub s = sub_of(d, i);
  const int fb = *S.final_buf;
  const JD_GLB int32_t* xp = S.xpos + fb * S.n;
  const JD_GLB int32_t* xb = S.xbk + fb * S.n;
  int32_t pos = s.first ? s.start : xp[i - 1];
  int b = s.first ? 0 : xb[i - 1] >> 8, k = s.first ? 0 : xb[i - 1] & 255;
  const int32_t own_end = xp[i];  // blocks starting before this are ours
  BitPeek br{d.data};
  // the block in progress at the entry belongs to the previous subsequence
  while (k != 0 && pos < s.seg_end) {
    int zz, val;
    bool be;
    jdec_step(d, br, comp_of(d, b), pos, b, k, &zz, &val, &be);
  }
  bool ok = true;
  int last = 0, cc = 0;
  // one code a trip; a block ends at a block end, the data's end (corrupt)
  // or an invalid code (corrupt)
  while (k != 0 || pos < own_end) {
    if (pos >= s.seg_end - 7) {
      if (k == 0 && padding_end(br, pos, b, k, s.seg_end)) break;
      if (pos >= s.seg_end) {  // the data ended inside a block
        ok = false;
        on_block(last);
        break;
      }
    }
    const int c = comp_of(d, b);
    int zz, val;
    bool be;
    const bool good = jdec_step(d, br, c, pos, b, k, &zz, &val, &be);
    cc = zz == 0 ? c : cc;
    if (zz >= 0) on_coef(cc, zz, val);
    last = zz == 0 ? 0 : zz > 0 ? zz : last;
    if (be) {
      on_block(last);
      last = 0;
    }
    if (!good) {
      ok = false;
      break;
    }
  }
  return ok;
}

}  // namespace jdec
}  // namespace uph
