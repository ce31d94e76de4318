// j2k_t1.h — the EBCOT code-block coder of JPEG 2000 (ISO/IEC 15444-1 Annex
// C: the MQ arithmetic coder; Annex D: significance propagation, magnitude
// refinement and cleanup passes over 4-row stripes), decoder and encoder.
// Code-block style 0 only (no bypass, no context reset, one codeword segment,
// no vertically causal contexts, no segmentation symbols).
//
// Decoded magnitudes carry one fraction bit, as in OpenJPEG's t1.c (the
// reconstruction sits half a quantisation step into the interval): a
// coefficient that becomes significant at bit-plane p is 3 * 2^p, each
// refinement at plane p moves it by 2^p.  Reversible data divides that by 2
// (exact when every pass was decoded); irreversible data scales it by half
// the quantisation step.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#ifndef J2K_HD
#define J2K_HD __host__ __device__
#endif

namespace uph {
namespace j2k {

// Table C.2: Qe, next index after an MPS / an LPS, MPS switch
struct MqState {
  uint16_t qe;
  uint8_t nmps, nlps, sw;
};
constexpr MqState kMq[47] = {
    {0x5601, 1, 1, 1},   {0x3401, 2, 6, 0},   {0x1801, 3, 9, 0},   {0x0AC1, 4, 12, 0},
    {0x0521, 5, 29, 0},  {0x0221, 38, 33, 0}, {0x5601, 7, 6, 1},   {0x5401, 8, 14, 0},
    {0x4801, 9, 14, 0},  {0x3801, 10, 14, 0}, {0x3001, 11, 17, 0}, {0x2401, 12, 18, 0},
    {0x1C01, 13, 20, 0}, {0x1601, 29, 21, 0}, {0x5601, 15, 14, 1}, {0x5401, 16, 14, 0},
    {0x5101, 17, 15, 0}, {0x4801, 18, 16, 0}, {0x3801, 19, 17, 0}, {0x3401, 20, 18, 0},
    {0x3001, 21, 19, 0}, {0x2801, 22, 19, 0}, {0x2401, 23, 20, 0}, {0x2201, 24, 21, 0},
    {0x1C01, 25, 22, 0}, {0x1801, 26, 23, 0}, {0x1601, 27, 24, 0}, {0x1401, 28, 25, 0},
    {0x1201, 29, 26, 0}, {0x1101, 30, 27, 0}, {0x0AC1, 31, 28, 0}, {0x09C1, 32, 29, 0},
    {0x08A1, 33, 30, 0}, {0x0521, 34, 31, 0}, {0x0441, 35, 32, 0}, {0x02A1, 36, 33, 0},
    {0x0221, 37, 34, 0}, {0x0141, 38, 35, 0}, {0x0111, 39, 36, 0}, {0x0085, 40, 37, 0},
    {0x0049, 41, 38, 0}, {0x0025, 42, 39, 0}, {0x0015, 43, 40, 0}, {0x0009, 44, 41, 0},
    {0x0005, 45, 42, 0}, {0x0001, 45, 43, 0}, {0x5601, 46, 46, 0}};

// contexts: 0-8 zero coding, 9-13 sign, 14-16 magnitude refinement, 17 run
// length, 18 uniform
constexpr int kCtxSc = 9, kCtxMr = 14, kCtxRl = 17, kCtxUni = 18, kNumCtx = 19;

struct MqContexts {
  uint8_t idx[kNumCtx], mps[kNumCtx];
  void reset() {
    memset(idx, 0, sizeof idx);
    memset(mps, 0, sizeof mps);
    idx[kCtxUni] = 46;
    idx[kCtxRl] = 3;
    idx[0] = 4;
  }
};

// Annex C.3 decoder.  The data must be followed by two 0xFF bytes (the
// coder then reads 1-bits past its end, as a marker would make it).
struct MqDecoder {
  const uint8_t* bp;
  uint32_t a, c;
  int ct;
  void bytein() {
    if (bp[0] == 0xFF) {
      if (bp[1] > 0x8F) {
        c += 0xFF00;
        ct = 8;
      } else {
        bp++;
        c += (uint32_t)bp[0] << 9;
        ct = 7;
      }
    } else {
      bp++;
      c += (uint32_t)bp[0] << 8;
      ct = 8;
    }
  }
  void init(const uint8_t* data) {
    bp = data;
    c = (uint32_t)bp[0] << 16;
    bytein();
    c <<= 7;
    ct -= 7;
    a = 0x8000;
  }
  void renorm() {
    do {
      if (ct == 0) bytein();
      a <<= 1;
      c <<= 1;
      ct--;
    } while (a < 0x8000);
  }
  // DECODE (C.3.2): the LPS sub-interval sits below the MPS one (the
  // encoder adds Qe to C for an MPS)
  int decode(MqContexts& cx, int k) {
    const MqState& s = kMq[cx.idx[k]];
    a -= s.qe;
    int d;
    if ((c >> 16) < s.qe) {  // LPS_EXCHANGE
      if (a < s.qe) {
        a = s.qe;
        d = cx.mps[k];
        cx.idx[k] = s.nmps;
      } else {
        a = s.qe;
        d = 1 - cx.mps[k];
        if (s.sw) cx.mps[k] = (uint8_t)(1 - cx.mps[k]);
        cx.idx[k] = s.nlps;
      }
      renorm();
      return d;
    }
    c -= (uint32_t)s.qe << 16;
    if (a & 0x8000) return cx.mps[k];
    if (a < s.qe) {  // MPS_EXCHANGE
      d = 1 - cx.mps[k];
      if (s.sw) cx.mps[k] = (uint8_t)(1 - cx.mps[k]);
      cx.idx[k] = s.nlps;
    } else {
      d = cx.mps[k];
      cx.idx[k] = s.nmps;
    }
    renorm();
    return d;
  }
};

// Annex C.2 encoder (software conventions of the standard: C register with
// spacer bits, byte-out with bit stuffing after 0xFF, FLUSH at the end).
struct MqEncoder {
  uint8_t* out;  // out[-1] is the byte before the codeword (the standard's BPST - 1)
  int64_t n;     // index of the standard's BP relative to out (starts at -1)
  uint32_t a, c;
  int ct;
  void init(uint8_t* buf) {  // buf[0] is that byte; the codeword starts at buf + 1
    out = buf + 1;
    out[-1] = 0;
    n = -1;
    a = 0x8000;
    c = 0;
    ct = 12;
  }
  void byteout() {
    if (out[n] == 0xFF) {
      n++;
      out[n] = (uint8_t)(c >> 20);
      c &= 0xFFFFF;
      ct = 7;
    } else if (c < 0x8000000) {
      n++;
      out[n] = (uint8_t)(c >> 19);
      c &= 0x7FFFF;
      ct = 8;
    } else {
      out[n]++;
      if (out[n] == 0xFF) {
        c &= 0x7FFFFFF;
        n++;
        out[n] = (uint8_t)(c >> 20);
        c &= 0xFFFFF;
        ct = 7;
      } else {
        n++;
        out[n] = (uint8_t)(c >> 19);
        c &= 0x7FFFF;
        ct = 8;
      }
    }
  }
  void renorm() {
    do {
      a <<= 1;
      c <<= 1;
      ct--;
      if (ct == 0) byteout();
    } while (a < 0x8000);
  }
  void encode(MqContexts& cx, int k, int d) {
    const MqState& s = kMq[cx.idx[k]];
    a -= s.qe;
    if (d == cx.mps[k]) {  // CODEMPS
      if ((a & 0x8000) == 0) {
        if (a < s.qe) a = s.qe;
        else c += s.qe;
        cx.idx[k] = s.nmps;
        renorm();
      } else {
        c += s.qe;
      }
    } else {  // CODELPS
      if (a < s.qe) c += s.qe;
      else a = s.qe;
      if (s.sw) cx.mps[k] = (uint8_t)(1 - cx.mps[k]);
      cx.idx[k] = s.nlps;
      renorm();
    }
  }
  // FLUSH (C.2.9): SETBITS, two byte-outs, a final 0xFF dropped; returns the
  // codeword's length (bytes at out[0 ..])
  int64_t flush() {
    const uint32_t t = c + a;
    c |= 0xFFFF;
    if (c >= t) c -= 0x8000;
    c <<= ct;
    byteout();
    c <<= ct;
    byteout();
    return out[n] == 0xFF ? n : n + 1;
  }
};

// ---------------------------------------------------------------------------
// Code-block passes.  Flags per coefficient (with a one-sample border):
constexpr uint8_t kSig = 1, kNeg = 2, kVisit = 4, kRefined = 8;

// Zero-coding context (Table D.1) from the significant neighbours; orient 0
// LL, 1 HL, 2 LH, 3 HH.
J2K_HD inline int zc_ctx(int orient, int h, int v, int d) {
  if (orient == 1) {
    const int t = h;
    h = v;
    v = t;
  }
  if (orient == 3) {
    const int hv = h + v;
    if (d >= 3) return 8;
    if (d == 2) return hv >= 1 ? 7 : 6;
    if (d == 1) return hv >= 2 ? 5 : hv == 1 ? 4 : 3;
    return hv >= 2 ? 2 : hv == 1 ? 1 : 0;
  }
  if (h == 2) return 8;
  if (h == 1) return v >= 1 ? 7 : d >= 1 ? 6 : 5;
  if (v == 2) return 4;
  if (v == 1) return 3;
  return d >= 2 ? 2 : d == 1 ? 1 : 0;
}

struct CodeBlockCoder {
  int w, h, orient;
  int fs;           // flags row stride (w + 2)
  uint8_t* f;       // (w + 2) x (h + 2) flags, f0 = f + fs + 1 is sample (0, 0)
  int32_t* v;       // w x h values (decode: with the fraction bit; encode: input)
  MqContexts cx;

  uint8_t* fl(int x, int y) { return f + (y + 1) * fs + (x + 1); }
  void counts(int x, int y, int* hh, int* vv, int* dd) {
    const uint8_t* p = fl(x, y);
    *hh = (p[-1] & kSig) + (p[1] & kSig);
    *vv = (p[-fs] & kSig) + (p[fs] & kSig);
    *dd = (p[-fs - 1] & kSig) + (p[-fs + 1] & kSig) + (p[fs - 1] & kSig) + (p[fs + 1] & kSig);
  }
  bool any_sig_nb(int x, int y) {
    int a, b, c;
    counts(x, y, &a, &b, &c);
    return a + b + c != 0;
  }
  // Table D.3: sign context and the XOR bit
  int sign_ctx(int x, int y, int* xr) {
    const uint8_t* p = fl(x, y);
    auto contrib = [](uint8_t q) { return (q & kSig) ? ((q & kNeg) ? -1 : 1) : 0; };
    int H = contrib(p[-1]) + contrib(p[1]);
    int V = contrib(p[-fs]) + contrib(p[fs]);
    H = H > 0 ? 1 : H < 0 ? -1 : 0;
    V = V > 0 ? 1 : V < 0 ? -1 : 0;
    if (H == 0 && V == 0) {
      *xr = 0;
      return kCtxSc + 0;
    }
    if (H == 0) {
      *xr = V < 0;
      return kCtxSc + 1;
    }
    *xr = H < 0;
    const int hv = H * V;  // V relative to H's sign
    return kCtxSc + (hv > 0 ? 4 : hv == 0 ? 3 : 2);
  }
  int mr_ctx(int x, int y) {
    if (*fl(x, y) & kRefined) return kCtxMr + 2;
    return kCtxMr + (any_sig_nb(x, y) ? 1 : 0);
  }

  // --- decoding ---
  void dec_sig(MqDecoder& mq, int x, int y, int32_t oneplushalf) {
    int xr;
    const int sc = sign_ctx(x, y, &xr);
    const int neg = mq.decode(cx, sc) ^ xr;
    *fl(x, y) |= (uint8_t)(kSig | (neg ? kNeg : 0));
    v[y * w + x] = neg ? -oneplushalf : oneplushalf;
  }
  void dec_sigpass(MqDecoder& mq, int bpno) {
    const int32_t one = 1 << bpno, oneplushalf = one | (one >> 1);
    for (int y0 = 0; y0 < h; y0 += 4)
      for (int x = 0; x < w; x++)
        for (int y = y0; y < y0 + 4 && y < h; y++) {
          uint8_t* p = fl(x, y);
          if ((*p & kSig) || !any_sig_nb(x, y)) continue;
          int a, b, c;
          counts(x, y, &a, &b, &c);
          if (mq.decode(cx, zc_ctx(orient, a, b, c))) dec_sig(mq, x, y, oneplushalf);
          *p |= kVisit;
        }
  }
  void dec_refpass(MqDecoder& mq, int bpno) {
    const int32_t poshalf = (1 << bpno) >> 1;
    for (int y0 = 0; y0 < h; y0 += 4)
      for (int x = 0; x < w; x++)
        for (int y = y0; y < y0 + 4 && y < h; y++) {
          uint8_t* p = fl(x, y);
          if ((*p & (kSig | kVisit)) != kSig) continue;
          const int b = mq.decode(cx, mr_ctx(x, y));
          int32_t& d = v[y * w + x];
          d += (b ^ (d < 0)) ? poshalf : -poshalf;
          *p |= kRefined;
        }
  }
  void dec_clnpass(MqDecoder& mq, int bpno) {
    const int32_t one = 1 << bpno, oneplushalf = one | (one >> 1);
    for (int y0 = 0; y0 < h; y0 += 4)
      for (int x = 0; x < w; x++) {
        int y = y0;
        if (y0 + 4 <= h) {
          bool run = true;
          for (int k = 0; k < 4 && run; k++)
            run = !(*fl(x, y0 + k) & (kSig | kVisit)) && !any_sig_nb(x, y0 + k);
          if (run) {
            if (!mq.decode(cx, kCtxRl)) continue;  // the four stay insignificant
            int r = mq.decode(cx, kCtxUni) << 1;
            r |= mq.decode(cx, kCtxUni);
            y = y0 + r;
            dec_sig(mq, x, y, oneplushalf);
            y++;
          }
        }
        for (; y < y0 + 4 && y < h; y++) {
          uint8_t* p = fl(x, y);
          if (*p & (kSig | kVisit)) continue;
          int a, b, c;
          counts(x, y, &a, &b, &c);
          if (mq.decode(cx, zc_ctx(orient, a, b, c))) dec_sig(mq, x, y, oneplushalf);
        }
      }
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) *fl(x, y) &= (uint8_t)~kVisit;
  }
  // npasses passes from plane numbps - 1 (cleanup first); data followed by
  // 0xFF 0xFF; v receives the values with their fraction bit
  void decode(const uint8_t* data, int npasses, int numbps) {
    memset(f, 0, (size_t)fs * (h + 2));
    memset(v, 0, sizeof(int32_t) * (size_t)w * h);
    cx.reset();
    MqDecoder mq;
    mq.init(data);
    int bpno = numbps;  // bpno_plus_one: plane p codes with one = 2^(p+1)
    int type = 2;
    for (int pass = 0; pass < npasses && bpno >= 1; pass++) {
      if (type == 0) dec_sigpass(mq, bpno);
      else if (type == 1) dec_refpass(mq, bpno);
      else dec_clnpass(mq, bpno);
      if (++type == 3) {
        type = 0;
        bpno--;
      }
    }
  }

  // --- encoding (v holds the signed integer coefficients) ---
  int numbps_of() const {
    uint32_t m = 0;
    for (int i = 0; i < w * h; i++) m |= (uint32_t)(v[i] < 0 ? -v[i] : v[i]);
    int n = 0;
    while (m) {
      n++;
      m >>= 1;
    }
    return n;
  }
  int mag(int x, int y) const { const int32_t t = v[y * w + x]; return t < 0 ? -t : t; }
  void enc_sig(MqEncoder& mq, int x, int y) {
    int xr;
    const int sc = sign_ctx(x, y, &xr);
    const int neg = v[y * w + x] < 0;
    mq.encode(cx, sc, neg ^ xr);
    *fl(x, y) |= (uint8_t)(kSig | (neg ? kNeg : 0));
  }
  void enc_sigpass(MqEncoder& mq, int p) {
    for (int y0 = 0; y0 < h; y0 += 4)
      for (int x = 0; x < w; x++)
        for (int y = y0; y < y0 + 4 && y < h; y++) {
          uint8_t* q = fl(x, y);
          if ((*q & kSig) || !any_sig_nb(x, y)) continue;
          int a, b, c;
          counts(x, y, &a, &b, &c);
          const int bit = (mag(x, y) >> p) & 1;
          mq.encode(cx, zc_ctx(orient, a, b, c), bit);
          if (bit) enc_sig(mq, x, y);
          *q |= kVisit;
        }
  }
  void enc_refpass(MqEncoder& mq, int p) {
    for (int y0 = 0; y0 < h; y0 += 4)
      for (int x = 0; x < w; x++)
        for (int y = y0; y < y0 + 4 && y < h; y++) {
          uint8_t* q = fl(x, y);
          if ((*q & (kSig | kVisit)) != kSig) continue;
          mq.encode(cx, mr_ctx(x, y), (mag(x, y) >> p) & 1);
          *q |= kRefined;
        }
  }
  void enc_clnpass(MqEncoder& mq, int p) {
    for (int y0 = 0; y0 < h; y0 += 4)
      for (int x = 0; x < w; x++) {
        int y = y0;
        if (y0 + 4 <= h) {
          bool run = true;
          for (int k = 0; k < 4 && run; k++)
            run = !(*fl(x, y0 + k) & (kSig | kVisit)) && !any_sig_nb(x, y0 + k);
          if (run) {
            int r = -1;
            for (int k = 0; k < 4 && r < 0; k++)
              if ((mag(x, y0 + k) >> p) & 1) r = k;
            if (r < 0) {
              mq.encode(cx, kCtxRl, 0);
              continue;
            }
            mq.encode(cx, kCtxRl, 1);
            mq.encode(cx, kCtxUni, r >> 1);
            mq.encode(cx, kCtxUni, r & 1);
            y = y0 + r;
            enc_sig(mq, x, y);
            y++;
          }
        }
        for (; y < y0 + 4 && y < h; y++) {
          uint8_t* q = fl(x, y);
          if (*q & (kSig | kVisit)) continue;
          int a, b, c;
          counts(x, y, &a, &b, &c);
          const int bit = (mag(x, y) >> p) & 1;
          mq.encode(cx, zc_ctx(orient, a, b, c), bit);
          if (bit) enc_sig(mq, x, y);
        }
      }
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) *fl(x, y) &= (uint8_t)~kVisit;
  }
  // every pass of every plane into one codeword; buf has room for
  // 2 * w * h * 32 / 8 + 64 bytes (its first byte is scratch); returns the
  // length of the codeword at buf + 1, *npasses the number of passes
  int64_t encode(uint8_t* buf, int numbps, int* npasses) {
    memset(f, 0, (size_t)fs * (h + 2));
    cx.reset();
    MqEncoder mq;
    mq.init(buf);
    int n = 0;
    for (int p = numbps - 1; p >= 0; p--) {
      if (p != numbps - 1) {
        enc_sigpass(mq, p);
        enc_refpass(mq, p);
        n += 2;
      }
      enc_clnpass(mq, p);
      n++;
    }
    *npasses = n;
    return mq.flush();
  }
};

}  // namespace j2k
}  // namespace uph
