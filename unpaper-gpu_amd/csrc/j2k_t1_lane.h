// j2k_t1_lane.h — the EBCOT code-block decoder (j2k_t1.h's passes) written
// for a wave that decodes 64 code-blocks at once, one a lane.  Every lane
// walks the same positions in the same order (pass k of every lane is the
// same pass type: cleanup first, then significance / refinement / cleanup
// per plane, whatever each lane's top plane), so the lanes' state can be laid
// out lane-minor and every load or store of it is one coalesced access:
//   flags  one 16-bit word per 4-sample stripe column (bits 4r + {0 sig,
//          1 negative, 2 visited this plane, 3 refined}), rows of Wg + 2
//          words with a zero border (stripe -1 / Sg, column -1 / Wg);
//   values uint32 per sample, rows of Wg: the magnitude bits decoded so far
//          (bpno_plus_one units, no fraction bit), stored when the sample
//          becomes significant and OR-ed by each refinement -- written, never
//          read, until the block is stored; the sign is in the flags and the
//          fraction bit (OpenJPEG's reconstruction point) is added at the end
//          from the lowest refinement plane decoded;
//   MQ     19 context bytes (index | MPS << 7) per lane, registers A, C, CT
//          and the byte pointer per lane.
// Lanes past their block's width, height or pass count only predicate their
// work.  With LS = 1 the same code decodes one block on the host (the CPU
// emulator, tests/c/j2k_emul.cpp).
#pragma once

#include <stdint.h>

#include "j2k_t1.h"

#ifndef J2K_HD
#define J2K_HD __host__ __device__
#endif

namespace uph {
namespace j2k {

// One code-block for the device decoder (j2k.cpp builds them, sorted so the
// 64 of a wave are alike in shape and pass count).
struct T1Job {
  uint32_t data;     // byte offset of the codeword, followed by 0xFF 0xFF
  uint32_t len;
  int64_t out;       // element offset of sample (0, 0) in the coefficient buffer
  int32_t stride;    // plane row stride (elements)
  uint16_t w, h;
  uint8_t orient, numbps, npasses, pad;
  float halfstep;    // irreversible: 0.5 * quantisation step; 0: reversible
};

// zero-coding contexts for (orient, h, v, d): [orient * 45 + h * 15 + v * 5 + d]
constexpr int kZcTable = 4 * 45;
inline void zc_table(uint8_t* t) {
  for (int o = 0; o < 4; o++)
    for (int h = 0; h < 3; h++)
      for (int v = 0; v < 3; v++)
        for (int d = 0; d < 5; d++) t[o * 45 + h * 15 + v * 5 + d] = (uint8_t)zc_ctx(o, h, v, d);
}

J2K_HD inline uint32_t t1_sig4(uint32_t w) {
  return (w & 1u) | ((w >> 3) & 2u) | ((w >> 6) & 4u) | ((w >> 9) & 8u);
}
// rows -1 .. 4 of a column (bit i = row i - 1): row 3 of the stripe above,
// the stripe's four, row 0 of the stripe below; sig (shift 0) or neg (1)
J2K_HD inline uint32_t t1_six(uint32_t u, uint32_t m, uint32_t d, int sh) {
  return ((u >> (12 + sh)) & 1u) | (t1_sig4(m >> sh) << 1) | (((d >> sh) & 1u) << 5);
}

// The type and plane of pass k (cleanup at numbps first): type 0 SPP, 1 MRP,
// 2 CUP; bpno in bpno_plus_one units (decoding stops below 1).
J2K_HD inline void t1_pass(int k, int numbps, int* type, int* bpno) {
  if (k == 0) {
    *type = 2;
    *bpno = numbps;
  } else {
    *type = (k - 1) % 3;
    *bpno = numbps - 1 - (k - 1) / 3;
  }
}

template <int LS>
struct T1Lane {
  // wave-uniform geometry
  int WS, Wg;  // flag row stride (Wg + 2), value row stride (Wg)
  uint16_t* fl;
  uint32_t* val;
  uint8_t* cx;
  const MqState* qe;
  const uint8_t* zct;
  // this lane's block
  int w, h, orient;
  int pm;  // lowest plane whose refinement pass was decoded (1 << 30: none)
  // MQ decoder; the codeword is read through a 12-byte window of aligned
  // words (w0 at q, w1, w2), the word 8 bytes ahead loaded when the window
  // moves, long before its bytes are needed
  const uint32_t* q;  // 4-byte aligned
  uint32_t w0, w1, w2;
  int bi;             // offset of the current byte (BP) from q: 0 .. 3
  uint32_t a, c;
  int ct;

  J2K_HD uint16_t& F(int s, int col) const { return fl[(int64_t)((s + 1) * WS + col + 1) * LS]; }
  J2K_HD uint32_t& V(int y, int x) const { return val[(int64_t)(y * Wg + x) * LS]; }
  // a refinement bit into the sample's magnitude (the device's lanes OR
  // with a no-return atomic: nothing waits for it)
  J2K_HD void vor(int y, int x, uint32_t bits) const {
#if defined(UPH_T1_NOVAL)  // timing variant: no value traffic (wrong output)
    (void)y, (void)x, (void)bits;
#elif defined(__HIP_DEVICE_COMPILE__)
    __hip_atomic_fetch_or(&V(y, x), bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
    V(y, x) |= bits;
#endif
  }

  // bytes BP and BP + 1 (bi + 1 <= 4 < 8)
  J2K_HD uint32_t byte_at(int i) const {
    const uint64_t v = ((uint64_t)w1 << 32) | w0;
    return (uint32_t)(v >> (8 * i)) & 0xFFu;
  }
  J2K_HD void advance() {  // BP++
    if (++bi == 4) {
      bi = 0;
      q++;
      w0 = w1;
      w1 = w2;
      w2 = q[2];
    }
  }
  J2K_HD void bytein() {
    if (byte_at(bi) == 0xFF) {
      if (byte_at(bi + 1) > 0x8F) {
        c += 0xFF00;
        ct = 8;
      } else {
        advance();
        c += byte_at(bi) << 9;
        ct = 7;
      }
    } else {
      advance();
      c += byte_at(bi) << 8;
      ct = 8;
    }
  }
  // data: 4-byte aligned, readable 12 bytes past the codeword's FF FF
  J2K_HD void mq_init(const uint8_t* data) {
    q = reinterpret_cast<const uint32_t*>(data);
    w0 = q[0];
    w1 = q[1];
    w2 = q[2];
    bi = 0;
    c = byte_at(0) << 16;
    bytein();
    c <<= 7;
    ct -= 7;
    a = 0x8000;
  }
  // RENORMD in chunks: the count of doublings that bring A to 0x8000 from
  // its leading zeros, applied up to the next byte boundary at a time (the
  // one-bit loop of C.3.3 would run up to 15 turns, and a wave takes every
  // turn any lane needs)
  J2K_HD void renorm() {
    int n = __builtin_clz(a) - 16;
    while (n > 0) {
      if (ct == 0) bytein();
      const int k = n < ct ? n : ct;
      a <<= k;
      c <<= k;
      ct -= k;
      n -= k;
    }
  }
  // MqDecoder::decode with the context byte in memory
  J2K_HD int dec(int k) {
    uint8_t& e = cx[k * LS];
    const uint32_t ent = e;
    const MqState s = qe[ent & 63u];
    const uint32_t mps = ent >> 7, flip = s.sw ? 1u - mps : mps;
    a -= s.qe;
    int d;
    if ((c >> 16) < s.qe) {  // LPS_EXCHANGE
      if (a < s.qe) {
        d = (int)mps;
        e = (uint8_t)(s.nmps | (mps << 7));
      } else {
        d = (int)(1u - mps);
        e = (uint8_t)(s.nlps | (flip << 7));
      }
      a = s.qe;
      renorm();
      return d;
    }
    c -= (uint32_t)s.qe << 16;
    if (a & 0x8000) return (int)mps;
    if (a < s.qe) {  // MPS_EXCHANGE
      d = (int)(1u - mps);
      e = (uint8_t)(s.nlps | (flip << 7));
    } else {
      d = (int)mps;
      e = (uint8_t)(s.nmps | (mps << 7));
    }
    renorm();
    return d;
  }
  J2K_HD void reset_contexts() {
    for (int k = 0; k < kNumCtx; k++) cx[k * LS] = 0;
    cx[kCtxUni * LS] = 46;
    cx[kCtxRl * LS] = 3;
    cx[0] = 4;
  }

  // sign decode of row r of the column (sig vectors L6/M6/R6, neg vectors
  // LN/MN/RN of the column's neighbourhood), then the sample is significant
  J2K_HD void dec_sign(int r, int y, int x, uint32_t one, uint32_t L6, uint32_t M6, uint32_t R6,
                       uint32_t LN, uint32_t MN, uint32_t RN, uint32_t* Mc) {
    auto contrib = [](uint32_t s6, uint32_t n6, int row) -> int {
      return ((s6 >> row) & 1u) ? (((n6 >> row) & 1u) ? -1 : 1) : 0;
    };
    int H = contrib(L6, LN, r + 1) + contrib(R6, RN, r + 1);
    int Vv = contrib(M6, MN, r) + contrib(M6, MN, r + 2);
    H = H > 0 ? 1 : H < 0 ? -1 : 0;
    Vv = Vv > 0 ? 1 : Vv < 0 ? -1 : 0;
    int ctx, xr;
    if (H == 0 && Vv == 0) {
      ctx = kCtxSc;
      xr = 0;
    } else if (H == 0) {
      ctx = kCtxSc + 1;
      xr = Vv < 0;
    } else {
      xr = H < 0;
      const int hv = H * Vv;
      ctx = kCtxSc + (hv > 0 ? 4 : hv == 0 ? 3 : 2);
    }
    const int neg = dec(ctx) ^ xr;
    *Mc |= (uint32_t)(1 | (neg << 1)) << (4 * r);
#ifndef UPH_T1_NOVAL
    V(y, x) = one;
#endif
  }

  // one stripe column of pass `type` at plane bpno (bpno_plus_one units)
  J2K_HD void column(int type, int bpno, int s, int col, uint32_t Ul, uint32_t Ml, uint32_t Dl,
                     uint32_t Uc, uint32_t* Mc, uint32_t Dc, uint32_t Ur, uint32_t Mr, uint32_t Dr) {
    const int rows = h - 4 * s < 4 ? h - 4 * s : 4;
    const uint32_t L6 = t1_six(Ul, Ml, Dl, 0), R6 = t1_six(Ur, Mr, Dr, 0);
    const uint32_t one = 1u << bpno;
    auto nb = [&](uint32_t M6, int r) -> uint32_t {
      return (((L6 | R6) >> r) & 7u) | ((M6 >> r) & 5u);
    };
    auto zc = [&](uint32_t M6, int r) -> int {
      const int hh = (int)(((L6 >> (r + 1)) & 1u) + ((R6 >> (r + 1)) & 1u));
      const int vv = (int)(((M6 >> r) & 1u) + ((M6 >> (r + 2)) & 1u));
      const int dd = (int)(((L6 >> r) & 1u) + ((L6 >> (r + 2)) & 1u) + ((R6 >> r) & 1u) +
                           ((R6 >> (r + 2)) & 1u));
      return zct[orient * 45 + hh * 15 + vv * 5 + dd];
    };
    auto sig_at = [&](int r) {
      const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
      dec_sign(r, 4 * s + r, col, one, L6, M6, R6, t1_six(Ul, Ml, Dl, 1), t1_six(Uc, *Mc, Dc, 1),
               t1_six(Ur, Mr, Dr, 1), Mc);
    };
    if (type == 0) {  // significance propagation
      for (int r = 0; r < rows; r++) {
        if ((*Mc >> (4 * r)) & 1u) continue;
        const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
        if (!nb(M6, r)) continue;
        if (dec(zc(M6, r))) sig_at(r);
        *Mc |= 4u << (4 * r);
      }
    } else if (type == 1) {  // magnitude refinement
      for (int r = 0; r < rows; r++) {
        if (((*Mc >> (4 * r)) & 5u) != 1u) continue;  // significant, not visited
        const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
        const int ctx = ((*Mc >> (4 * r)) & 8u) ? kCtxMr + 2 : kCtxMr + (nb(M6, r) ? 1 : 0);
        if (dec(ctx)) vor(4 * s + r, col, one);
        *Mc |= 8u << (4 * r);
      }
    } else {  // cleanup
      int r0 = 0;
      bool done = false;
      if (rows == 4 && (*Mc & 0x5555u) == 0u) {
        const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
        if (!nb(M6, 0) && !nb(M6, 1) && !nb(M6, 2) && !nb(M6, 3)) {
          if (!dec(kCtxRl)) {
            done = true;
          } else {
            int r = dec(kCtxUni) << 1;
            r |= dec(kCtxUni);
            sig_at(r);
            r0 = r + 1;
          }
        }
      }
      if (!done)
        for (int r = r0; r < rows; r++) {
          if ((*Mc >> (4 * r)) & 5u) continue;  // significant or visited
          const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
          if (dec(zc(M6, r))) sig_at(r);
        }
      *Mc &= ~0x4444u;
    }
  }
};

// Decodes the lane's block (lockstep over the wave: every lane runs every
// loop; `any` is the wave-wide OR of a predicate, so passes no lane takes are
// skipped).  Flags of stripes [-1, Sg] x columns [-1, Wg] are zeroed first.
template <int LS, class Any>
J2K_HD void t1_decode_lane(T1Lane<LS>& L, bool active, const uint8_t* data, int numbps,
                           int npasses, int Sg, int maxpasses, Any any);

// ---------------------------------------------------------------------------
// The encoder, a lane per code-block the same way (j2k_t1.h's enc_* passes):
// the block's magnitudes as four 16-bit rows per stripe column (one 8-byte
// word a column, lane-minor), the flags as above with every sample's sign
// preset (a sign only counts once the sample is significant), the MQ
// encoder's registers per lane and its bytes into the lane's output region.
struct T1EncJob {
  int64_t in;      // element offset of sample (0, 0) in the coefficient buffer (int32)
  int32_t stride;  // plane row stride (elements)
  uint16_t w, h;
  uint32_t out;    // byte offset of the block's output region (t1_enc_cap bytes)
  uint8_t orient, pad[3];
};
// output bytes a block's region holds: two a sample (lossless 8-bit data
// codes to ~1 byte a sample at worst, random noise) and the flush; a block
// that needs more is reported (T1EncLane::over), not written past its region
J2K_HD inline uint32_t t1_enc_cap(int w, int h) { return (uint32_t)(w * h * 2 + 256); }

template <int LS>
struct T1EncLane {
  int WS, Wg;
  uint16_t* fl;          // flags, as T1Lane
  const uint64_t* mg;    // magnitudes: word (s * Wg + col) * LS, row r in bits 16 r
  uint8_t* cx;
  const MqState* qe;
  const uint8_t* zct;
  int w, h, orient;
  // MQ encoder (C.2): the last byte emitted is kept in `last` (its index n);
  // bytes past `cap` are counted, not stored, and set `over`
  uint8_t* out;
  int32_t n, cap;
  bool over;
  uint32_t last;
  uint32_t a, c;
  int ct;

  J2K_HD uint16_t& F(int s, int col) const { return fl[(int64_t)((s + 1) * WS + col + 1) * LS]; }
  J2K_HD uint64_t M4(int s, int col) const { return mg[(int64_t)(s * Wg + col) * LS]; }

  J2K_HD void init() {
    n = -1;
    over = false;
    last = 0;
    a = 0x8000;
    c = 0;
    ct = 12;
  }
  J2K_HD void emit(uint32_t b) {
    if (++n < cap) out[n] = (uint8_t)b;
    else over = true;
    last = b;
  }
  J2K_HD void byteout() {
    if (last == 0xFF) {
      emit(c >> 20);
      c &= 0xFFFFF;
      ct = 7;
    } else if (c < 0x8000000) {
      emit(c >> 19);
      c &= 0x7FFFF;
      ct = 8;
    } else {
      last++;  // the carry into the byte already out
      if (n >= 0 && n < cap) out[n] = (uint8_t)last;
      if (last == 0xFF) {
        c &= 0x7FFFFFF;
        emit(c >> 20);
        c &= 0xFFFFF;
        ct = 7;
      } else {
        emit(c >> 19);
        c &= 0x7FFFF;
        ct = 8;
      }
    }
  }
  // RENORME in chunks up to each byte-out, as the decoder's
  J2K_HD void renorm() {
    int n = __builtin_clz(a) - 16;
    while (n > 0) {
      const int k = n < ct ? n : ct;
      a <<= k;
      c <<= k;
      ct -= k;
      n -= k;
      if (ct == 0) byteout();
    }
  }
  J2K_HD void enc(int k, int d) {
    uint8_t& e = cx[k * LS];
    const uint32_t ent = e;
    const MqState s = qe[ent & 63u];
    const uint32_t mps = ent >> 7;
    a -= s.qe;
    if ((uint32_t)d == mps) {  // CODEMPS
      if ((a & 0x8000) == 0) {
        if (a < s.qe) a = s.qe;
        else c += s.qe;
        e = (uint8_t)(s.nmps | (mps << 7));
        renorm();
      } else {
        c += s.qe;
      }
    } else {  // CODELPS
      if (a < s.qe) c += s.qe;
      else a = s.qe;
      e = (uint8_t)(s.nlps | ((s.sw ? 1u - mps : mps) << 7));
      renorm();
    }
  }
  // FLUSH (C.2.9); the codeword's length (a final 0xFF dropped)
  J2K_HD int32_t flush() {
    const uint32_t t = c + a;
    c |= 0xFFFF;
    if (c >= t) c -= 0x8000;
    c <<= ct;
    byteout();
    c <<= ct;
    byteout();
    return last == 0xFF ? n : n + 1;
  }
  J2K_HD void reset_contexts() {
    for (int k = 0; k < kNumCtx; k++) cx[k * LS] = 0;
    cx[kCtxUni * LS] = 46;
    cx[kCtxRl * LS] = 3;
    cx[0] = 4;
  }

  J2K_HD void enc_sign(int r, uint32_t L6, uint32_t M6, uint32_t R6, uint32_t LN, uint32_t MN,
                       uint32_t RN, uint32_t* Mc) {
    auto contrib = [](uint32_t s6, uint32_t n6, int row) -> int {
      return ((s6 >> row) & 1u) ? (((n6 >> row) & 1u) ? -1 : 1) : 0;
    };
    int H = contrib(L6, LN, r + 1) + contrib(R6, RN, r + 1);
    int Vv = contrib(M6, MN, r) + contrib(M6, MN, r + 2);
    H = H > 0 ? 1 : H < 0 ? -1 : 0;
    Vv = Vv > 0 ? 1 : Vv < 0 ? -1 : 0;
    int ctx, xr;
    if (H == 0 && Vv == 0) {
      ctx = kCtxSc;
      xr = 0;
    } else if (H == 0) {
      ctx = kCtxSc + 1;
      xr = Vv < 0;
    } else {
      xr = H < 0;
      const int hv = H * Vv;
      ctx = kCtxSc + (hv > 0 ? 4 : hv == 0 ? 3 : 2);
    }
    const int neg = (int)((*Mc >> (4 * r + 1)) & 1u);
    enc(ctx, neg ^ xr);
    *Mc |= 1u << (4 * r);
  }

  // one stripe column of pass `type` at magnitude plane p; m4 its magnitudes
  J2K_HD void column(int type, int p, int s, uint64_t m4, uint32_t Ul, uint32_t Ml, uint32_t Dl,
                     uint32_t Uc, uint32_t* Mc, uint32_t Dc, uint32_t Ur, uint32_t Mr, uint32_t Dr) {
    const int rows = h - 4 * s < 4 ? h - 4 * s : 4;
    const uint32_t L6 = t1_six(Ul, Ml, Dl, 0), R6 = t1_six(Ur, Mr, Dr, 0);
    auto bit = [&](int r) -> int { return (int)((m4 >> (16 * r + p)) & 1u); };
    auto nb = [&](uint32_t M6, int r) -> uint32_t {
      return (((L6 | R6) >> r) & 7u) | ((M6 >> r) & 5u);
    };
    auto zc = [&](uint32_t M6, int r) -> int {
      const int hh = (int)(((L6 >> (r + 1)) & 1u) + ((R6 >> (r + 1)) & 1u));
      const int vv = (int)(((M6 >> r) & 1u) + ((M6 >> (r + 2)) & 1u));
      const int dd = (int)(((L6 >> r) & 1u) + ((L6 >> (r + 2)) & 1u) + ((R6 >> r) & 1u) +
                           ((R6 >> (r + 2)) & 1u));
      return zct[orient * 45 + hh * 15 + vv * 5 + dd];
    };
    auto sig_at = [&](int r) {
      enc_sign(r, L6, t1_six(Uc, *Mc, Dc, 0), R6, t1_six(Ul, Ml, Dl, 1), t1_six(Uc, *Mc, Dc, 1),
               t1_six(Ur, Mr, Dr, 1), Mc);
    };
    if (type == 0) {  // significance propagation
      for (int r = 0; r < rows; r++) {
        if ((*Mc >> (4 * r)) & 1u) continue;
        const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
        if (!nb(M6, r)) continue;
        const int b = bit(r);
        enc(zc(M6, r), b);
        if (b) sig_at(r);
        *Mc |= 4u << (4 * r);
      }
    } else if (type == 1) {  // magnitude refinement
      for (int r = 0; r < rows; r++) {
        if (((*Mc >> (4 * r)) & 5u) != 1u) continue;
        const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
        const int ctx = ((*Mc >> (4 * r)) & 8u) ? kCtxMr + 2 : kCtxMr + (nb(M6, r) ? 1 : 0);
        enc(ctx, bit(r));
        *Mc |= 8u << (4 * r);
      }
    } else {  // cleanup
      int r0 = 0;
      bool done = false;
      if (rows == 4 && (*Mc & 0x5555u) == 0u) {
        const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
        if (!nb(M6, 0) && !nb(M6, 1) && !nb(M6, 2) && !nb(M6, 3)) {
          int r = -1;
          for (int k = 0; k < 4 && r < 0; k++)
            if (bit(k)) r = k;
          if (r < 0) {
            enc(kCtxRl, 0);
            done = true;
          } else {
            enc(kCtxRl, 1);
            enc(kCtxUni, r >> 1);
            enc(kCtxUni, r & 1);
            sig_at(r);
            r0 = r + 1;
          }
        }
      }
      if (!done)
        for (int r = r0; r < rows; r++) {
          if ((*Mc >> (4 * r)) & 5u) continue;
          const uint32_t M6 = t1_six(Uc, *Mc, Dc, 0);
          const int b = bit(r);
          enc(zc(M6, r), b);
          if (b) sig_at(r);
        }
      *Mc &= ~0x4444u;
    }
  }
};

// Encodes the lane's block (nb magnitude planes, every pass), lockstep over
// the wave like t1_decode_lane; flags must hold the preset signs (and zero
// elsewhere, the border included).  Returns the codeword's length.
template <int LS, class Any>
J2K_HD int32_t t1_encode_lane(T1EncLane<LS>& L, bool active, int nb, int Sg, int maxpasses,
                              Any any) {
  if (active) {
    L.reset_contexts();
    L.init();
  }
  for (int k = 0; k < maxpasses; k++) {
    int type, p;
    t1_pass(k, nb - 1, &type, &p);  // plane p in magnitude units
    const bool on = active && k < 3 * nb - 2;
    if (!any(on)) continue;
    for (int s = 0; s < Sg; s++) {
      uint32_t Ul = 0, Ml = 0, Dl = 0;
      uint32_t Uc = L.F(s - 1, 0), Mc = L.F(s, 0), Dc = L.F(s + 1, 0);
      uint32_t Ur = L.F(s - 1, 1), Mr = L.F(s, 1), Dr = L.F(s + 1, 1);
      const bool srow = on && 4 * s < L.h;
      uint64_t m4 = srow ? L.M4(s, 0) : 0, m4n = 0;
      for (int col = 0; col < L.Wg; col++) {
        uint32_t Un = 0, Mn = 0, Dn = 0;
        if (col + 2 <= L.Wg) {
          Un = L.F(s - 1, col + 2);
          Mn = L.F(s, col + 2);
          Dn = L.F(s + 1, col + 2);
        }
        if (srow && col + 1 < L.Wg) m4n = L.M4(s, col + 1);
        if (srow && col < L.w) {
          L.column(type, p, s, m4, Ul, Ml, Dl, Uc, &Mc, Dc, Ur, Mr, Dr);
          L.F(s, col) = (uint16_t)Mc;
        }
        m4 = m4n;
        Ul = Uc;
        Uc = Ur;
        Ur = Un;
        Ml = Mc;
        Mc = Mr;
        Mr = Mn;
        Dl = Dc;
        Dc = Dr;
        Dr = Dn;
      }
    }
  }
  return active ? L.flush() : 0;
}

template <int LS, class Any>
J2K_HD void t1_decode_lane(T1Lane<LS>& L, bool active, const uint8_t* data, int numbps,
                           int npasses, int Sg, int maxpasses, Any any) {
  for (int i = 0; i < (Sg + 2) * L.WS; i++) L.fl[(int64_t)i * LS] = 0;
  L.pm = 1 << 30;
  if (active) {
    L.reset_contexts();
    L.mq_init(data);
  }
  for (int k = 0; k < maxpasses; k++) {
    int type, bpno;
    t1_pass(k, numbps, &type, &bpno);
    const bool on = active && k < npasses && bpno >= 1;
    if (!any(on)) continue;
    if (on && type == 1) L.pm = bpno;
    for (int s = 0; s < Sg; s++) {
      // the three stripes' words of columns col - 1 .. col + 1, and col + 2
      // in flight (the row's border column Wg + 1 ends every row)
      uint32_t Ul = 0, Ml = 0, Dl = 0;  // column -1: the border
      uint32_t Uc = L.F(s - 1, 0), Mc = L.F(s, 0), Dc = L.F(s + 1, 0);
      uint32_t Ur = L.F(s - 1, 1), Mr = L.F(s, 1), Dr = L.F(s + 1, 1);
      const bool srow = on && 4 * s < L.h;
      for (int col = 0; col < L.Wg; col++) {
        uint32_t Un = 0, Mn = 0, Dn = 0;
        if (col + 2 <= L.Wg) {
          Un = L.F(s - 1, col + 2);
          Mn = L.F(s, col + 2);
          Dn = L.F(s + 1, col + 2);
        }
        if (srow && col < L.w) {
          L.column(type, bpno, s, col, Ul, Ml, Dl, Uc, &Mc, Dc, Ur, Mr, Dr);
          L.F(s, col) = (uint16_t)Mc;
        }
        Ul = Uc;
        Uc = Ur;
        Ur = Un;
        Ml = Mc;
        Mc = Mr;
        Mr = Mn;
        Dl = Dc;
        Dc = Dr;
        Dr = Dn;
      }
    }
  }
}

// The decoded block into the coefficient buffer: reversible values halved
// (the fraction bit), irreversible ones scaled by half the step (as float
// bits); samples never significant are 0.
template <int LS>
J2K_HD void t1_store_lane(const T1Lane<LS>& L, bool active, const T1Job& job, uint32_t* coef,
                          int Hg) {
  for (int y = 0; y < Hg; y++)
    for (int x = 0; x < L.Wg; x++) {
      if (!active || y >= L.h || x >= L.w) continue;
      const uint32_t wd = (uint32_t)L.F(y >> 2, x) >> (4 * (y & 3));
      int32_t q = 0;
      if (wd & 1u) {
        // magnitude bits, then the fraction bit below the last plane decoded
        // for the sample: its significance plane, or the lowest refinement
        // plane under it
        const uint32_t m = L.V(y, x);
        const int p0 = 31 - __builtin_clz(m);
        const int pl = p0 < L.pm ? p0 : L.pm;
        const int32_t mag = (int32_t)(m | (1u << pl >> 1));
        q = (wd & 2u) ? -mag : mag;
      }
      uint32_t o;
      if (job.halfstep == 0.0f) {
        o = (uint32_t)(q / 2);
      } else {
        const float f = (float)q * job.halfstep;
        o = __builtin_bit_cast(uint32_t, f);
      }
      coef[job.out + (int64_t)y * job.stride + x] = o;
    }
}

}  // namespace j2k
}  // namespace uph
