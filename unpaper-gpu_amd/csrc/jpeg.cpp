// jpeg.cpp — host half of the JPEG decode peer (see jpeg.h):
// marker parsing and Huffman decoding into the packed coefficient layout the
// device kernels (kernels_jpeg.hip) turn into pixels.
//
// Reference: the reference decodes JPEG inputs with FFmpeg (file.c:29-128,
// the batch decode queue's swscale conversion in sheet_stages.c:99-122) and
// with nvImageCodec on its GPU path (imageprocess/nvimgcodec.c:679-1007,
// nvimgcodec_decode / _decode_file / _decode_batch).  Decoding follows ITU-T
// T.81 (baseline and extended sequential Huffman, Annex F) with libjpeg's
// conventions where T.81 leaves room: the colour transform from the JFIF /
// Adobe markers or component ids (jdapimin.c default_decompress_parms),
// component geometry (jdinput.c initial_setup, per_scan_setup).
#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "jpeg.h"
#include "runtime.h"

namespace uph {

namespace {

constexpr int kLook = 10;  // Huffman lookahead bits

struct Huff {
  bool present = false;
  uint16_t look[1 << kLook];  // len << 8 | symbol, 0 = longer code
  // AC tables: a whole coefficient per lookahead when its code and magnitude
  // bits fit: bits 0-4 bits consumed, 5-8 run, 9 end-of-block, 16-31 value
  // (0 = take the general path)
  uint32_t fast[1 << kLook];
  int32_t maxcode[18];        // largest code of each length, -1 if none
  int32_t valptr[17];
  int32_t mincode[17];
  uint8_t vals[256];
};

bool build_huff(Huff* t, const uint8_t* bits /*16*/, const uint8_t* vals, int nvals) {
  memset(t->look, 0, sizeof(t->look));
  memcpy(t->vals, vals, (size_t)nvals);
  int code = 0, k = 0;
  for (int len = 1; len <= 16; len++) {
    t->valptr[len] = k;
    t->mincode[len] = code;
    for (int i = 0; i < bits[len - 1]; i++, k++, code++) {
      // an over-subscribed table (more codes of this length than 2^len)
      // is refused before its codes index the lookahead table
      if (code >= (1 << len)) return false;
      if (len <= kLook) {
        const int shift = kLook - len;
        for (int j = 0; j < (1 << shift); j++)
          t->look[(code << shift) | j] = (uint16_t)(len << 8 | vals[k]);
      }
    }
    t->maxcode[len] = bits[len - 1] ? code - 1 : -1;
    code <<= 1;
  }
  t->maxcode[17] = 0x7fffffff;
  t->present = true;
  for (int p = 0; p < (1 << kLook); p++) {
    const uint16_t e = t->look[p];
    t->fast[p] = 0;
    if (!e) continue;
    const int len = e >> 8, rs = e & 0xff, r = rs >> 4, sz = rs & 15;
    if (rs == 0) {  // end of block
      t->fast[p] = (uint32_t)len | 1u << 9;
    } else if (sz && len + sz <= kLook) {
      const uint32_t m = ((uint32_t)p >> (kLook - len - sz)) & ((1u << sz) - 1u);
      const int v = m < (1u << (sz - 1)) ? (int)m - (1 << sz) + 1 : (int)m;
      t->fast[p] = (uint32_t)(len + sz) | (uint32_t)r << 5 | (uint32_t)(uint16_t)(int16_t)v << 16;
    }
  }
  return true;
}

// MSB-first bit reader over entropy-coded data: byte stuffing removed; at a
// marker it feeds zero bits (libjpeg's behaviour for corrupt data) and stops.
struct Bits {
  const uint8_t* p;
  const uint8_t* end;
  uint64_t buf = 0;
  int n = 0;
  int fed = 0;  // zero bytes fed past a marker or the end of the data
  bool marker = false;
  // true when decoding consumed fed zeros: the data ended (or a marker came)
  // inside the entropy-coded segment
  bool underrun() const { return n < 8 * fed; }
  void fill() {
    // fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker): as
    // many whole bytes as fit in one go
    if (!marker && p + 8 <= end) {
      uint64_t w;
      memcpy(&w, p, 8);
      w = __builtin_bswap64(w);
      const uint64_t nw = ~w;
      if (!((nw - 0x0101010101010101ull) & ~nw & 0x8080808080808080ull)) {
        const int take = (63 - n) >> 3;  // n + 8 take <= 63
        if (take > 0) {
          buf |= (w >> (64 - 8 * take)) << (64 - n - 8 * take);
          p += take;
          n += 8 * take;
        }
        return;
      }
    }
    while (n <= 56) {
      uint32_t byte = 0;
      if (marker || p >= end) fed++;
      if (!marker && p < end) {
        byte = *p;
        if (byte == 0xFF) {
          if (p + 1 < end && p[1] == 0x00) {
            p += 2;
          } else {
            marker = true;  // leave p at the marker
            fed++;
            byte = 0;
          }
        } else {
          p++;
        }
      }
      buf |= (uint64_t)byte << (56 - n);
      n += 8;
    }
  }
  uint32_t get(int s) {  // s in 1..16
    if (n < s) fill();
    const uint32_t v = (uint32_t)(buf >> (64 - s));
    buf <<= s;
    n -= s;
    return v;
  }
  int decode(const Huff& t) {
    if (n < 16) fill();
    const uint16_t e = t.look[buf >> (64 - kLook)];
    if (e) {
      const int len = e >> 8;
      buf <<= len;
      n -= len;
      return e & 0xff;
    }
    for (int len = kLook + 1; len <= 16; len++) {
      const int32_t code = (int32_t)(buf >> (64 - len));
      if (code <= t.maxcode[len]) {
        buf <<= len;
        n -= len;
        return t.vals[t.valptr[len] + code - t.mincode[len]];
      }
    }
    return -1;  // no such code: corrupt data
  }
  void reset() {  // byte-align at a restart marker
    buf = 0;
    n = 0;
    fed = 0;
    marker = false;
  }
};

inline int extend(uint32_t v, int s) {
  return v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v;
}

uint16_t be16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }

struct Parser {
  const uint8_t* d;
  size_t n;
  const char* name;
  size_t pos = 0;
  // frame
  bool have_frame = false;
  int sof = -1;
  int w = 0, h = 0, nf = 0;
  int cid[4] = {}, hs[4] = {}, vs[4] = {}, tq[4] = {};
  uint16_t qt[4][64];  // zigzag order
  bool have_qt[4] = {};
  bool latched[4] = {};
  Huff dc[4], ac[4];
  int restart = 0;
  bool jfif = false, adobe = false;
  int adobe_transform = -1;
  // progressive (SOF2): every component's coefficients, zigzag order, over
  // its MCU-padded blocks (bw x bh), refined scan after scan
  bool progressive = false;
  std::vector<int16_t> pc[3];
  // device entropy decoding (jpeg_stream_prepare): the one scan's data is
  // copied, not decoded; a file that needs more (progressive, more scans)
  // sets not_device
  JdecStreamHost* stream = nullptr;
  bool not_device = false;
};

bool ffail(const Parser& P, const char* what) {
  return fail("jpeg: %s: %s", P.name, what);
}

// Reads the next marker code at P.pos (skipping fill bytes); -1 at the end.
int next_marker(Parser& P) {
  while (P.pos < P.n && P.d[P.pos] != 0xFF) P.pos++;  // tolerate garbage between segments
  while (P.pos < P.n && P.d[P.pos] == 0xFF) P.pos++;
  if (P.pos >= P.n) return -1;
  return P.d[P.pos++];
}

bool segment(Parser& P, const uint8_t** body, int* len) {
  if (P.pos + 2 > P.n) return ffail(P, "truncated segment");
  const int L = be16(P.d + P.pos);
  if (L < 2 || P.pos + (size_t)L > P.n) return ffail(P, "bad segment length");
  *body = P.d + P.pos + 2;
  *len = L - 2;
  P.pos += (size_t)L;
  return true;
}

bool parse_sof(Parser& P, int code, const uint8_t* b, int len) {
  if (P.have_frame) return ffail(P, "more than one frame");
  if (code != 0xC0 && code != 0xC1 && code != 0xC2) {
    if (code >= 0xC9) return ffail(P, "arithmetic-coded JPEG is not supported");
    return ffail(P, "lossless / hierarchical JPEG is not supported");
  }
  P.progressive = code == 0xC2;
  if (len < 6) return ffail(P, "bad SOF");
  if (b[0] != 8) return ffail(P, "only 8-bit samples are supported");
  P.h = be16(b + 1);
  P.w = be16(b + 3);
  P.nf = b[5];
  if (P.h == 0) return ffail(P, "height defined by DNL is not supported");
  if (P.w == 0) return ffail(P, "zero width");
  if (P.nf != 1 && P.nf != 3) return ffail(P, "only 1- and 3-component images are supported");
  if (len < 6 + 3 * P.nf) return ffail(P, "bad SOF");
  for (int i = 0; i < P.nf; i++) {
    P.cid[i] = b[6 + 3 * i];
    P.hs[i] = b[7 + 3 * i] >> 4;
    P.vs[i] = b[7 + 3 * i] & 15;
    P.tq[i] = b[8 + 3 * i];
    if (P.hs[i] < 1 || P.hs[i] > 4 || P.vs[i] < 1 || P.vs[i] > 4 || P.tq[i] > 3)
      return ffail(P, "bad component parameters");
  }
  P.sof = code;
  P.have_frame = true;
  return true;
}

bool parse_dqt(Parser& P, const uint8_t* b, int len) {
  int i = 0;
  while (i < len) {
    const int pq = b[i] >> 4, t = b[i] & 15;
    i++;
    if (t > 3 || pq > 1 || i + 64 * (pq + 1) > len) return ffail(P, "bad DQT");
    for (int k = 0; k < 64; k++) P.qt[t][k] = pq ? be16(b + i + 2 * k) : b[i + k];
    i += 64 * (pq + 1);
    P.have_qt[t] = true;
  }
  return true;
}

bool parse_dht(Parser& P, const uint8_t* b, int len) {
  int i = 0;
  while (i < len) {
    if (i + 17 > len) return ffail(P, "bad DHT");
    const int tc = b[i] >> 4, th = b[i] & 15;
    if (tc > 1 || th > 3) return ffail(P, "bad DHT");
    int nv = 0;
    for (int k = 0; k < 16; k++) nv += b[i + 1 + k];
    if (nv > 256 || i + 17 + nv > len) return ffail(P, "bad DHT");
    if (!build_huff(tc ? &P.ac[th] : &P.dc[th], b + i + 1, b + i + 17, nv))
      return ffail(P, "bad Huffman table");
    i += 17 + nv;
  }
  return true;
}

// Geometry of the frame (jdinput.c initial_setup) into the header.
void frame_geometry(const Parser& P, JpegHeader* H) {
  H->width = P.w;
  H->height = P.h;
  H->ncomp = P.nf;
  H->hmax = H->vmax = 1;
  for (int i = 0; i < P.nf; i++) {
    H->hmax = H->hmax > P.hs[i] ? H->hmax : P.hs[i];
    H->vmax = H->vmax > P.vs[i] ? H->vmax : P.vs[i];
  }
  const int mcux = (P.w + 8 * H->hmax - 1) / (8 * H->hmax);
  const int mcuy = (P.h + 8 * H->vmax - 1) / (8 * H->vmax);
  int64_t off = 0;
  for (int i = 0; i < P.nf; i++) {
    JpegComp& c = H->comp[i];
    c.h = P.nf == 1 ? 1 : P.hs[i];
    c.v = P.nf == 1 ? 1 : P.vs[i];
    const int hm = P.nf == 1 ? 1 : H->hmax, vm = P.nf == 1 ? 1 : H->vmax;
    c.dw = (int32_t)(((int64_t)P.w * c.h + hm - 1) / hm);
    c.dh = (int32_t)(((int64_t)P.h * c.v + vm - 1) / vm);
    const int wib = (c.dw + 7) / 8, hib = (c.dh + 7) / 8;
    c.bw = P.nf == 1 ? wib : (mcux * c.h > wib ? mcux * c.h : wib);
    c.bh = P.nf == 1 ? hib : (mcuy * c.v > hib ? mcuy * c.v : hib);
    c.pitch = c.bw * 8;
    c.plane_off = off;
    off += (int64_t)c.pitch * c.bh * 8;
  }
  H->scratch_bytes = P.nf == 1 ? 0 : off;
}

bool decode_scan(Parser& P, const uint8_t* b, int len, JpegDecoded* out) {
  JpegHeader& H = out->h;
  if (!P.have_frame) return ffail(P, "SOS before SOF");
  if (len < 1) return ffail(P, "bad SOS");
  const int ns = b[0];
  if (ns < 1 || ns > 4 || len < 4 + 2 * ns) return ffail(P, "bad SOS");
  if (H.nscans >= kJpegMaxScans) return ffail(P, "too many scans");
  JpegScan& S = H.scan[H.nscans];
  int tdc[4], tac[4];
  for (int i = 0; i < ns; i++) {
    const int id = b[1 + 2 * i];
    int c = -1;
    for (int k = 0; k < P.nf; k++)
      if (P.cid[k] == id) c = k;
    if (c < 0) return ffail(P, "scan names an unknown component");
    S.comp[i] = c;
    tdc[i] = b[2 + 2 * i] >> 4;
    tac[i] = b[2 + 2 * i] & 15;
    if (tdc[i] > 3 || tac[i] > 3 || !P.dc[tdc[i]].present || !P.ac[tac[i]].present)
      return ffail(P, "scan uses a missing Huffman table");
    if (!P.have_qt[P.tq[c]]) return ffail(P, "component uses a missing quantisation table");
  }
  const int ss = b[1 + 2 * ns], se = b[2 + 2 * ns], ahal = b[3 + 2 * ns];
  if (ss != 0 || se != 63 || ahal != 0) return ffail(P, "not a sequential scan");
  if (H.nscans == 0) frame_geometry(P, &H);
  // libjpeg latches a component's quantisation table when the component
  // first appears in a scan (jdinput.c latch_quant_tables): a DQT between
  // scans applies to the components that appear later
  for (int i = 0; i < ns; i++) {
    const int c = S.comp[i];
    if (P.latched[c]) continue;
    for (int k = 0; k < 64; k++) H.comp[c].qzz[k] = P.qt[P.tq[c]][k];
    P.latched[c] = true;
  }
  S.ncomp = ns;
  if (ns == 1) {  // non-interleaved: one block per MCU over the component's real blocks
    const JpegComp& c = H.comp[S.comp[0]];
    S.mcus_x = (c.dw + 7) / 8;
    S.mcus_y = (c.dh + 7) / 8;
    S.blocks_per_mcu = 1;
  } else {
    S.mcus_x = (P.w + 8 * H.hmax - 1) / (8 * H.hmax);
    S.mcus_y = (P.h + 8 * H.vmax - 1) / (8 * H.vmax);
    S.blocks_per_mcu = 0;
    for (int i = 0; i < ns; i++) S.blocks_per_mcu += H.comp[S.comp[i]].h * H.comp[S.comp[i]].v;
    if (S.blocks_per_mcu > 10) return ffail(P, "more than 10 blocks per MCU");
  }
  S.first_block = H.nblocks;
  S.first_group = (int32_t)H.ngroups;
  const int64_t nb = (int64_t)S.mcus_x * S.mcus_y * S.blocks_per_mcu;
  // every block takes at least two bits (a DC and an AC code): a frame header
  // claiming more blocks than the file's remaining bytes can hold is refused
  // before anything is sized from it
  if (nb > 4 * (int64_t)(P.n - P.pos) + 64) return ffail(P, "frame larger than the file's data");
  out->counts.reserve((size_t)(H.nblocks + nb));
  // per block of an MCU: its component (for the Huffman tables and predictor)
  int bcomp[10];
  {
    int k = 0;
    for (int i = 0; i < ns; i++) {
      const int nbl = ns == 1 ? 1 : H.comp[S.comp[i]].h * H.comp[S.comp[i]].v;
      for (int j = 0; j < nbl; j++) bcomp[k++] = i;
    }
  }
  Bits bits{P.d + P.pos, P.d + P.n};
  int pred[4] = {0, 0, 0, 0};
  // counts sized up front; coefficients written in place at `pos` (a block
  // clears its 64 slots first, so the prefix up to its last non-zero is exact)
  const size_t cbase = out->counts.size();
  out->counts.resize(cbase + (size_t)nb);
  uint8_t* counts = out->counts.data() + cbase;
  size_t pos = out->coefs.size();
  out->coefs.resize(pos + (size_t)std::max<int64_t>(nb * 8, 1 << 16));
  int64_t bi = 0;
  int64_t mcu = 0;
  const int64_t nmcu = (int64_t)S.mcus_x * S.mcus_y;
  for (int my = 0; my < S.mcus_y; my++) {
    // the data ran out (zero bits fed past its end or a marker): stop now
    // rather than decode the rest of the frame from zeros
    if (bits.underrun()) return ffail(P, "truncated or corrupt entropy-coded data");
    out->groups.push_back((uint32_t)pos);
    if (pos > 0xF0000000u) return ffail(P, "image too large");
    for (int mx = 0; mx < S.mcus_x; mx++, mcu++) {
      if (P.restart && mcu > 0 && mcu % P.restart == 0) {
        // restart marker: byte-align, skip RSTn, reset the predictors
        if (bits.underrun()) return ffail(P, "truncated or corrupt entropy-coded data");
        const uint8_t* q = bits.p;
        while (q + 1 < bits.end && !(q[0] == 0xFF && q[1] >= 0xD0 && q[1] <= 0xD7)) q++;
        if (q + 1 >= bits.end) return ffail(P, "missing restart marker");
        bits.p = q + 2;
        bits.reset();
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
      }
      if (pos + 64 * 10 > out->coefs.size()) out->coefs.resize(out->coefs.size() * 2);
      for (int k = 0; k < S.blocks_per_mcu; k++) {
        const int i = bcomp[k];
        int16_t* o = out->coefs.data() + pos;
        memset(o, 0, 64 * sizeof(int16_t));  // runs of zeros need no stores
        const int t = bits.decode(P.dc[tdc[i]]);
        if (t < 0 || t > 11) return ffail(P, "corrupt entropy-coded data (DC)");
        const int diff = t ? extend(bits.get(t), t) : 0;
        pred[i] += diff;
        o[0] = (int16_t)pred[i];
        int last = o[0] ? 0 : -1;
        const Huff& ac = P.ac[tac[i]];
        for (int kk = 1; kk < 64;) {
          if (bits.n < 16) bits.fill();
          const uint32_t f = ac.fast[bits.buf >> (64 - kLook)];
          if (f) {
            const int used = f & 31;
            bits.buf <<= used;
            bits.n -= used;
            if (f & (1u << 9)) break;  // EOB
            const int r = (f >> 5) & 15;
            kk += r;
            if (kk > 63) return ffail(P, "corrupt entropy-coded data (AC run)");
            o[kk] = (int16_t)(f >> 16);
            last = kk++;
            continue;
          }
          const int rs = bits.decode(ac);
          if (rs < 0) return ffail(P, "corrupt entropy-coded data (AC)");
          const int r = rs >> 4, sz = rs & 15;
          if (sz) {
            kk += r;
            if (kk > 63 || sz > 10) return ffail(P, "corrupt entropy-coded data (AC run)");
            o[kk] = (int16_t)extend(bits.get(sz), sz);
            last = kk++;
          } else if (r == 15) {
            kk += 16;
          } else {
            break;  // EOB
          }
        }
        counts[bi++] = (uint8_t)(last + 1);
        pos += (size_t)(last + 1);
      }
    }
  }
  out->coefs.resize(pos);
  (void)nmcu;
  if (bits.underrun()) return ffail(P, "truncated or corrupt entropy-coded data");
  H.nblocks += nb;
  H.ngroups += S.mcus_y;
  H.nscans++;
  // continue parsing after the entropy-coded segment: at the marker the bit
  // reader stopped on (or scan forward to the next non-RST marker)
  size_t q = (size_t)(bits.p - P.d);
  while (q + 1 < P.n && !(P.d[q] == 0xFF && P.d[q + 1] != 0x00 &&
                          !(P.d[q + 1] >= 0xD0 && P.d[q + 1] <= 0xD7)))
    q++;
  P.pos = q;
  return true;
}

// Progressive scans (T.81 G.1.2; libjpeg jdphuff.c decode_mcu_DC_first /
// _DC_refine / _AC_first / _AC_refine): DC scans interleaved or not, AC
// scans of one component, spectral selection Ss..Se, successive
// approximation Ah/Al, end-of-band runs.  Coefficients accumulate in P.pc.
bool decode_prog_scan(Parser& P, const uint8_t* b, int len, JpegDecoded* out) {
  JpegHeader& H = out->h;
  if (!P.have_frame) return ffail(P, "SOS before SOF");
  if (len < 1) return ffail(P, "bad SOS");
  const int ns = b[0];
  if (ns < 1 || ns > 4 || len < 4 + 2 * ns) return ffail(P, "bad SOS");
  int comp[4], tdc[4], tac[4];
  const int ss = b[1 + 2 * ns], se = b[2 + 2 * ns], ah = b[3 + 2 * ns] >> 4, al = b[3 + 2 * ns] & 15;
  // jdphuff.c start_pass_phuff_decoder's checks
  if (ss == 0 ? se != 0 : (se < ss || se > 63 || ns != 1)) return ffail(P, "bad progressive scan");
  if ((ah != 0 && ah != al + 1) || al > 13) return ffail(P, "bad successive approximation");
  if (H.nscans == 0 && P.pc[0].empty()) {
    frame_geometry(P, &H);
    int64_t nb = 0;
    for (int c = 0; c < P.nf; c++) nb += (int64_t)H.comp[c].bw * H.comp[c].bh;
    // the DC scan codes each block in at least one bit
    if (nb > 8 * (int64_t)(P.n - P.pos) + 64 || nb > (1 << 24))
      return ffail(P, "frame larger than the file's data");
    for (int c = 0; c < P.nf; c++) P.pc[c].assign((size_t)H.comp[c].bw * H.comp[c].bh * 64, 0);
  }
  for (int i = 0; i < ns; i++) {
    const int id = b[1 + 2 * i];
    int c = -1;
    for (int k = 0; k < P.nf; k++)
      if (P.cid[k] == id) c = k;
    if (c < 0) return ffail(P, "scan names an unknown component");
    comp[i] = c;
    tdc[i] = b[2 + 2 * i] >> 4;
    tac[i] = b[2 + 2 * i] & 15;
    if (ss == 0 && ah == 0 && (tdc[i] > 3 || !P.dc[tdc[i]].present))
      return ffail(P, "scan uses a missing Huffman table");
    if (ss > 0 && (tac[i] > 3 || !P.ac[tac[i]].present))
      return ffail(P, "scan uses a missing Huffman table");
    if (!P.have_qt[P.tq[c]]) return ffail(P, "component uses a missing quantisation table");
    if (!P.latched[c]) {
      for (int k = 0; k < 64; k++) H.comp[c].qzz[k] = P.qt[P.tq[c]][k];
      P.latched[c] = true;
    }
  }
  // MCU geometry: interleaved (DC scans of several components) over the
  // frame's MCUs, else one block per MCU over the component's real blocks
  int mcus_x, mcus_y;
  if (ns == 1) {
    const JpegComp& c = H.comp[comp[0]];
    mcus_x = (c.dw + 7) / 8;
    mcus_y = (c.dh + 7) / 8;
  } else {
    mcus_x = (P.w + 8 * H.hmax - 1) / (8 * H.hmax);
    mcus_y = (P.h + 8 * H.vmax - 1) / (8 * H.vmax);
  }
  Bits bits{P.d + P.pos, P.d + P.n};
  int pred[4] = {0, 0, 0, 0};
  int eobrun = 0;
  const int p1 = 1 << al, m1 = -(1 << al);
  int64_t mcu = 0;
  for (int my = 0; my < mcus_y; my++) {
    if (bits.underrun()) return ffail(P, "truncated or corrupt entropy-coded data");
    for (int mx = 0; mx < mcus_x; mx++, mcu++) {
      if (P.restart && mcu > 0 && mcu % P.restart == 0) {
        if (bits.underrun()) return ffail(P, "truncated or corrupt entropy-coded data");
        const uint8_t* q = bits.p;
        while (q + 1 < bits.end && !(q[0] == 0xFF && q[1] >= 0xD0 && q[1] <= 0xD7)) q++;
        if (q + 1 >= bits.end) return ffail(P, "missing restart marker");
        bits.p = q + 2;
        bits.reset();
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
        eobrun = 0;
      }
      for (int i = 0; i < ns; i++) {
        const JpegComp& C = H.comp[comp[i]];
        const int nbx = ns == 1 ? 1 : C.h, nby = ns == 1 ? 1 : C.v;
        for (int by = 0; by < nby; by++)
          for (int bx = 0; bx < nbx; bx++) {
            const int64_t gx = (int64_t)mx * nbx + bx, gy = (int64_t)my * nby + by;
            int16_t* blk = P.pc[comp[i]].data() + (gy * C.bw + gx) * 64;
            if (ss == 0) {
              if (ah == 0) {  // DC first
                const int t = bits.decode(P.dc[tdc[i]]);
                if (t < 0 || t > 11) return ffail(P, "corrupt entropy-coded data (DC)");
                pred[i] += t ? extend(bits.get(t), t) : 0;
                blk[0] = (int16_t)(pred[i] * (1 << al));
              } else if (bits.get(1)) {  // DC refine
                blk[0] = (int16_t)(blk[0] | p1);
              }
              continue;
            }
            const Huff& ac = P.ac[tac[i]];
            int k = ss;
            if (ah == 0) {  // AC first
              if (eobrun > 0) {
                eobrun--;
                continue;
              }
              for (; k <= se; k++) {
                const int rs = bits.decode(ac);
                if (rs < 0) return ffail(P, "corrupt entropy-coded data (AC)");
                const int r = rs >> 4, sz = rs & 15;
                if (sz) {
                  k += r;
                  if (k > se || sz > 10) return ffail(P, "corrupt entropy-coded data (AC run)");
                  blk[k] = (int16_t)(extend(bits.get(sz), sz) * (1 << al));
                } else if (r == 15) {
                  k += 15;
                } else {
                  eobrun = (1 << r) - 1;
                  if (r) eobrun += (int)bits.get(r);
                  break;
                }
              }
              continue;
            }
            // AC refine
            auto refine = [&](int16_t* coef) {
              if (bits.get(1) && (*coef & p1) == 0) *coef = (int16_t)(*coef + (*coef >= 0 ? p1 : m1));
            };
            if (eobrun == 0) {
              for (; k <= se; k++) {
                const int rs = bits.decode(ac);
                if (rs < 0) return ffail(P, "corrupt entropy-coded data (AC)");
                int r = rs >> 4;
                int sv = 0;
                if (rs & 15) {
                  if ((rs & 15) != 1) return ffail(P, "corrupt entropy-coded data (AC refine)");
                  sv = bits.get(1) ? p1 : m1;
                } else if (r != 15) {
                  eobrun = 1 << r;
                  if (r) eobrun += (int)bits.get(r);
                  break;
                }
                do {
                  int16_t* coef = blk + k;
                  if (*coef != 0) {
                    refine(coef);
                  } else {
                    if (--r < 0) break;  // the zero the new coefficient goes to
                  }
                  k++;
                } while (k <= se);
                if (sv) {
                  if (k > se) return ffail(P, "corrupt entropy-coded data (AC refine)");
                  blk[k] = (int16_t)sv;
                }
              }
            }
            if (eobrun > 0) {
              for (; k <= se; k++)
                if (blk[k] != 0) refine(blk + k);
              eobrun--;
            }
          }
      }
    }
  }
  if (bits.underrun()) return ffail(P, "truncated or corrupt entropy-coded data");
  size_t q = (size_t)(bits.p - P.d);
  while (q + 1 < P.n && !(P.d[q] == 0xFF && P.d[q + 1] != 0x00 &&
                          !(P.d[q + 1] >= 0xD0 && P.d[q + 1] <= 0xD7)))
    q++;
  P.pos = q;
  return true;
}

// The finished progressive coefficients as one sequential scan (interleaved
// over the frame's MCUs for colour, the real blocks for gray) in the packed
// layout the device decodes.
bool flatten_progressive(Parser& P, JpegDecoded* out) {
  JpegHeader& H = out->h;
  if (P.pc[0].empty()) return ffail(P, "no scan");
  for (int c = 0; c < P.nf; c++)
    if (!P.latched[c]) return ffail(P, "a component is missing from the scans");
  JpegScan& S = H.scan[0];
  S.ncomp = P.nf;
  for (int i = 0; i < P.nf; i++) S.comp[i] = i;
  if (P.nf == 1) {
    S.mcus_x = (H.comp[0].dw + 7) / 8;
    S.mcus_y = (H.comp[0].dh + 7) / 8;
    S.blocks_per_mcu = 1;
  } else {
    S.mcus_x = (P.w + 8 * H.hmax - 1) / (8 * H.hmax);
    S.mcus_y = (P.h + 8 * H.vmax - 1) / (8 * H.vmax);
    S.blocks_per_mcu = 0;
    for (int i = 0; i < P.nf; i++) S.blocks_per_mcu += H.comp[i].h * H.comp[i].v;
    if (S.blocks_per_mcu > 10) return ffail(P, "more than 10 blocks per MCU");
  }
  S.first_block = 0;
  S.first_group = 0;
  const int64_t nb = (int64_t)S.mcus_x * S.mcus_y * S.blocks_per_mcu;
  out->counts.resize((size_t)nb);
  out->coefs.clear();
  out->groups.clear();
  int64_t bi = 0;
  auto put = [&](const int16_t* blk) {
    int last = 63;
    while (last >= 0 && blk[last] == 0) last--;
    out->counts[(size_t)bi++] = (uint8_t)(last + 1);
    out->coefs.insert(out->coefs.end(), blk, blk + last + 1);
  };
  for (int my = 0; my < S.mcus_y; my++) {
    out->groups.push_back((uint32_t)out->coefs.size());
    if (out->coefs.size() > 0xF0000000u) return ffail(P, "image too large");
    for (int mx = 0; mx < S.mcus_x; mx++) {
      if (P.nf == 1) {
        put(P.pc[0].data() + ((int64_t)my * H.comp[0].bw + mx) * 64);
        continue;
      }
      for (int c = 0; c < P.nf; c++) {
        const JpegComp& C = H.comp[c];
        for (int by = 0; by < C.v; by++)
          for (int bx = 0; bx < C.h; bx++)
            put(P.pc[c].data() + (((int64_t)my * C.v + by) * C.bw + (int64_t)mx * C.h + bx) * 64);
      }
    }
  }
  H.nblocks = nb;
  H.ngroups = S.mcus_y;
  H.nscans = 1;
  return true;
}

// The one scan of a sequential file for the device decoder: scan header,
// geometry, decode tables, and the entropy-coded data with the byte stuffing
// and the restart markers removed (each restart segment starts on a byte).
bool stream_scan(Parser& P, const uint8_t* b, int len) {
  JdecStreamHost& S = *P.stream;
  JdecHeader& D = S.hd;
  JpegHeader& H = D.h;
  if (!P.have_frame) return ffail(P, "SOS before SOF");
  if (H.nscans > 0) return P.not_device = true, false;  // several scans: host decoder
  if (len < 1) return ffail(P, "bad SOS");
  const int ns = b[0];
  if (ns < 1 || ns > 4 || len < 4 + 2 * ns) return ffail(P, "bad SOS");
  if (ns != P.nf) return P.not_device = true, false;  // one scan per component
  JpegScan& Sc = H.scan[0];
  for (int i = 0; i < ns; i++) {
    const int id = b[1 + 2 * i];
    int c = -1;
    for (int k = 0; k < P.nf; k++)
      if (P.cid[k] == id) c = k;
    if (c < 0) return ffail(P, "scan names an unknown component");
    Sc.comp[i] = c;
    D.tdc[i] = b[2 + 2 * i] >> 4;
    D.tac[i] = b[2 + 2 * i] & 15;
    if (D.tdc[i] > 3 || D.tac[i] > 3 || !P.dc[D.tdc[i]].present || !P.ac[D.tac[i]].present)
      return ffail(P, "scan uses a missing Huffman table");
    if (!P.have_qt[P.tq[c]]) return ffail(P, "component uses a missing quantisation table");
  }
  if (b[1 + 2 * ns] != 0 || b[2 + 2 * ns] != 63 || b[3 + 2 * ns] != 0)
    return ffail(P, "not a sequential scan");
  frame_geometry(P, &H);
  for (int i = 0; i < ns; i++)
    for (int k = 0; k < 64; k++) H.comp[Sc.comp[i]].qzz[k] = P.qt[P.tq[Sc.comp[i]]][k];
  Sc.ncomp = ns;
  if (ns == 1) {
    Sc.mcus_x = (H.comp[Sc.comp[0]].dw + 7) / 8;
    Sc.mcus_y = (H.comp[Sc.comp[0]].dh + 7) / 8;
    Sc.blocks_per_mcu = 1;
    D.bcomp[0] = 0;
  } else {
    Sc.mcus_x = (P.w + 8 * H.hmax - 1) / (8 * H.hmax);
    Sc.mcus_y = (P.h + 8 * H.vmax - 1) / (8 * H.vmax);
    int nb = 0;
    for (int i = 0; i < ns; i++) nb += H.comp[Sc.comp[i]].h * H.comp[Sc.comp[i]].v;
    if (nb > 10) return ffail(P, "more than 10 blocks per MCU");
    Sc.blocks_per_mcu = 0;
    for (int i = 0; i < ns; i++)
      for (int j = 0; j < H.comp[Sc.comp[i]].h * H.comp[Sc.comp[i]].v; j++)
        D.bcomp[Sc.blocks_per_mcu++] = i;
  }
  Sc.first_block = 0;
  Sc.first_group = 0;
  H.nblocks = (int64_t)Sc.mcus_x * Sc.mcus_y * Sc.blocks_per_mcu;
  H.ngroups = Sc.mcus_y;
  H.nscans = 1;
  // each block takes at least two bits
  if (H.nblocks > 4 * (int64_t)(P.n - P.pos) + 64) return ffail(P, "frame larger than the file's data");
  for (int t = 0; t < 4; t++) {
    const Huff* src[2] = {&P.dc[t], &P.ac[t]};
    JdecTable* dst[2] = {&D.dc[t], &D.ac[t]};
    for (int k = 0; k < 2; k++) {
      if (!src[k]->present) continue;
      memcpy(dst[k]->look, src[k]->look, sizeof(dst[k]->look));
      for (int l = 0; l < 18; l++) dst[k]->maxcode[l] = src[k]->maxcode[l];
      for (int l = 1; l <= 16; l++) dst[k]->valoff[l] = src[k]->valptr[l] - src[k]->mincode[l];
      memcpy(dst[k]->vals, src[k]->vals, 256);
    }
  }
  D.restart = P.restart;
  // unstuff: 0xFF 0x00 -> 0xFF, RSTn -> a new segment, fill bytes skipped,
  // any other marker ends the data
  std::vector<uint8_t>& out = S.data;
  out.clear();
  out.reserve(P.n - P.pos + 16);
  S.seg.assign(1, 0);
  const uint8_t* p = P.d + P.pos;
  const uint8_t* end = P.d + P.n;
  while (p < end) {
    const uint8_t* ff = (const uint8_t*)memchr(p, 0xFF, (size_t)(end - p));
    if (!ff) {
      out.insert(out.end(), p, end);
      p = end;
      break;
    }
    out.insert(out.end(), p, ff);
    p = ff;
    if (p + 1 >= end) break;
    const uint8_t m = p[1];
    if (m == 0x00) {
      out.push_back(0xFF);
      p += 2;
    } else if (m == 0xFF) {
      p += 1;  // fill byte
    } else if (m >= 0xD0 && m <= 0xD7) {
      if (out.size() >= kJdecMaxBytes) return P.not_device = true, false;  // host decoder
      S.seg.push_back((int32_t)out.size() * 8);
      p += 2;
    } else {
      break;  // EOI or another marker
    }
  }
  P.pos = (size_t)(p - P.d);
  if (out.size() >= kJdecMaxBytes) return P.not_device = true, false;  // host decoder
  const int64_t nbits = (int64_t)out.size() * 8;
  S.seg.push_back((int32_t)nbits);
  D.nseg = (int32_t)S.seg.size() - 1;
  D.nbits = nbits;
  const int64_t nmcu = (int64_t)Sc.mcus_x * Sc.mcus_y;
  if (P.restart) {
    if ((int64_t)D.nseg != (nmcu + P.restart - 1) / P.restart)
      return ffail(P, "restart markers do not match the restart interval");
  } else if (D.nseg != 1) {
    return ffail(P, "restart marker without a restart interval");
  }
  S.segsub.assign((size_t)D.nseg + 1, 0);
  S.segmac.assign((size_t)D.nseg + 1, 0);
  int64_t nsub = 0, nmac = 0;
  for (int g = 0; g < D.nseg; g++) {
    S.segsub[(size_t)g] = (int32_t)nsub;
    S.segmac[(size_t)g] = (int32_t)nmac;
    const int64_t bits = S.seg[(size_t)g + 1] - S.seg[(size_t)g];
    const int64_t k = std::max<int64_t>(1, (bits + kJdecSubBits - 1) / kJdecSubBits);
    nsub += k;
    nmac += (k + kJdecMacro - 1) / kJdecMacro;
    if (nsub > 0x7fffffff) return ffail(P, "image too large");
  }
  S.segsub[(size_t)D.nseg] = (int32_t)nsub;
  S.segmac[(size_t)D.nseg] = (int32_t)nmac;
  D.nsub = nsub;
  D.nmac = nmac;
  out.resize(out.size() + 48, 0);  // slack for the device's read-ahead (jpeg_huff_core.h)
  return true;
}

// marker loop; full = false stops after the frame header (probe)
bool parse(Parser& P, bool full, JpegDecoded* out) {
  if (P.n < 4 || P.d[0] != 0xFF || P.d[1] != 0xD8) return ffail(P, "not a JPEG file");
  P.pos = 2;
  for (;;) {
    const int m = next_marker(P);
    if (m < 0) {
      const bool any = P.stream ? P.stream->hd.h.nscans > 0 : (out->h.nscans > 0 || !P.pc[0].empty());
      if (full && any) break;  // missing EOI: tolerated, as libjpeg
      return ffail(P, "unexpected end of file");
    }
    if (m == 0xD9) break;                              // EOI
    if ((m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;  // stray RSTn / TEM
    const uint8_t* b;
    int len;
    if (!segment(P, &b, &len)) return false;
    if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      if (!parse_sof(P, m, b, len)) return false;
      if (!full) return true;
    } else if (m == 0xC4) {
      if (!parse_dht(P, b, len)) return false;
    } else if (m == 0xCC) {
      return ffail(P, "arithmetic-coded JPEG is not supported");
    } else if (m == 0xDB) {
      if (!parse_dqt(P, b, len)) return false;
    } else if (m == 0xDD) {
      if (len < 2) return ffail(P, "bad DRI");
      P.restart = be16(b);
    } else if (m == 0xDA) {
      if (!full) return ffail(P, "SOS before SOF");
      if (P.stream) {
        if (P.progressive) return P.not_device = true, false;
        if (!stream_scan(P, b, len)) return false;
      } else if (!(P.progressive ? decode_prog_scan(P, b, len, out) : decode_scan(P, b, len, out))) {
        return false;
      }
    } else if (m == 0xE0) {
      if (len >= 5 && !memcmp(b, "JFIF", 5)) P.jfif = true;
    } else if (m == 0xEE) {
      if (len >= 12 && !memcmp(b, "Adobe", 5)) {
        P.adobe = true;
        P.adobe_transform = b[11];
      }
    }
    // other APPn, COM, DHP, EXP: skipped
  }
  if (!P.have_frame) return ffail(P, "no frame header");
  return true;
}

// jdapimin.c default_decompress_parms: the colour space of a 3-component file
int color_of(const Parser& P) {
  if (P.nf == 1) return 0;
  if (P.jfif) return 1;
  if (P.adobe) return P.adobe_transform == 0 ? 2 : 1;
  if (P.cid[0] == 'R' && P.cid[1] == 'G' && P.cid[2] == 'B') return 2;
  return 1;
}

bool read_file(const char* path, std::vector<uint8_t>* buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return fail("jpeg: cannot open %s: %s", path, strerror(errno));
  bool ok = fseek(f, 0, SEEK_END) == 0;
  const long sz = ok ? ftell(f) : -1;
  ok = ok && sz >= 0 && sz < (1l << 31) && fseek(f, 0, SEEK_SET) == 0;
  if (ok) {
    buf->resize((size_t)sz);
    ok = fread(buf->data(), 1, (size_t)sz, f) == (size_t)sz;
  }
  fclose(f);
  return ok || fail("jpeg: cannot read %s", path);
}

int64_t align16(int64_t v) { return (v + 15) & ~(int64_t)15; }

}  // namespace

bool jpeg_probe_mem(const uint8_t* d, size_t n, const char* name, UphipPnmInfo* info) {
  Parser P{d, n, name};
  if (!parse(P, false, nullptr)) return false;
  info->width = P.w;
  info->height = P.h;
  info->format = P.nf == 1 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24;
  return true;
}

bool jpeg_entropy_decode(const uint8_t* d, size_t n, const char* name, JpegDecoded* out) {
  try {
    *out = JpegDecoded();
    Parser P{d, n, name};
    if (!parse(P, true, out)) return false;
    if (P.progressive && !flatten_progressive(P, out)) return false;
    if (out->h.nscans == 0) return ffail(P, "no scan");
    out->h.color = color_of(P);
    // every component must be covered by a scan
    bool seen[3] = {false, false, false};
    for (int s = 0; s < out->h.nscans; s++)
      for (int i = 0; i < out->h.scan[s].ncomp; i++) seen[out->h.scan[s].comp[i]] = true;
    for (int i = 0; i < P.nf; i++)
      if (!seen[i]) return ffail(P, "a component is missing from the scans");
    out->groups.push_back((uint32_t)out->coefs.size());
    JpegHeader& H = out->h;
    H.counts_off = align16((int64_t)sizeof(JpegHeader));
    H.groups_off = align16(H.counts_off + H.nblocks);
    H.coefs_off = align16(H.groups_off + 4 * (H.ngroups + 1));
    H.total_bytes = align16(H.coefs_off + 2 * (int64_t)out->coefs.size());
    return true;
  } catch (const std::bad_alloc&) {
    return fail("jpeg: %s: out of memory", name);
  }
}

int jpeg_stream_prepare(const uint8_t* d, size_t n, const char* name, JdecStreamHost* out) {
  try {
    out->hd = JdecHeader{};
    std::unique_ptr<Parser> P(new Parser{d, n, name});
    P->stream = out;
    if (!parse(*P, true, nullptr)) return P->not_device ? 0 : -1;
    if (out->hd.h.nscans == 0) return ffail(*P, "no scan"), -1;
    JdecHeader& D = out->hd;
    JpegHeader& H = D.h;
    H.color = color_of(*P);
    // the packed layout the device writes (upper bound: 64 coefficients a block)
    H.counts_off = align16((int64_t)sizeof(JpegHeader));
    H.groups_off = align16(H.counts_off + H.nblocks);
    H.coefs_off = align16(H.groups_off + 4 * (H.ngroups + 1));
    H.total_bytes = align16(H.coefs_off + 2 * 64 * H.nblocks);
    D.seg_off = align16((int64_t)sizeof(JdecHeader));
    D.segsub_off = align16(D.seg_off + 4 * (int64_t)out->seg.size());
    D.segmac_off = align16(D.segsub_off + 4 * (int64_t)out->segsub.size());
    D.data_off = align16(D.segmac_off + 4 * (int64_t)out->segmac.size());
    D.total_bytes = align16(D.data_off + (int64_t)out->data.size());
    return 1;
  } catch (const std::bad_alloc&) {
    return fail("jpeg: %s: out of memory", name), -1;
  }
}

void jpeg_stream_pack(const JdecStreamHost& s, uint8_t* dst) {
  const JdecHeader& D = s.hd;
  memcpy(dst, &D, sizeof(D));
  memcpy(dst + D.seg_off, s.seg.data(), 4 * s.seg.size());
  memcpy(dst + D.segsub_off, s.segsub.data(), 4 * s.segsub.size());
  memcpy(dst + D.segmac_off, s.segmac.data(), 4 * s.segmac.size());
  memcpy(dst + D.data_off, s.data.data(), s.data.size());
}

void jpeg_pack(const JpegDecoded& j, uint8_t* dst) {
  const JpegHeader& H = j.h;
  memset(dst, 0, (size_t)H.total_bytes);
  memcpy(dst, &H, sizeof(H));
  memcpy(dst + H.counts_off, j.counts.data(), j.counts.size());
  memcpy(dst + H.groups_off, j.groups.data(), 4 * j.groups.size());
  memcpy(dst + H.coefs_off, j.coefs.data(), 2 * j.coefs.size());
}

bool jpeg_read_file(const char* path, std::vector<uint8_t>* buf) { return read_file(path, buf); }

}  // namespace uph

namespace uph {

// Entropy-decode on the host, upload, decode on the current device/stream
// into device memory (synchronous).
bool jpeg_decode_to_device(const uint8_t* data, size_t size, const char* name, uint8_t* ddst,
                           int64_t pitch, UphipPnmInfo* info) {
  // one-scan sequential files: Huffman decoding on the device too
  JdecStreamHost S;
  const int dev = jpeg_stream_prepare(data, size, name, &S);
  if (dev < 0) return false;
  JpegDecoded j;
  if (!dev && !jpeg_entropy_decode(data, size, name, &j)) return false;
  const JpegHeader& H = dev ? S.hd.h : j.h;
  const int fmt = H.ncomp == 1 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24;
  if (info) {
    if (info->width > 0 && (info->width != H.width || info->height != H.height || info->format != fmt))
      return fail("jpeg: %s is %dx%d format %d, expected %dx%d format %d", name, H.width, H.height,
                  fmt, info->width, info->height, info->format);
    info->width = H.width;
    info->height = H.height;
    info->format = fmt;
  }
  if (pitch < (int64_t)H.width * (H.ncomp == 1 ? 1 : 3)) return fail("jpeg: pitch too small");
  hipStream_t st = current_stream();
  uint8_t* dp = (uint8_t*)scratch(0, (size_t)H.total_bytes);
  uint8_t* ds = H.scratch_bytes ? (uint8_t*)scratch(1, (size_t)H.scratch_bytes) : nullptr;
  if (!dp || (H.scratch_bytes && !ds)) return false;
  if (!dev) {
    std::vector<uint8_t> packed((size_t)H.total_bytes);
    jpeg_pack(j, packed.data());
    return UPH_HIP(hipMemcpyAsync(dp, packed.data(), packed.size(), hipMemcpyHostToDevice, st)) &&
           jpeg_launch(H, dp, ds, ddst, pitch, st) && UPH_HIP(hipStreamSynchronize(st));
  }
  std::vector<uint8_t> up((size_t)S.hd.total_bytes);
  jpeg_stream_pack(S, up.data());
  uint8_t* dstream = (uint8_t*)scratch(3, up.size());
  uint8_t* dscr = (uint8_t*)scratch(4, jdec_scratch_bytes(S.hd) + sizeof(JdecJob));
  int32_t* dstatus = (int32_t*)scratch(5, 4);
  int32_t status = 0;
  if (!dstream || !dscr || !dstatus ||
      !UPH_HIP(hipMemsetAsync(dstatus, 0, 4, st)) ||
      !UPH_HIP(hipMemcpyAsync(dstream, up.data(), up.size(), hipMemcpyHostToDevice, st)) ||
      !jdec_launch(S.hd, dstream, dp, dscr, dstatus, st) || !jpeg_launch(H, dp, ds, ddst, pitch, st) ||
      !UPH_HIP(hipMemcpyAsync(&status, dstatus, 4, hipMemcpyDeviceToHost, st)) ||
      !UPH_HIP(hipStreamSynchronize(st)))
    return false;
  if (status) return fail("jpeg: %s: corrupt entropy-coded data (device decode, 0x%x)", name, status);
  return true;
}

}  // namespace uph

using namespace uph;

extern "C" {

int uphip_jpeg_probe(const char* path, UphipPnmInfo* info) {
  if (!path || !info) return fail("jpeg_probe: null argument"), -1;
  // the frame header is near the start; read what there is up to 1 MiB
  FILE* f = fopen(path, "rb");
  if (!f) return fail("jpeg: cannot open %s: %s", path, strerror(errno)), -1;
  std::vector<uint8_t> buf(1 << 20);
  buf.resize(fread(buf.data(), 1, buf.size(), f));
  fclose(f);
  if (jpeg_probe_mem(buf.data(), buf.size(), path, info)) return 0;
  // a header past the first MiB (large APPn segments): the whole file
  uphip_clear_error();
  if (!jpeg_read_file(path, &buf)) return -1;
  return jpeg_probe_mem(buf.data(), buf.size(), path, info) ? 0 : -1;
}

int64_t uphip_jpeg_entropy_decode(const void* data, size_t size, void* packed, int64_t capacity) {
  if (!data) return fail("jpeg_entropy_decode: null argument"), -1;
  JpegDecoded j;
  if (!jpeg_entropy_decode((const uint8_t*)data, size, "<memory>", &j)) return -1;
  if (packed && capacity >= j.h.total_bytes) jpeg_pack(j, (uint8_t*)packed);
  return j.h.total_bytes;
}

int uphip_jpeg_decode(const void* data, size_t size, void* device_dst, int64_t pitch,
                      UphipPnmInfo* info) {
  if (!data || !device_dst) return fail("jpeg_decode: null argument"), -1;
  if (!runtime_ready()) return fail("jpeg_decode: no HIP device"), -1;
  return jpeg_decode_to_device((const uint8_t*)data, size, "<memory>", (uint8_t*)device_dst, pitch,
                               info)
             ? 0
             : -1;
}

int uphip_jpeg_read(const char* path, void* dst, int64_t linesize, const UphipPnmInfo* expect) {
  if (!path || !dst) return fail("jpeg_read: null argument"), -1;
  if (!runtime_ready()) return fail("jpeg_read: no HIP device (JPEG decodes on the device)"), -1;
  std::vector<uint8_t> file;
  if (!jpeg_read_file(path, &file)) return -1;
  UphipPnmInfo info{0, 0, 0};
  if (!jpeg_probe_mem(file.data(), file.size(), path, &info)) return -1;
  if (expect && (expect->width != info.width || expect->height != info.height ||
                 expect->format != info.format))
    return fail("jpeg: %s is %dx%d format %d, expected %dx%d format %d", path, info.width,
                info.height, info.format, expect->width, expect->height, expect->format),
           -1;
  const int64_t rb = row_bytes(info.width, info.format);
  if (linesize < rb) return fail("jpeg_read: linesize too small"), -1;
  const int64_t dpitch = (rb + 255) & ~(int64_t)255;
  uint8_t* dd = (uint8_t*)scratch(2, (size_t)(dpitch * info.height));
  if (!dd || !jpeg_decode_to_device(file.data(), file.size(), path, dd, dpitch, &info)) return -1;
  return UPH_HIP(hipMemcpy2D(dst, (size_t)linesize, dd, (size_t)dpitch, (size_t)rb,
                             (size_t)info.height, hipMemcpyDeviceToHost))
             ? 0
             : -1;
}

}  // extern "C"
