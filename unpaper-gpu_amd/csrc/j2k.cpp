// j2k.cpp — JPEG 2000 codestream parsing, packet headers (Tier 2) and
// code-blocks (Tier 1, j2k_t1.h) on the host; see j2k.h.  Peer of
// nvimgcodec.c's JPEG2000 decode (:840) and nvimgcodec_encode_jp2
// (:1133-1165).  Follows ISO/IEC 15444-1: Annex A (markers), B (tiles,
// resolutions, subbands, precincts, code-blocks, packets), E (quantisation).
#include "j2k.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <set>
#include <string>

#include "j2k_t1.h"
#include "j2k_t1_lane.h"
#include "runtime.h"

namespace uph {
namespace j2k {

namespace {

int ceildiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
int ceil_pow2(int64_t a, int e) { return (int)((a + ((int64_t)1 << e) - 1) >> e); }
int floor_log2(uint32_t v) {
  int n = -1;
  while (v) {
    n++;
    v >>= 1;
  }
  return n;
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  const char* name;
  bool ok = true;
  bool need(size_t n) {
    if ((size_t)(end - p) < n) ok = false;
    return ok;
  }
  uint32_t u8() { return need(1) ? *p++ : 0; }
  uint32_t u16() {
    if (!need(2)) return 0;
    const uint32_t v = (uint32_t)p[0] << 8 | p[1];
    p += 2;
    return v;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
    p += 4;
    return v;
  }
};

bool jfail(const char* name, const char* what) { return fail("jp2: %s: %s", name, what); }

// Coding style (COD / COC) of a component
struct Cod {
  int scod = 0;       // bit 0: precincts given, 1: SOP, 2: EPH
  int prog = 0, layers = 1, mct = 0;
  int nlevels = 5, cbw = 6, cbh = 6, cbsty = 0, reversible = 1;
  int ppx[kMaxLevels + 1], ppy[kMaxLevels + 1];
  Cod() {
    for (int i = 0; i <= kMaxLevels; i++) ppx[i] = ppy[i] = 15;
  }
};
// Quantisation (QCD / QCC) of a component
struct Qcd {
  int guard = 2, style = 0;
  int nexp = 0;
  int expn[3 * kMaxLevels + 1], mant[3 * kMaxLevels + 1];
};

struct Params {
  Cod cod[kMaxComps];
  Qcd qcd[kMaxComps];
};

bool read_spcod(Reader& r, Cod& c, bool precincts) {
  c.nlevels = (int)r.u8();
  c.cbw = (int)r.u8() + 2;
  c.cbh = (int)r.u8() + 2;
  c.cbsty = (int)r.u8();
  c.reversible = (int)r.u8();
  if (c.nlevels > kMaxLevels) return false;
  for (int i = 0; i <= c.nlevels; i++) {
    const int v = precincts ? (int)r.u8() : 0xFF;
    c.ppx[i] = v & 15;
    c.ppy[i] = v >> 4;
  }
  return r.ok;
}

bool read_sqcd(Reader& r, const uint8_t* end, Qcd& q) {
  const int s = (int)r.u8();
  q.guard = s >> 5;
  q.style = s & 31;
  q.nexp = 0;
  if (q.style == 0) {
    while (r.p < end && q.nexp < 3 * kMaxLevels + 1) {
      q.expn[q.nexp] = (int)r.u8() >> 3;
      q.mant[q.nexp++] = 0;
    }
  } else if (q.style == 1 || q.style == 2) {
    while (r.p + 1 < end && q.nexp < 3 * kMaxLevels + 1) {
      const int v = (int)r.u16();
      q.expn[q.nexp] = v >> 11;
      q.mant[q.nexp++] = v & 0x7FF;
    }
  } else {
    return false;
  }
  return r.ok && q.nexp > 0;
}

// ---------------------------------------------------------------------------
// tag trees (B.10.2)
struct TagTree {
  struct Node {
    int parent, value, low, known;
  };
  std::vector<Node> n;
  int w = 0, h = 0;
  void init(int w0, int h0) {
    w = w0;
    h = h0;
    n.clear();
    if (w0 <= 0 || h0 <= 0) return;
    std::vector<int> lw, lh, base;
    int cw = w0, ch = h0, total = 0;
    for (;;) {
      lw.push_back(cw);
      lh.push_back(ch);
      base.push_back(total);
      total += cw * ch;
      if (cw == 1 && ch == 1) break;
      cw = (cw + 1) / 2;
      ch = (ch + 1) / 2;
    }
    n.assign((size_t)total, Node{-1, 999, 0, 0});
    for (size_t l = 0; l + 1 < lw.size(); l++)
      for (int y = 0; y < lh[l]; y++)
        for (int x = 0; x < lw[l]; x++)
          n[(size_t)(base[l] + y * lw[l] + x)].parent = base[l + 1] + (y / 2) * lw[l + 1] + x / 2;
  }
  // encoder: leaf values, then each node the minimum of its children
  void set_values(const std::vector<int>& leaves) {
    for (auto& q : n) {
      q.value = 999;
      q.low = 0;
      q.known = 0;
    }
    for (size_t i = 0; i < leaves.size(); i++) {
      int k = (int)i;
      while (k >= 0) {
        if (leaves[i] < n[(size_t)k].value) n[(size_t)k].value = leaves[i];
        k = n[(size_t)k].parent;
      }
    }
  }
};

// packet header bits (B.10.1): after a 0xFF byte only 7 bits are used
struct BitIn {
  const uint8_t* p;
  const uint8_t* end;
  uint32_t buf = 0;
  int ct = 0;
  void bytein() {
    buf = (buf << 8) & 0xFFFF;
    ct = buf == 0xFF00 ? 7 : 8;
    if (p < end) buf |= *p++;
  }
  int bit() {
    if (ct == 0) bytein();
    ct--;
    return (int)((buf >> ct) & 1);
  }
  uint32_t bits(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | (uint32_t)bit();
    return v;
  }
  void align() {
    if ((buf & 0xFF) == 0xFF) bytein();
    ct = 0;
  }
};

int tgt_decode(TagTree& t, BitIn& b, int leaf, int threshold) {
  int stk[40], sp = 0;
  int k = leaf;
  while (t.n[(size_t)k].parent >= 0) {
    stk[sp++] = k;
    k = t.n[(size_t)k].parent;
  }
  int low = 0;
  for (;;) {
    TagTree::Node& q = t.n[(size_t)k];
    if (low > q.low) q.low = low;
    else low = q.low;
    while (low < threshold && low < q.value) {
      if (b.bit()) q.value = low;
      else low++;
    }
    q.low = low;
    if (sp == 0) break;
    k = stk[--sp];
  }
  return t.n[(size_t)k].value < threshold ? 1 : 0;
}

// ---------------------------------------------------------------------------
// tile structures
struct CBlk {
  int x0, y0, x1, y1;  // band coordinates
  bool seen = false;
  int numbps = 0, npasses = 0, lblock = 3;
  std::vector<uint8_t> data;
  // this packet's contribution (header pass)
  int np_pkt = 0, len_pkt = 0;
};
struct Band {
  int orient;        // 0 LL, 1 HL, 2 LH, 3 HH
  int x0, y0, x1, y1;
  int cbw, cbh;      // code-block size exponents (after the precinct limit)
  int Mb;            // magnitude bits (guard + exponent - 1)
  float step;        // irreversible: quantisation step
  int px, py;        // position in the tile-component plane
  int cbx0, cby0, ncbx, ncby;  // code-block grid
  std::vector<CBlk> cb;
};
struct Precinct {
  // per band: the precinct's code-blocks (grid indices into Band::cb) and trees
  int bx0[3], by0[3], nw[3], nh[3];
  TagTree incl[3], imsb[3];
};
struct Res {
  int x0, y0, x1, y1;
  int ppx, ppy, npx, npy;
  int nbands;
  Band band[3];
  std::vector<Precinct> prc;
};
struct TCState {
  Cod cod;
  Qcd qcd;
  int prec = 8;
  std::vector<Res> res;
};

void band_geometry(const TileComp& tc, const Cod& cod, const Qcd& qcd, int prec, TCState* s) {
  const int NL = cod.nlevels;
  s->res.assign((size_t)NL + 1, Res());
  for (int r = 0; r <= NL; r++) {
    Res& R = s->res[(size_t)r];
    R.x0 = tc.rx0[r];
    R.y0 = tc.ry0[r];
    R.x1 = tc.rx1[r];
    R.y1 = tc.ry1[r];
    R.ppx = cod.ppx[r];
    R.ppy = cod.ppy[r];
    R.npx = R.x1 > R.x0 ? ceil_pow2(R.x1, R.ppx) - (R.x0 >> R.ppx) : 0;
    R.npy = R.y1 > R.y0 ? ceil_pow2(R.y1, R.ppy) - (R.y0 >> R.ppy) : 0;
    R.nbands = r == 0 ? 1 : 3;
    for (int b = 0; b < R.nbands; b++) {
      Band& B = R.band[b];
      B.orient = r == 0 ? 0 : b + 1;
      const int nb = r == 0 ? NL : NL - r + 1;  // decomposition level of the band
      const int xob = (B.orient == 1 || B.orient == 3) ? 1 : 0;
      const int yob = (B.orient == 2 || B.orient == 3) ? 1 : 0;
      const int64_t sx = nb > 0 ? ((int64_t)1 << (nb - 1)) * xob : 0;
      const int64_t sy = nb > 0 ? ((int64_t)1 << (nb - 1)) * yob : 0;
      B.x0 = nb > 0 ? ceil_pow2((int64_t)tc.x0 - sx, nb) : tc.x0;
      B.x1 = nb > 0 ? ceil_pow2((int64_t)tc.x1 - sx, nb) : tc.x1;
      B.y0 = nb > 0 ? ceil_pow2((int64_t)tc.y0 - sy, nb) : tc.y0;
      B.y1 = nb > 0 ? ceil_pow2((int64_t)tc.y1 - sy, nb) : tc.y1;
      const int pw = r == 0 ? R.ppx : R.ppx - 1, ph = r == 0 ? R.ppy : R.ppy - 1;
      B.cbw = std::min(cod.cbw, pw);
      B.cbh = std::min(cod.cbh, ph);
      // quantisation: the band's index in QCD order (LL, then HL LH HH per level)
      const int bi = r == 0 ? 0 : 3 * (r - 1) + b + 1;
      int expn, mant;
      if (qcd.style == 1) {
        expn = qcd.expn[0] - NL + nb;  // E-5: derived from the LL band's
        mant = qcd.mant[0];
        if (r == 0) expn = qcd.expn[0];
      } else {
        const int k = std::min(bi, qcd.nexp - 1);
        expn = qcd.expn[k];
        mant = qcd.mant[k];
      }
      B.Mb = qcd.guard + expn - 1;
      const int gain = B.orient == 0 ? 0 : B.orient == 3 ? 2 : 1;
      B.step = (float)((1.0 + mant / 2048.0) * std::pow(2.0, (double)(prec + gain - expn)));
      // plane position: LL of the lower resolution at the origin, HL to its
      // right, LH below it, HH below-right
      const int lw = r == 0 ? 0 : tc.rx1[r - 1] - tc.rx0[r - 1];
      const int lh = r == 0 ? 0 : tc.ry1[r - 1] - tc.ry0[r - 1];
      B.px = (B.orient == 1 || B.orient == 3) ? lw : 0;
      B.py = (B.orient == 2 || B.orient == 3) ? lh : 0;
      if (B.x1 > B.x0 && B.y1 > B.y0) {
        B.cbx0 = B.x0 >> B.cbw;
        B.cby0 = B.y0 >> B.cbh;
        B.ncbx = ceil_pow2(B.x1, B.cbw) - B.cbx0;
        B.ncby = ceil_pow2(B.y1, B.cbh) - B.cby0;
      } else {
        B.cbx0 = B.cby0 = B.ncbx = B.ncby = 0;
      }
      B.cb.assign((size_t)B.ncbx * B.ncby, CBlk());
      for (int j = 0; j < B.ncby; j++)
        for (int i = 0; i < B.ncbx; i++) {
          CBlk& c = B.cb[(size_t)j * B.ncbx + i];
          c.x0 = std::max(B.x0, (B.cbx0 + i) << B.cbw);
          c.x1 = std::min(B.x1, (B.cbx0 + i + 1) << B.cbw);
          c.y0 = std::max(B.y0, (B.cby0 + j) << B.cbh);
          c.y1 = std::min(B.y1, (B.cby0 + j + 1) << B.cbh);
        }
    }
    // precincts: in band coordinates a precinct of resolution r > 0 is
    // 2^(PP - 1) wide
    R.prc.assign((size_t)R.npx * R.npy, Precinct());
    for (int py = 0; py < R.npy; py++)
      for (int px = 0; px < R.npx; px++) {
        Precinct& P = R.prc[(size_t)py * R.npx + px];
        for (int b = 0; b < R.nbands; b++) {
          const Band& B = R.band[b];
          const int sh = r == 0 ? 0 : 1;
          const int pxs = R.ppx - sh, pys = R.ppy - sh;
          const int gx = (R.x0 >> R.ppx) + px, gy = (R.y0 >> R.ppy) + py;  // precinct grid index
          int bx0 = std::max(B.x0, gx << pxs), bx1 = std::min(B.x1, (gx + 1) << pxs);
          int by0 = std::max(B.y0, gy << pys), by1 = std::min(B.y1, (gy + 1) << pys);
          if (B.ncbx == 0 || bx1 <= bx0 || by1 <= by0) {
            P.nw[b] = P.nh[b] = 0;
            P.bx0[b] = P.by0[b] = 0;
          } else {
            P.bx0[b] = (bx0 >> B.cbw) - B.cbx0;
            P.by0[b] = (by0 >> B.cbh) - B.cby0;
            P.nw[b] = ceil_pow2(bx1, B.cbw) - (bx0 >> B.cbw);
            P.nh[b] = ceil_pow2(by1, B.cbh) - (by0 >> B.cbh);
          }
          P.incl[b].init(P.nw[b], P.nh[b]);
          P.imsb[b].init(P.nw[b], P.nh[b]);
        }
      }
  }
}

int getnumpasses(BitIn& b) {
  if (!b.bit()) return 1;
  if (!b.bit()) return 2;
  int n = (int)b.bits(2);
  if (n != 3) return 3 + n;
  n = (int)b.bits(5);
  if (n != 31) return 6 + n;
  return 37 + (int)b.bits(7);
}

// One packet (B.10): header, then the code-blocks' contributions.  Returns
// false on truncated / inconsistent data.
bool read_packet(const uint8_t*& p, const uint8_t* end, const Cod& cod, Res& R, int prcno,
                 int layer) {
  if (prcno >= (int)R.prc.size()) return true;  // no such precinct: no packet
  if ((cod.scod & 2) && end - p >= 6 && p[0] == 0xFF && p[1] == 0x91) p += 6;  // SOP
  Precinct& P = R.prc[(size_t)prcno];
  BitIn bi{p, end};
  const int present = bi.bit();
  std::vector<CBlk*> inc;
  if (present) {
    for (int b = 0; b < R.nbands; b++) {
      Band& B = R.band[b];
      for (int j = 0; j < P.nh[b]; j++)
        for (int i = 0; i < P.nw[b]; i++) {
          CBlk& c = B.cb[(size_t)(P.by0[b] + j) * B.ncbx + (P.bx0[b] + i)];
          const int leaf = j * P.nw[b] + i;
          int included;
          if (!c.seen) included = tgt_decode(P.incl[b], bi, leaf, layer + 1);
          else included = bi.bit();
          if (!included) continue;
          if (!c.seen) {
            int z = 0;
            while (!tgt_decode(P.imsb[b], bi, leaf, z)) {
              if (++z > 64) return false;
            }
            c.numbps = B.Mb + 1 - z;
            c.seen = true;
            c.lblock = 3;
          }
          const int np = getnumpasses(bi);
          int inc_l = 0;
          while (bi.bit()) inc_l++;
          c.lblock += inc_l;
          const int nbits = c.lblock + floor_log2((uint32_t)np);
          if (nbits > 31) return false;
          c.np_pkt = np;
          c.len_pkt = (int)bi.bits(nbits);
          inc.push_back(&c);
        }
    }
  }
  bi.align();
  p = bi.p;
  if ((cod.scod & 4) && end - p >= 2 && p[0] == 0xFF && p[1] == 0x92) p += 2;  // EPH
  for (CBlk* c : inc) {
    if (end - p < c->len_pkt) return false;
    c->data.insert(c->data.end(), p, p + c->len_pkt);
    c->npasses += c->np_pkt;
    p += c->len_pkt;
  }
  return true;
}

struct Siz {
  int32_t X, Y, XO, YO, XT, YT, XTO, YTO, C;
  int prec[kMaxComps], sgnd[kMaxComps], dx[kMaxComps], dy[kMaxComps];
};

// the codestream inside a JP2 file (the jp2c box), or the data itself
bool find_codestream(const uint8_t* d, size_t n, const char* name, const uint8_t** cs,
                     size_t* csn) {
  if (n >= 4 && d[0] == 0xFF && d[1] == 0x4F && d[2] == 0xFF && d[3] == 0x51) {
    *cs = d;
    *csn = n;
    return true;
  }
  size_t pos = 0;
  while (pos + 8 <= n) {
    uint64_t len = (uint64_t)d[pos] << 24 | (uint64_t)d[pos + 1] << 16 | (uint64_t)d[pos + 2] << 8 | d[pos + 3];
    const uint32_t type = (uint32_t)d[pos + 4] << 24 | (uint32_t)d[pos + 5] << 16 |
                          (uint32_t)d[pos + 6] << 8 | d[pos + 7];
    size_t hdr = 8;
    if (len == 1) {
      if (pos + 16 > n) break;
      len = 0;
      for (int i = 0; i < 8; i++) len = (len << 8) | d[pos + 8 + i];
      hdr = 16;
    } else if (len == 0) {
      len = n - pos;
    }
    if (len < hdr || pos + len > n) break;
    if (type == 0x6A703263u) {  // 'jp2c'
      *cs = d + pos + hdr;
      *csn = (size_t)len - hdr;
      return true;
    }
    pos += (size_t)len;
  }
  return jfail(name, "no JPEG 2000 codestream");
}

bool read_siz(Reader& r, const char* name, Siz* s) {
  const uint32_t len = r.u16();
  const uint8_t* end = r.p + len - 2;
  r.u16();  // Rsiz
  s->X = (int32_t)r.u32();
  s->Y = (int32_t)r.u32();
  s->XO = (int32_t)r.u32();
  s->YO = (int32_t)r.u32();
  s->XT = (int32_t)r.u32();
  s->YT = (int32_t)r.u32();
  s->XTO = (int32_t)r.u32();
  s->YTO = (int32_t)r.u32();
  s->C = (int)r.u16();
  // (offsets read as int32: a u32 above INT_MAX is negative and refused; the
  // first tile must overlap the image area, A.5.1)
  if (!r.ok || s->X <= 0 || s->Y <= 0 || s->XT <= 0 || s->YT <= 0 || s->XO < 0 || s->YO < 0 ||
      s->XTO < 0 || s->YTO < 0 || s->X <= s->XO || s->Y <= s->YO || s->XTO > s->XO ||
      s->YTO > s->YO || (int64_t)s->XTO + s->XT <= s->XO || (int64_t)s->YTO + s->YT <= s->YO)
    return jfail(name, "bad SIZ");
  if (s->C != 1 && s->C != 3) return jfail(name, "only 1- and 3-component images are supported");
  for (int c = 0; c < s->C; c++) {
    const int v = (int)r.u8();
    s->prec[c] = (v & 0x7F) + 1;
    s->sgnd[c] = v >> 7;
    s->dx[c] = (int)r.u8();
    s->dy[c] = (int)r.u8();
    if (s->prec[c] != 8 || s->sgnd[c]) return jfail(name, "only 8-bit unsigned components are supported");
    if (s->dx[c] != 1 || s->dy[c] != 1) return jfail(name, "subsampled components are not supported");
  }
  if ((int64_t)(s->X - s->XO) * (s->Y - s->YO) > ((int64_t)1 << 28))  // 16k x 16k
    return jfail(name, "image too large");
  r.p = end;
  return r.ok;
}

// main header up to the first SOT; tile-parts' data collected per tile
struct Stream {
  Siz siz;
  Params main;
  std::vector<std::vector<uint8_t>> tile_data;
  std::vector<int> tile_has_params;
  std::vector<Params> tile_params;
};

bool read_marker_segment(Reader& r, const char* name, int m, const Siz& siz, Params& P,
                         bool* cod_seen) {
  const uint8_t* seg = r.p;
  const uint32_t len = r.u16();
  if (!r.ok || len < 2 || (size_t)(r.end - seg) < len) return jfail(name, "truncated marker segment");
  const uint8_t* end = seg + len;
  switch (m) {
    case 0xFF52: {  // COD
      Cod c;
      c.scod = (int)r.u8();
      c.prog = (int)r.u8();
      c.layers = (int)r.u16();
      c.mct = (int)r.u8();
      if (!read_spcod(r, c, c.scod & 1)) return jfail(name, "bad COD");
      for (int k = 0; k < siz.C; k++) P.cod[k] = c;
      *cod_seen = true;
      break;
    }
    case 0xFF53: {  // COC
      const int k = siz.C >= 257 ? (int)r.u16() : (int)r.u8();
      if (k >= siz.C) return jfail(name, "bad COC");
      Cod c = P.cod[k];
      c.scod = (c.scod & ~1) | ((int)r.u8() & 1);
      if (!read_spcod(r, c, c.scod & 1)) return jfail(name, "bad COC");
      P.cod[k] = c;
      break;
    }
    case 0xFF5C: {  // QCD
      Qcd q;
      if (!read_sqcd(r, end, q)) return jfail(name, "bad QCD");
      for (int k = 0; k < siz.C; k++) P.qcd[k] = q;
      break;
    }
    case 0xFF5D: {  // QCC
      const int k = siz.C >= 257 ? (int)r.u16() : (int)r.u8();
      if (k >= siz.C) return jfail(name, "bad QCC");
      Qcd q;
      if (!read_sqcd(r, end, q)) return jfail(name, "bad QCC");
      P.qcd[k] = q;
      break;
    }
    case 0xFF5E:
      return jfail(name, "region of interest (RGN) is not supported");
    case 0xFF5F:
      return jfail(name, "progression order changes (POC) are not supported");
    case 0xFF60:
    case 0xFF61:
      return jfail(name, "packed packet headers (PPM/PPT) are not supported");
    default:  // TLM, PLM, PLT, CRG, COM, ...: skipped
      break;
  }
  r.p = end;
  return true;
}

bool read_stream(const uint8_t* d, size_t n, const char* name, Stream* S, bool header_only) {
  const uint8_t* cs;
  size_t csn;
  if (!find_codestream(d, n, name, &cs, &csn)) return false;
  Reader r{cs, cs + csn, name};
  if (r.u16() != 0xFF4F) return jfail(name, "no SOC marker");
  if (r.u16() != 0xFF51) return jfail(name, "SIZ must follow SOC");
  if (!read_siz(r, name, &S->siz)) return false;
  if (header_only) return true;
  bool cod_seen = false;
  for (;;) {
    const uint32_t m = r.u16();
    if (!r.ok) return jfail(name, "truncated main header");
    if (m == 0xFF90) break;
    if (m == 0xFFD9) return jfail(name, "no tiles");
    if (!read_marker_segment(r, name, (int)m, S->siz, S->main, &cod_seen)) return false;
  }
  if (!cod_seen) return jfail(name, "no COD marker");
  const Siz& z = S->siz;
  const int ntx = ceildiv((int64_t)z.X - z.XTO, z.XT), nty = ceildiv((int64_t)z.Y - z.YTO, z.YT);
  if ((int64_t)ntx * nty > 65535) return jfail(name, "too many tiles");
  S->tile_data.assign((size_t)ntx * nty, std::vector<uint8_t>());
  S->tile_has_params.assign((size_t)ntx * nty, 0);
  S->tile_params.assign((size_t)ntx * nty, S->main);
  // tile-parts: SOT already read
  for (;;) {
    const uint8_t* sot = r.p - 2;
    const uint32_t lsot = r.u16();
    const int isot = (int)r.u16();
    const uint32_t psot = r.u32();
    const int tpsot = (int)r.u8();
    r.u8();  // TNsot
    if (!r.ok || lsot != 10 || isot >= ntx * nty) return jfail(name, "bad SOT");
    const uint8_t* tp_end = psot ? sot + psot : r.end;
    if (tp_end > r.end) {
      tp_end = r.end;  // truncated last tile-part: decode what there is
    }
    Params& TP = S->tile_params[(size_t)isot];
    bool tcod = false;
    for (;;) {
      const uint32_t m = r.u16();
      if (!r.ok) return jfail(name, "truncated tile-part header");
      if (m == 0xFF93) break;  // SOD
      if (tpsot != 0 && (m == 0xFF52 || m == 0xFF53 || m == 0xFF5C || m == 0xFF5D))
        return jfail(name, "coding parameters in a later tile-part");
      if (!read_marker_segment(r, name, (int)m, z, TP, &tcod)) return false;
    }
    if (r.p > tp_end) return jfail(name, "bad tile-part length");
    auto& td = S->tile_data[(size_t)isot];
    td.insert(td.end(), r.p, tp_end);
    r.p = tp_end;
    if (r.end - r.p < 2) break;
    const uint32_t m = r.u16();
    if (m == 0xFFD9) break;  // EOC
    if (m != 0xFF90) return jfail(name, "expected SOT or EOC");
  }
  return true;
}

// tile-component geometry (B.3, B.5)
// (tile bounds in int64: XTO + (tx + 1) * XT overflows int32 for large XT;
// clipped to the image, so the results fit again)
void tile_geometry(const Siz& z, int tx, int ty, int ntx, const Params& P, Tile* T) {
  T->x0 = (int32_t)std::max<int64_t>(z.XTO + (int64_t)tx * z.XT, z.XO);
  T->x1 = (int32_t)std::min<int64_t>(z.XTO + (int64_t)(tx + 1) * z.XT, z.X);
  T->y0 = (int32_t)std::max<int64_t>(z.YTO + (int64_t)ty * z.YT, z.YO);
  T->y1 = (int32_t)std::min<int64_t>(z.YTO + (int64_t)(ty + 1) * z.YT, z.Y);
  (void)ntx;
  T->mct = (z.C == 3 && P.cod[0].mct) ? 1 : 0;
  for (int c = 0; c < z.C; c++) {
    TileComp& tc = T->tc[c];
    tc.x0 = T->x0;  // XRsiz = YRsiz = 1
    tc.y0 = T->y0;
    tc.x1 = T->x1;
    tc.y1 = T->y1;
    tc.nlevels = P.cod[c].nlevels;
    for (int r = 0; r <= tc.nlevels; r++) {
      const int s = tc.nlevels - r;
      tc.rx0[r] = ceil_pow2(tc.x0, s);
      tc.ry0[r] = ceil_pow2(tc.y0, s);
      tc.rx1[r] = ceil_pow2(tc.x1, s);
      tc.ry1[r] = ceil_pow2(tc.y1, s);
    }
    tc.stride = tc.x1 - tc.x0;
  }
}

// packets of a tile in its progression order (B.12.1)
bool read_packets(const std::vector<uint8_t>& data, const char* name, const Cod& c0, int ncomp,
                  std::vector<TCState>& st, const Tile& T) {
  const uint8_t* p = data.data();
  const uint8_t* end = p + data.size();
  int maxres = 0;
  for (int c = 0; c < ncomp; c++) maxres = std::max(maxres, st[(size_t)c].cod.nlevels + 1);
  const int L = c0.layers;
  auto packet = [&](int l, int r, int c, int k) -> bool {
    TCState& S = st[(size_t)c];
    if (r > S.cod.nlevels) return true;
    if (p >= end) return true;  // truncated: the rest is empty
    return read_packet(p, end, S.cod, S.res[(size_t)r], k, l);
  };
  // precinct start of (c, r, k) on the tile's reference grid, for the
  // position-driven orders
  struct Pos {
    int64_t y, x;
    int c, r, k;
  };
  auto positions = [&]() {
    std::vector<Pos> v;
    for (int c = 0; c < ncomp; c++) {
      const TCState& S = st[(size_t)c];
      for (int r = 0; r <= S.cod.nlevels; r++) {
        const Res& R = S.res[(size_t)r];
        const int sh = S.cod.nlevels - r;
        for (int py = 0; py < R.npy; py++)
          for (int px = 0; px < R.npx; px++) {
            const int64_t gx = (int64_t)((R.x0 >> R.ppx) + px) << R.ppx;
            const int64_t gy = (int64_t)((R.y0 >> R.ppy) + py) << R.ppy;
            const int64_t x = std::max<int64_t>(T.x0, gx << sh);
            const int64_t y = std::max<int64_t>(T.y0, gy << sh);
            v.push_back(Pos{y, x, c, r, py * R.npx + px});
          }
      }
    }
    return v;
  };
  switch (c0.prog) {
    case 0:  // LRCP
      for (int l = 0; l < L; l++)
        for (int r = 0; r < maxres; r++)
          for (int c = 0; c < ncomp; c++) {
            if (r > st[(size_t)c].cod.nlevels) continue;
            const Res& R = st[(size_t)c].res[(size_t)r];
            for (int k = 0; k < R.npx * R.npy; k++)
              if (!packet(l, r, c, k)) return jfail(name, "corrupt packet");
          }
      break;
    case 1:  // RLCP
      for (int r = 0; r < maxres; r++)
        for (int l = 0; l < L; l++)
          for (int c = 0; c < ncomp; c++) {
            if (r > st[(size_t)c].cod.nlevels) continue;
            const Res& R = st[(size_t)c].res[(size_t)r];
            for (int k = 0; k < R.npx * R.npy; k++)
              if (!packet(l, r, c, k)) return jfail(name, "corrupt packet");
          }
      break;
    case 2: {  // RPCL: resolution, then position (y, x), component, layer
      std::vector<Pos> v = positions();
      std::stable_sort(v.begin(), v.end(), [](const Pos& a, const Pos& b) {
        if (a.r != b.r) return a.r < b.r;
        if (a.y != b.y) return a.y < b.y;
        if (a.x != b.x) return a.x < b.x;
        return a.c < b.c;
      });
      for (const Pos& q : v)
        for (int l = 0; l < L; l++)
          if (!packet(l, q.r, q.c, q.k)) return jfail(name, "corrupt packet");
      break;
    }
    case 3: {  // PCRL: position, component, resolution, layer
      std::vector<Pos> v = positions();
      std::stable_sort(v.begin(), v.end(), [](const Pos& a, const Pos& b) {
        if (a.y != b.y) return a.y < b.y;
        if (a.x != b.x) return a.x < b.x;
        if (a.c != b.c) return a.c < b.c;
        return a.r < b.r;
      });
      for (const Pos& q : v)
        for (int l = 0; l < L; l++)
          if (!packet(l, q.r, q.c, q.k)) return jfail(name, "corrupt packet");
      break;
    }
    case 4: {  // CPRL: component, position, resolution, layer
      std::vector<Pos> v = positions();
      std::stable_sort(v.begin(), v.end(), [](const Pos& a, const Pos& b) {
        if (a.c != b.c) return a.c < b.c;
        if (a.y != b.y) return a.y < b.y;
        if (a.x != b.x) return a.x < b.x;
        return a.r < b.r;
      });
      for (const Pos& q : v)
        for (int l = 0; l < L; l++)
          if (!packet(l, q.r, q.c, q.k)) return jfail(name, "corrupt packet");
      break;
    }
    default:
      return jfail(name, "unknown progression order");
  }
  return true;
}

}  // namespace

bool is_j2k(const uint8_t* d, size_t n) {
  static const uint8_t sig[12] = {0x00, 0x00, 0x00, 0x0C, 0x6A, 0x50, 0x20, 0x20, 0x0D, 0x0A, 0x87, 0x0A};
  if (n >= 4 && d[0] == 0xFF && d[1] == 0x4F && d[2] == 0xFF && d[3] == 0x51) return true;
  return n >= 12 && memcmp(d, sig, 12) == 0;
}

bool probe(const uint8_t* d, size_t n, const char* name, UphipPnmInfo* info) {
  Stream S;
  if (!read_stream(d, n, name, &S, true)) return false;
  info->width = S.siz.X - S.siz.XO;
  info->height = S.siz.Y - S.siz.YO;
  info->format = S.siz.C == 1 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24;
  return true;
}

bool decode_host(const uint8_t* d, size_t n, const char* name, Image* img,
                 std::vector<uint32_t>* coef, T1Batch* t1) {
  try {
    std::unique_ptr<Stream> Sp(new Stream);
    Stream& S = *Sp;
    if (!read_stream(d, n, name, &S, false)) return false;
    const Siz& z = S.siz;
    img->width = z.X - z.XO;
    img->height = z.Y - z.YO;
    img->ncomp = z.C;
    img->x0 = z.XO;
    img->y0 = z.YO;
    img->reversible = S.main.cod[0].reversible;
    const int ntx = ceildiv((int64_t)z.X - z.XTO, z.XT), nty = ceildiv((int64_t)z.Y - z.YTO, z.YT);
    img->tiles.assign((size_t)ntx * nty, Tile());
    int64_t total = 0;
    for (int t = 0; t < ntx * nty; t++) {
      const Params& P = S.tile_params[(size_t)t];
      for (int c = 0; c < z.C; c++) {
        if (P.cod[c].reversible != img->reversible)
          return jfail(name, "mixed reversible and irreversible components");
        if (P.cod[c].cbsty != 0) return jfail(name, "code-block styles other than 0 are not supported");
        if (P.cod[c].cbw > 10 || P.cod[c].cbh > 10 || P.cod[c].cbw + P.cod[c].cbh > 12)
          return jfail(name, "bad code-block size");
      }
      Tile& T = img->tiles[(size_t)t];
      tile_geometry(z, t % ntx, t / ntx, ntx, P, &T);
      if (T.x1 <= T.x0 || T.y1 <= T.y0) return jfail(name, "empty tile");
      for (int c = 0; c < z.C; c++) {
        T.tc[c].off = total;
        total += (int64_t)(T.tc[c].x1 - T.tc[c].x0) * (T.tc[c].y1 - T.tc[c].y0);
      }
    }
    img->coef_elems = total;
    if (t1) {
      t1->jobs.clear();
      t1->data.clear();
      t1->maxw = t1->maxh = 0;
    } else {
      coef->assign((size_t)total, 0u);
    }
    std::vector<uint8_t> flags;
    std::vector<int32_t> vals;
    std::vector<uint8_t> buf;
    for (int t = 0; t < ntx * nty; t++) {
      const Params& P = S.tile_params[(size_t)t];
      Tile& T = img->tiles[(size_t)t];
      std::vector<TCState> st((size_t)z.C);
      for (int c = 0; c < z.C; c++) {
        st[(size_t)c].cod = P.cod[c];
        st[(size_t)c].qcd = P.qcd[c];
        st[(size_t)c].prec = z.prec[c];
        band_geometry(T.tc[c], P.cod[c], P.qcd[c], z.prec[c], &st[(size_t)c]);
      }
      if (!read_packets(S.tile_data[(size_t)t], name, P.cod[0], z.C, st, T)) return false;
      // Tier 1 into the planes
      for (int c = 0; c < z.C; c++) {
        const TileComp& tc = T.tc[c];
        uint32_t* plane = t1 ? nullptr : coef->data() + tc.off;
        for (auto& R : st[(size_t)c].res)
          for (int b = 0; b < R.nbands; b++) {
            Band& B = R.band[b];
            for (CBlk& cb : B.cb) {
              if (cb.npasses == 0 || cb.data.empty()) continue;
              const int w = cb.x1 - cb.x0, h = cb.y1 - cb.y0;
              if (w <= 0 || h <= 0) continue;
              if (cb.numbps <= 0 || cb.numbps > 30) return jfail(name, "bad code-block bit-planes");
              if (t1) {  // for the device decoder
                T1Job job;
                job.data = (uint32_t)t1->data.size();
                job.len = (uint32_t)cb.data.size();
                job.out = tc.off + (int64_t)(B.py + cb.y0 - B.y0) * tc.stride + (B.px + cb.x0 - B.x0);
                job.stride = tc.stride;
                job.w = (uint16_t)w;
                job.h = (uint16_t)h;
                job.orient = (uint8_t)B.orient;
                job.numbps = (uint8_t)cb.numbps;
                // passes past plane 1 decode nothing
                job.npasses = (uint8_t)std::min(cb.npasses, 3 * cb.numbps - 2);
                job.pad = 0;
                job.halfstep = img->reversible ? 0.0f : 0.5f * B.step;
                t1->jobs.push_back(job);
                t1->data.insert(t1->data.end(), cb.data.begin(), cb.data.end());
                t1->data.push_back(0xFF);
                t1->data.push_back(0xFF);
                while (t1->data.size() & 3) t1->data.push_back(0);
                t1->maxw = std::max(t1->maxw, w);
                t1->maxh = std::max(t1->maxh, h);
                if (t1->data.size() > 0xFFFFFFF0u) return jfail(name, "code-block data too large");
                continue;
              }
              flags.assign((size_t)(w + 2) * (h + 2), 0);
              vals.assign((size_t)w * h, 0);
              buf.assign(cb.data.begin(), cb.data.end());
              buf.push_back(0xFF);
              buf.push_back(0xFF);
              CodeBlockCoder cc;
              cc.w = w;
              cc.h = h;
              cc.orient = B.orient;
              cc.fs = w + 2;
              cc.f = flags.data();
              cc.v = vals.data();
              cc.decode(buf.data(), cb.npasses, cb.numbps);
              for (int y = 0; y < h; y++) {
                uint32_t* row = plane + (int64_t)(B.py + cb.y0 - B.y0 + y) * tc.stride +
                                (B.px + cb.x0 - B.x0);
                for (int x = 0; x < w; x++) {
                  const int32_t q = vals[(size_t)y * w + x];
                  if (img->reversible) {
                    row[x] = (uint32_t)(q / 2);
                  } else {
                    const float f = (float)q * (0.5f * B.step);
                    memcpy(&row[x], &f, 4);
                  }
                }
              }
            }
          }
      }
    }
    if (t1) t1->data.insert(t1->data.end(), 16, 0);  // the decoder's read-ahead
    if (t1)  // alike blocks share a wave: by width, height, then passes
      std::stable_sort(t1->jobs.begin(), t1->jobs.end(), [](const T1Job& x, const T1Job& y) {
        if (x.w != y.w) return x.w > y.w;
        if (x.h != y.h) return x.h > y.h;
        return x.npasses > y.npasses;
      });
    return true;
  } catch (const std::bad_alloc&) {
    return fail("jp2: %s: out of memory", name);
  }
}


// ---------------------------------------------------------------------------
// Lossless encoder: one tile, one layer, LRCP, 64 x 64 code-blocks, the
// default (maximal) precincts, reversible 5/3 with the RCT for RGB, no
// quantisation (QCD style 0), two guard bits unless a code-block needs more.
namespace {

struct BitOut {
  std::vector<uint8_t>* out;
  uint32_t buf = 0;
  int ct = 8;
  void byteout() {  // OpenJPEG bio.c: a byte after 0xFF carries 7 bits
    buf = (buf << 8) & 0xFFFF;
    ct = buf == 0xFF00 ? 7 : 8;
    out->push_back((uint8_t)(buf >> 8));
  }
  void bit(int b) {
    if (ct == 0) byteout();
    ct--;
    buf |= (uint32_t)b << ct;
  }
  void bits(uint32_t v, int n) {
    for (int i = n - 1; i >= 0; i--) bit((int)((v >> i) & 1));
  }
  void flush() {
    byteout();
    if (ct == 7) byteout();
  }
};

void tgt_encode(TagTree& t, BitOut& b, int leaf, int threshold) {
  int stk[40], sp = 0;
  int k = leaf;
  while (t.n[(size_t)k].parent >= 0) {
    stk[sp++] = k;
    k = t.n[(size_t)k].parent;
  }
  int low = 0;
  for (;;) {
    TagTree::Node& q = t.n[(size_t)k];
    if (low > q.low) q.low = low;
    else low = q.low;
    while (low < threshold) {
      if (low >= q.value) {
        if (!q.known) {
          b.bit(1);
          q.known = 1;
        }
        break;
      }
      b.bit(0);
      low++;
    }
    q.low = low;
    if (sp == 0) break;
    k = stk[--sp];
  }
}

void putnumpasses(BitOut& b, int n) {
  if (n == 1) b.bit(0);
  else if (n == 2) b.bits(2, 2);
  else if (n <= 5) b.bits(0xC | (uint32_t)(n - 3), 4);
  else if (n <= 36) b.bits(0x1E0 | (uint32_t)(n - 6), 9);
  else b.bits(0xFF80 | (uint32_t)(n - 37), 16);
}

void put16(std::vector<uint8_t>& o, uint32_t v) {
  o.push_back((uint8_t)(v >> 8));
  o.push_back((uint8_t)v);
}
void put32(std::vector<uint8_t>& o, uint32_t v) {
  put16(o, v >> 16);
  put16(o, v & 0xFFFF);
}

int encode_levels(int32_t w, int32_t h) {
  int nl = 0;
  while (nl < 5 && (w >> (nl + 1)) >= 1 && (h >> (nl + 1)) >= 1) nl++;
  return nl;
}

}  // namespace

bool encode_geometry(int32_t w, int32_t h, int32_t ncomp, Image* img) {
  if (w <= 0 || h <= 0 || (ncomp != 1 && ncomp != 3)) return fail("jp2 encode: bad geometry");
  if ((int64_t)w * h > ((int64_t)1 << 30)) return fail("jp2 encode: image too large");
  img->width = w;
  img->height = h;
  img->ncomp = ncomp;
  img->x0 = img->y0 = 0;
  img->reversible = 1;
  img->tiles.assign(1, Tile());
  Tile& T = img->tiles[0];
  T.x0 = T.y0 = 0;
  T.x1 = w;
  T.y1 = h;
  T.mct = ncomp == 3 ? 1 : 0;
  const int NL = encode_levels(w, h);
  for (int c = 0; c < ncomp; c++) {
    TileComp& tc = T.tc[c];
    tc.x0 = tc.y0 = 0;
    tc.x1 = w;
    tc.y1 = h;
    tc.nlevels = NL;
    for (int r = 0; r <= NL; r++) {
      tc.rx0[r] = tc.ry0[r] = 0;
      tc.rx1[r] = ceil_pow2(w, NL - r);
      tc.ry1[r] = ceil_pow2(h, NL - r);
    }
    tc.stride = w;
    tc.off = (int64_t)c * w * h;
  }
  img->coef_elems = (int64_t)ncomp * w * h;
  return true;
}

namespace {

// the encoder's coding parameters and code-block geometry, per component
void encode_params(const Image& img, std::vector<TCState>* st) {
  const Tile& T = img.tiles[0];
  const int C = img.ncomp, NL = T.tc[0].nlevels;
  Cod cod;
  cod.scod = 0;
  cod.prog = 0;
  cod.layers = 1;
  cod.mct = T.mct;
  cod.nlevels = NL;
  cod.cbw = cod.cbh = 6;
  cod.cbsty = 0;
  cod.reversible = 1;
  st->assign((size_t)C, TCState());
  for (int c = 0; c < C; c++) {
    Qcd q;
    q.guard = 2;
    q.style = 0;
    q.nexp = 3 * NL + 1;
    for (int i = 0; i < q.nexp; i++) {
      const int orient = i == 0 ? 0 : (i - 1) % 3 + 1;
      const int gain = orient == 0 ? 0 : orient == 3 ? 2 : 1;
      q.expn[i] = 8 + gain;  // OpenJPEG: exponent = precision + band gain, MCT or not
      q.mant[i] = 0;
    }
    (*st)[(size_t)c].cod = cod;
    (*st)[(size_t)c].qcd = q;
    band_geometry(T.tc[c], cod, q, 8, &(*st)[(size_t)c]);
  }
}

}  // namespace

bool encode_jobs(const Image& img, std::vector<T1EncJob>* jobs, size_t* out_bytes) {
  try {
    std::vector<TCState> st;
    encode_params(img, &st);
    jobs->clear();
    size_t o = 0;
    for (int c = 0; c < img.ncomp; c++) {
      const TileComp& tc = img.tiles[0].tc[c];
      for (auto& R : st[(size_t)c].res)
        for (int b = 0; b < R.nbands; b++) {
          const Band& B = R.band[b];
          for (const CBlk& cb : B.cb) {
            const int bw = cb.x1 - cb.x0, bh = cb.y1 - cb.y0;
            if (bw <= 0 || bh <= 0) continue;
            T1EncJob j{};
            j.in = tc.off + (int64_t)(B.py + cb.y0 - B.y0) * tc.stride + (B.px + cb.x0 - B.x0);
            j.stride = tc.stride;
            j.w = (uint16_t)bw;
            j.h = (uint16_t)bh;
            j.out = (uint32_t)o;
            j.orient = (uint8_t)B.orient;
            jobs->push_back(j);
            o += (t1_enc_cap(bw, bh) + 15) & ~15u;
            if (o > 0xFFFFFFF0u) return fail("jp2 encode: image too large");
          }
        }
    }
    *out_bytes = o;
    return true;
  } catch (const std::bad_alloc&) {
    return fail("jp2 encode: out of memory");
  }
}

namespace {
bool encode_finish(const Image& img, const uint32_t* coef, const uint32_t* doff,
                   const uint32_t* dlen, const uint8_t* dnb, const uint8_t* ddata,
                   std::vector<uint8_t>* out);
}  // namespace

bool encode_host(const Image& img, const uint32_t* coef, std::vector<uint8_t>* out) {
  return encode_finish(img, coef, nullptr, nullptr, nullptr, nullptr, out);
}
bool encode_host_coded(const Image& img, const uint32_t* off, const uint32_t* len,
                       const uint8_t* nb, const uint8_t* data, std::vector<uint8_t>* out) {
  return encode_finish(img, nullptr, off, len, nb, data, out);
}

namespace {
// the code-blocks coded here (coef) or taken from the device (off / len / nb
// / data, in encode_jobs' order), then packets, codestream and JP2 boxes
bool encode_finish(const Image& img, const uint32_t* coef, const uint32_t* doff,
                   const uint32_t* dlen, const uint8_t* dnb, const uint8_t* ddata,
                   std::vector<uint8_t>* out) {
  try {
    const Tile& T = img.tiles[0];
    const int C = img.ncomp, NL = T.tc[0].nlevels;
    const int w = img.width, h = img.height;
    const int ebase = 8;  // OpenJPEG: exponent = precision + band gain, MCT or not
    std::vector<TCState> st;
    encode_params(img, &st);
    // code every code-block; the magnitude bits set the guard bits
    int guard = 2;
    std::vector<uint8_t> flags, buf;
    std::vector<int32_t> vals;
    size_t bi = 0;  // block index in encode_jobs' order
    for (int c = 0; c < C; c++) {
      const TileComp& tc = T.tc[c];
      for (int r = 0; r <= NL; r++) {
        Res& R = st[(size_t)c].res[(size_t)r];
        for (int b = 0; b < R.nbands; b++) {
          Band& B = R.band[b];
          for (CBlk& cb : B.cb) {
            const int bw = cb.x1 - cb.x0, bh = cb.y1 - cb.y0;
            cb.npasses = 0;
            cb.data.clear();
            if (bw <= 0 || bh <= 0) continue;
            if (!coef) {  // coded on the device
              const int nb = dnb[bi];
              cb.numbps = nb;
              if (nb > 0) {
                cb.npasses = 3 * nb - 2;
                cb.data.assign(ddata + doff[bi], ddata + doff[bi] + dlen[bi]);
                while (guard + B.Mb - 2 < nb) guard++;
              }
              bi++;
              continue;
            }
            vals.resize((size_t)bw * bh);
            for (int y = 0; y < bh; y++) {
              const uint32_t* row = coef + tc.off + (int64_t)(B.py + cb.y0 - B.y0 + y) * tc.stride +
                                    (B.px + cb.x0 - B.x0);
              for (int x = 0; x < bw; x++) vals[(size_t)y * bw + x] = (int32_t)row[x];
            }
            flags.assign((size_t)(bw + 2) * (bh + 2), 0);
            CodeBlockCoder cc;
            cc.w = bw;
            cc.h = bh;
            cc.orient = B.orient;
            cc.fs = bw + 2;
            cc.f = flags.data();
            cc.v = vals.data();
            const int nb = cc.numbps_of();
            cb.numbps = nb;
            if (nb == 0) continue;
            buf.assign((size_t)bw * bh * 16 + 1024, 0);
            int np = 0;
            const int64_t len = cc.encode(buf.data(), nb, &np);
            cb.npasses = np;
            cb.data.assign(buf.begin() + 1, buf.begin() + 1 + len);
            // Mb = guard + expn - 1 must cover the code-block's planes
            while (guard + B.Mb - 2 < nb) guard++;  // B.Mb was computed with guard 2
          }
        }
      }
    }
    if (guard > 7) return fail("jp2 encode: coefficients too large");
    // packets (LRCP, one layer): header + body per (r, c, precinct 0)
    std::vector<uint8_t> body;
    for (int r = 0; r <= NL; r++)
      for (int c = 0; c < C; c++) {
        Res& R = st[(size_t)c].res[(size_t)r];
        for (int k = 0; k < R.npx * R.npy; k++) {
          Precinct& P = R.prc[(size_t)k];
          std::vector<uint8_t> hdr;
          BitOut bo{&hdr};
          bool any = false;
          for (int b = 0; b < R.nbands; b++) {
            Band& B = R.band[b];
            if (P.nw[b] == 0 || P.nh[b] == 0) continue;
            std::vector<int> incl((size_t)P.nw[b] * P.nh[b]), zbp(incl.size());
            for (int j = 0; j < P.nh[b]; j++)
              for (int i = 0; i < P.nw[b]; i++) {
                const CBlk& cb = B.cb[(size_t)(P.by0[b] + j) * B.ncbx + (P.bx0[b] + i)];
                incl[(size_t)j * P.nw[b] + i] = cb.npasses > 0 ? 0 : 1;
                zbp[(size_t)j * P.nw[b] + i] = (guard + B.Mb - 2) - cb.numbps;  // empty: all planes
                any |= cb.npasses > 0;
              }
            P.incl[b].set_values(incl);
            P.imsb[b].set_values(zbp);
          }
          // OpenJPEG (t2.c) writes every packet as present, an all-empty one
          // as zero inclusion bits; the bytes then equal its encoder's
          (void)any;
          {
            bo.bit(1);
            for (int b = 0; b < R.nbands; b++) {
              Band& B = R.band[b];
              for (int j = 0; j < P.nh[b]; j++)
                for (int i = 0; i < P.nw[b]; i++) {
                  CBlk& cb = B.cb[(size_t)(P.by0[b] + j) * B.ncbx + (P.bx0[b] + i)];
                  const int leaf = j * P.nw[b] + i;
                  tgt_encode(P.incl[b], bo, leaf, 1);
                  if (cb.npasses == 0) continue;
                  tgt_encode(P.imsb[b], bo, leaf, 999);
                  putnumpasses(bo, cb.npasses);
                  const int len = (int)cb.data.size();
                  const int lp = floor_log2((uint32_t)cb.npasses);
                  const int need = len > 0 ? floor_log2((uint32_t)len) + 1 : 1;
                  const int incr = std::max(0, need - (cb.lblock + lp));
                  for (int q = 0; q < incr; q++) bo.bit(1);
                  bo.bit(0);
                  cb.lblock += incr;
                  bo.bits((uint32_t)len, cb.lblock + lp);
                }
            }
          }
          bo.flush();
          body.insert(body.end(), hdr.begin(), hdr.end());
          for (int b = 0; b < R.nbands; b++) {
            Band& B = R.band[b];
            for (int j = 0; j < P.nh[b]; j++)
              for (int i = 0; i < P.nw[b]; i++) {
                const CBlk& cb = B.cb[(size_t)(P.by0[b] + j) * B.ncbx + (P.bx0[b] + i)];
                if (cb.npasses) body.insert(body.end(), cb.data.begin(), cb.data.end());
              }
          }
        }
      }
    // codestream
    std::vector<uint8_t> cs;
    put16(cs, 0xFF4F);  // SOC
    put16(cs, 0xFF51);  // SIZ
    put16(cs, (uint32_t)(38 + 3 * C));
    put16(cs, 0);
    put32(cs, (uint32_t)w);
    put32(cs, (uint32_t)h);
    put32(cs, 0);
    put32(cs, 0);
    put32(cs, (uint32_t)w);
    put32(cs, (uint32_t)h);
    put32(cs, 0);
    put32(cs, 0);
    put16(cs, (uint32_t)C);
    for (int c = 0; c < C; c++) {
      cs.push_back(7);
      cs.push_back(1);
      cs.push_back(1);
    }
    put16(cs, 0xFF52);  // COD
    put16(cs, 12);
    cs.push_back(0);                    // Scod: default precincts, no SOP / EPH
    cs.push_back(0);                    // LRCP
    put16(cs, 1);                       // one layer
    cs.push_back((uint8_t)T.mct);       // RCT for RGB
    cs.push_back((uint8_t)NL);
    cs.push_back(4);                    // 64 x 64 code-blocks
    cs.push_back(4);
    cs.push_back(0);                    // code-block style 0
    cs.push_back(1);                    // reversible 5/3
    put16(cs, 0xFF5C);  // QCD
    put16(cs, (uint32_t)(3 + 3 * NL + 1));
    cs.push_back((uint8_t)(guard << 5));  // no quantisation
    for (int i = 0; i < 3 * NL + 1; i++) {
      const int orient = i == 0 ? 0 : (i - 1) % 3 + 1;
      const int gain = orient == 0 ? 0 : orient == 3 ? 2 : 1;
      cs.push_back((uint8_t)((ebase + gain) << 3));
    }
    const size_t sot = cs.size();
    put16(cs, 0xFF90);  // SOT
    put16(cs, 10);
    put16(cs, 0);
    put32(cs, (uint32_t)(14 + body.size()));  // Psot: SOT .. end of the tile-part
    cs.push_back(0);
    cs.push_back(1);
    put16(cs, 0xFF93);  // SOD
    (void)sot;
    cs.insert(cs.end(), body.begin(), body.end());
    put16(cs, 0xFFD9);  // EOC
    // JP2 boxes: signature, file type, header (ihdr, colr), codestream
    std::vector<uint8_t>& o = *out;
    o.clear();
    const uint8_t sig[12] = {0x00, 0x00, 0x00, 0x0C, 0x6A, 0x50, 0x20, 0x20, 0x0D, 0x0A, 0x87, 0x0A};
    o.insert(o.end(), sig, sig + 12);
    put32(o, 20);
    put32(o, 0x66747970);  // ftyp
    put32(o, 0x6A703220);  // 'jp2 '
    put32(o, 0);
    put32(o, 0x6A703220);
    put32(o, 8 + 22 + 15);
    put32(o, 0x6A703268);  // jp2h
    put32(o, 22);
    put32(o, 0x69686472);  // ihdr
    put32(o, (uint32_t)h);
    put32(o, (uint32_t)w);
    put16(o, (uint32_t)C);
    o.push_back(7);  // 8 bits unsigned
    o.push_back(7);  // JPEG 2000 compression
    o.push_back(0);
    o.push_back(0);
    put32(o, 15);
    put32(o, 0x636F6C72);  // colr
    o.push_back(1);         // enumerated colour space
    o.push_back(0);
    o.push_back(0);
    put32(o, C == 3 ? 16u : 17u);  // sRGB / greyscale
    put32(o, (uint32_t)(8 + cs.size()));
    put32(o, 0x6A703263);  // jp2c
    o.insert(o.end(), cs.begin(), cs.end());
    return true;
  } catch (const std::bad_alloc&) {
    return fail("jp2 encode: out of memory");
  }
}
}  // namespace

}  // namespace j2k
}  // namespace uph

using namespace uph;

namespace {

constexpr int kT1MaxSlots = 1024;  // k_j2k_t1 workgroups (scratch slots) of one launch

bool j2k_decode_to_device(const uint8_t* data, size_t size, const char* name, uint8_t* ddst,
                          int64_t pitch, UphipPnmInfo* info) {
  j2k::Image img;
  j2k::T1Batch tb;
  if (!j2k::decode_host(data, size, name, &img, nullptr, &tb)) return false;
  const int fmt = img.ncomp == 1 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24;
  if (info) {
    if (info->width > 0 && (info->width != img.width || info->height != img.height || info->format != fmt))
      return fail("jp2: %s is %dx%d format %d, expected %dx%d format %d", name, img.width, img.height,
                  fmt, info->width, info->height, info->format);
    info->width = img.width;
    info->height = img.height;
    info->format = fmt;
  }
  if (pitch < (int64_t)img.width * img.ncomp) return fail("jp2: pitch too small");
  // code-block jobs and codewords up, coefficients decoded on the device
  hipStream_t st = current_stream();
  const int njobs = (int)tb.jobs.size();
  const size_t jb = (sizeof(j2k::T1Job) * (size_t)njobs + 255) & ~(size_t)255;
  const int nslots = std::min((njobs + 63) / 64, kT1MaxSlots);
  uint8_t* dup = (uint8_t*)scratch(3, jb + tb.data.size() + 4);
  uint32_t* dc = (uint32_t*)scratch(6, (size_t)img.coef_elems * 4 + 4);
  void* tmp = scratch(7, j2k::decode_tmp_bytes(img));
  void* t1s = scratch(4, (size_t)std::max(nslots, 1) * j2k::t1_slot_bytes(tb.maxw, tb.maxh));
  return dup && dc && tmp && t1s &&
         (njobs == 0 || UPH_HIP(hipMemcpyAsync(dup, tb.jobs.data(), sizeof(j2k::T1Job) * (size_t)njobs,
                                               hipMemcpyHostToDevice, st))) &&
         (tb.data.empty() || UPH_HIP(hipMemcpyAsync(dup + jb, tb.data.data(), tb.data.size(),
                                                    hipMemcpyHostToDevice, st))) &&
         UPH_HIP(hipMemsetAsync(dc, 0, (size_t)img.coef_elems * 4, st)) &&
         j2k::t1_launch((const j2k::T1Job*)dup, njobs, dup + jb, dc, t1s, nslots, tb.maxw, tb.maxh, st) &&
         j2k::decode_launch(img, dc, ddst, pitch, tmp, st) && UPH_HIP(hipStreamSynchronize(st));
}

bool read_whole(const char* path, std::vector<uint8_t>* buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return fail("jp2: cannot open %s", path);
  bool ok = fseek(f, 0, SEEK_END) == 0;
  const long sz = ok ? ftell(f) : -1;
  ok = ok && sz >= 0 && sz < (1l << 31) && fseek(f, 0, SEEK_SET) == 0;
  if (ok) {
    buf->resize((size_t)sz);
    ok = fread(buf->data(), 1, (size_t)sz, f) == (size_t)sz;
  }
  fclose(f);
  return ok || fail("jp2: cannot read %s", path);
}

}  // namespace

extern "C" {

int uphip_jp2_probe(const char* path, UphipPnmInfo* info) {
  if (!path || !info) return fail("jp2_probe: null argument"), -1;
  std::vector<uint8_t> buf;
  if (!read_whole(path, &buf)) return -1;
  return j2k::probe(buf.data(), buf.size(), path, info) ? 0 : -1;
}

int uphip_jp2_decode(const void* data, size_t size, void* device_dst, int64_t pitch,
                     UphipPnmInfo* info) {
  if (!data || !device_dst) return fail("jp2_decode: null argument"), -1;
  if (!runtime_ready()) return fail("jp2_decode: no HIP device"), -1;
  return j2k_decode_to_device((const uint8_t*)data, size, "<memory>", (uint8_t*)device_dst, pitch,
                              info)
             ? 0
             : -1;
}

int uphip_jp2_read(const char* path, void* dst, int64_t linesize, const UphipPnmInfo* expect) {
  if (!path || !dst) return fail("jp2_read: null argument"), -1;
  if (!runtime_ready()) return fail("jp2_read: no HIP device (JPEG 2000 decodes on the device)"), -1;
  std::vector<uint8_t> file;
  if (!read_whole(path, &file)) return -1;
  UphipPnmInfo info{0, 0, 0};
  if (!j2k::probe(file.data(), file.size(), path, &info)) return -1;
  if (expect && (expect->width != info.width || expect->height != info.height ||
                 expect->format != info.format))
    return fail("jp2: %s is %dx%d format %d, expected %dx%d format %d", path, info.width,
                info.height, info.format, expect->width, expect->height, expect->format),
           -1;
  const int64_t rb = (int64_t)info.width * (info.format == UPHIP_FMT_GRAY8 ? 1 : 3);
  if (linesize < rb) return fail("jp2_read: linesize too small"), -1;
  const int64_t dpitch = (rb + 255) & ~(int64_t)255;
  uint8_t* dd = (uint8_t*)scratch(2, (size_t)(dpitch * info.height));
  if (!dd || !j2k_decode_to_device(file.data(), file.size(), path, dd, dpitch, &info)) return -1;
  return UPH_HIP(hipMemcpy2D(dst, (size_t)linesize, dd, (size_t)dpitch, (size_t)rb,
                             (size_t)info.height, hipMemcpyDeviceToHost))
             ? 0
             : -1;
}

int64_t uphip_jp2_entropy_decode(const void* data, size_t size, void* coef, int64_t capacity,
                                 UphipPnmInfo* info) {
  if (!data) return fail("jp2_entropy_decode: null argument"), -1;
  j2k::Image img;
  std::vector<uint32_t> c;
  if (!j2k::decode_host((const uint8_t*)data, size, "<memory>", &img, &c)) return -1;
  if (info) {
    info->width = img.width;
    info->height = img.height;
    info->format = img.ncomp == 1 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24;
  }
  const int64_t bytes = (int64_t)c.size() * 4;
  if (coef && capacity >= bytes) memcpy(coef, c.data(), (size_t)bytes);
  return bytes;
}

int64_t uphip_jp2_encode(const void* device_src, int64_t pitch, int32_t width, int32_t height,
                         int32_t format, void* out, int64_t capacity) {
  if (!device_src) return fail("jp2_encode: null argument"), -1;
  if (format != UPHIP_FMT_GRAY8 && format != UPHIP_FMT_RGB24)
    return fail("jp2_encode: GRAY8 or RGB24 only"), -1;
  if (!runtime_ready()) return fail("jp2_encode: no HIP device"), -1;
  const int ncomp = format == UPHIP_FMT_GRAY8 ? 1 : 3;
  if (pitch < (int64_t)width * ncomp) return fail("jp2_encode: pitch too small"), -1;
  j2k::Image img;
  if (!j2k::encode_geometry(width, height, ncomp, &img)) return -1;
  std::vector<j2k::T1EncJob> jobs;
  size_t obytes = 0;
  if (!j2k::encode_jobs(img, &jobs, &obytes)) return -1;
  const int njobs = (int)jobs.size();
  int maxw = 1, maxh = 1;
  for (const j2k::T1EncJob& j : jobs) {
    maxw = std::max(maxw, (int)j.w);
    maxh = std::max(maxh, (int)j.h);
  }
  // device: forward transforms, code-blocks, codewords packed; host: packets
  hipStream_t st = current_stream();
  const int nslots = std::min((njobs + 63) / 64, kT1MaxSlots);
  const size_t jb = (sizeof(j2k::T1EncJob) * (size_t)njobs + 255) & ~(size_t)255;
  const size_t lb = ((size_t)njobs * 4 + 4 + 255) & ~(size_t)255;
  uint32_t* dc = (uint32_t*)scratch(6, (size_t)img.coef_elems * 4);
  uint8_t* dj = (uint8_t*)scratch(3, jb);
  void* t1s = scratch(4, (size_t)std::max(nslots, 1) * j2k::t1enc_slot_bytes(maxw, maxh));
  uint8_t* dw = (uint8_t*)scratch(5, obytes + 2 * lb + (size_t)njobs + 16);
  uint8_t* dpk = (uint8_t*)scratch(1, obytes + 16);
  void* tmp = scratch(7, (size_t)img.coef_elems * 4);
  if (!dc || !dj || !t1s || !dw || !dpk || !tmp) return -1;
  uint32_t* dlen = (uint32_t*)(dw + obytes);
  uint32_t* doff = (uint32_t*)(dw + obytes + lb);
  uint8_t* dnb = dw + obytes + 2 * lb;
  std::vector<uint32_t> off((size_t)njobs + 1), len((size_t)njobs);
  std::vector<uint8_t> nb((size_t)njobs);
  if (!j2k::encode_launch(img, (const uint8_t*)device_src, pitch, dc, tmp, st) ||
      !UPH_HIP(hipMemcpyAsync(dj, jobs.data(), sizeof(j2k::T1EncJob) * (size_t)njobs,
                              hipMemcpyHostToDevice, st)) ||
      !j2k::t1enc_launch((const j2k::T1EncJob*)dj, njobs, dc, dw, dlen, dnb, t1s, nslots, maxw, maxh,
                         st) ||
      !j2k::t1enc_pack((const j2k::T1EncJob*)dj, njobs, dw, dlen, doff, dpk, obytes, nullptr, false, st) ||
      !UPH_HIP(hipMemcpyAsync(off.data(), doff, 4 * ((size_t)njobs + 1), hipMemcpyDeviceToHost, st)) ||
      !UPH_HIP(hipMemcpyAsync(len.data(), dlen, 4 * (size_t)njobs, hipMemcpyDeviceToHost, st)) ||
      !UPH_HIP(hipMemcpyAsync(nb.data(), dnb, (size_t)njobs, hipMemcpyDeviceToHost, st)) ||
      !UPH_HIP(hipStreamSynchronize(st)))
    return -1;
  for (uint8_t v : nb)
    if (v > 16)
      return fail(v == 0xFE ? "jp2_encode: a code-block's codeword outgrew its region"
                            : "jp2_encode: coefficients beyond 16 bits"),
             -1;
  std::vector<uint8_t> packed((size_t)off[(size_t)njobs] + 1);
  if (off[(size_t)njobs] &&
      !UPH_HIP(hipMemcpy(packed.data(), dpk, off[(size_t)njobs], hipMemcpyDeviceToHost)))
    return -1;
  std::vector<uint8_t> file;
  if (!j2k::encode_host_coded(img, off.data(), len.data(), nb.data(), packed.data(), &file)) return -1;
  if (out && capacity >= (int64_t)file.size()) memcpy(out, file.data(), file.size());
  return (int64_t)file.size();
}

}  // extern "C"
