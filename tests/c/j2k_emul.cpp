// j2k_emul.cpp — TEST INFRASTRUCTURE: the JPEG 2000 decode with the device
// half (csrc/kernels_j2k.hip: inverse wavelet per level, rows then columns,
// inverse component transform, DC shift) replayed on the CPU with the same
// line functions (csrc/j2k_dwt.h), after the library's host half
// (j2k::decode_host), so that the CPU suite checks the decoder against PIL
// (OpenJPEG) without a GPU; likewise the lossless encode (the device's
// forward transforms replayed, then j2k::encode_host).  Built by
// `make j2k_emul`.
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <vector>

#include "j2k.h"
#include "j2k_dwt.h"
#include "j2k_t1_lane.h"

using namespace uph::j2k;

extern "C" {

// Decodes `file` into out (rows of width * ncomp bytes); returns the byte
// count (written when cap suffices) or -1 (uphip_last_error); info3 =
// {width, height, ncomp}.
static int64_t finish(const Image& img, std::vector<uint32_t>& coef, uint8_t* out, int64_t cap,
                      int32_t* info3, bool pairs = false);

int64_t j2k_emulate(const uint8_t* file, size_t n, uint8_t* out, int64_t cap, int32_t* info3) {
  Image img;
  std::vector<uint32_t> coef;
  if (!decode_host(file, n, "<emul>", &img, &coef)) return -1;
  return finish(img, coef, out, cap, info3);
}

// The same with the code-blocks through the device decoder's lane code
// (j2k_t1_lane.h, LS = 1): every job of a 64-job group decoded with the
// group's width, height and pass count as the kernel's lanes are.
int64_t j2k_emulate_t1lane(const uint8_t* file, size_t n, uint8_t* out, int64_t cap,
                           int32_t* info3) {
  Image img;
  T1Batch tb;
  if (!decode_host(file, n, "<emul>", &img, nullptr, &tb)) return -1;
  std::vector<uint32_t> coef((size_t)img.coef_elems, 0u);
  MqState qe[47];
  for (int i = 0; i < 47; i++) qe[i] = kMq[i];
  uint8_t zct[kZcTable];
  zc_table(zct);
  const int njobs = (int)tb.jobs.size();
  std::vector<uint16_t> fl;
  std::vector<uint32_t> val;
  uint8_t cx[kNumCtx];
  for (int g0 = 0; g0 < njobs; g0 += 64) {
    int Wg = 0, Hg = 0, P = 0;
    for (int j = g0; j < njobs && j < g0 + 64; j++) {
      Wg = std::max(Wg, (int)tb.jobs[(size_t)j].w);
      Hg = std::max(Hg, (int)tb.jobs[(size_t)j].h);
      P = std::max(P, (int)tb.jobs[(size_t)j].npasses);
    }
    for (int j = g0; j < njobs && j < g0 + 64; j++) {
      const T1Job& job = tb.jobs[(size_t)j];
      fl.assign((size_t)((Hg + 3) / 4 + 2) * (Wg + 2), 0xABCD);  // the lane code zeroes them
      val.assign((size_t)Hg * Wg, 0x5A5A5A5A);
      T1Lane<1> L;
      L.WS = Wg + 2;
      L.Wg = Wg;
      L.fl = fl.data();
      L.val = val.data();
      L.cx = cx;
      L.qe = qe;
      L.zct = zct;
      L.w = job.w;
      L.h = job.h;
      L.orient = job.orient;
      t1_decode_lane(L, true, tb.data.data() + job.data, job.numbps, job.npasses, (Hg + 3) / 4, P,
                     [](bool b) { return b; });
      t1_store_lane(L, true, job, coef.data(), Hg);
    }
  }
  return finish(img, coef, out, cap, info3, true);
}

// the inverse pair kernels (k_j2k_irow / k_j2k_icol) on the CPU
extern "C++" {
template <class T, int CAS>
static void pair_level(T* plane, T* tmp, int stride, int rw, int rh) {
  for (int y = 0; y < rh; y++)
    for (int t = 0; 2 * t < rw; t++) {
      T o0, o1;
      idwt_pair<T, CAS>(plane + (int64_t)y * stride, 1, rw, t, &o0, &o1);
      tmp[(int64_t)y * stride + 2 * t] = o0;
      if (2 * t + 1 < rw) tmp[(int64_t)y * stride + 2 * t + 1] = o1;
    }
}
template <class T, int CAS>
static void pair_cols(T* tmp, T* plane, int stride, int rw, int rh) {
  for (int x = 0; x < rw; x++)
    for (int t = 0; 2 * t < rh; t++) {
      T o0, o1;
      idwt_pair<T, CAS>(tmp + x, stride, rh, t, &o0, &o1);
      plane[(int64_t)(2 * t) * stride + x] = o0;
      if (2 * t + 1 < rh) plane[(int64_t)(2 * t + 1) * stride + x] = o1;
    }
}
template <class T>
static void pair_2d(T* plane, T* tmp, int stride, int rw, int rh, int cx, int cy) {
  if (cx) pair_level<T, 1>(plane, tmp, stride, rw, rh);
  else pair_level<T, 0>(plane, tmp, stride, rw, rh);
  if (cy) pair_cols<T, 1>(tmp, plane, stride, rw, rh);
  else pair_cols<T, 0>(tmp, plane, stride, rw, rh);
}
}  // extern "C++"

static int64_t finish(const Image& img, std::vector<uint32_t>& coef, uint8_t* out, int64_t cap,
                      int32_t* info3, bool pairs) {
  info3[0] = img.width;
  info3[1] = img.height;
  info3[2] = img.ncomp;
  const int64_t bytes = (int64_t)img.width * img.height * img.ncomp;
  if (!out || cap < bytes) return bytes;
  std::vector<uint32_t> tmp;
  for (const Tile& t : img.tiles) {
    for (int c = 0; c < img.ncomp; c++) {
      const TileComp& tc = t.tc[c];
      for (int r = 1; r <= tc.nlevels; r++) {
        const int rw = tc.rx1[r] - tc.rx0[r], rh = tc.ry1[r] - tc.ry0[r];
        if (rw <= 0 || rh <= 0) continue;
        uint32_t* plane = coef.data() + tc.off;
        tmp.assign((size_t)rw * rh, 0u);
        const int cx = tc.rx0[r] & 1, cy = tc.ry0[r] & 1;
        if (pairs) {  // as the device does
          std::vector<uint32_t> t2((size_t)tc.stride * rh);
          if (img.reversible) pair_2d((int32_t*)plane, (int32_t*)t2.data(), tc.stride, rw, rh, cx, cy);
          else pair_2d((float*)plane, (float*)t2.data(), tc.stride, rw, rh, cx, cy);
          continue;
        }
        for (int y = 0; y < rh; y++) {  // k_j2k_rows
          uint32_t* row = plane + (int64_t)y * tc.stride;
          uint32_t* tl = tmp.data() + (int64_t)y * rw;
          interleave(row, 1, rw, cx, tl, 1);
          if (img.reversible) idwt53_line((int32_t*)tl, rw, cx, 1);
          else idwt97_line((float*)tl, rw, cx, 1);
          memcpy(row, tl, 4 * (size_t)rw);
        }
        for (int x = 0; x < rw; x++) {  // k_j2k_cols
          interleave(plane + x, tc.stride, rh, cy, tmp.data() + x, rw);
          if (img.reversible) idwt53_line((int32_t*)(tmp.data() + x), rh, cy, rw);
          else idwt97_line((float*)(tmp.data() + x), rh, cy, rw);
          for (int i = 0; i < rh; i++) plane[(int64_t)i * tc.stride + x] = tmp[(size_t)i * rw + x];
        }
      }
    }
    const int w = t.x1 - t.x0, h = t.y1 - t.y0;
    for (int y = 0; y < h; y++)  // k_j2k_out
      for (int x = 0; x < w; x++) {
        auto at = [&](int c) { return coef[(size_t)(t.tc[c].off + (int64_t)y * t.tc[c].stride + x)]; };
        uint8_t* d = out + ((int64_t)(t.y0 + y - img.y0) * img.width + (t.x0 + x - img.x0)) * img.ncomp;
        auto f = [](uint32_t u) {
          float v;
          memcpy(&v, &u, 4);
          return v;
        };
        if (img.ncomp == 1) {
          d[0] = img.reversible ? clamp8((int32_t)at(0) + 128) : clamp8(round_half_even(f(at(0))) + 128);
          continue;
        }
        if (img.reversible) {
          if (t.mct) {
            rct_inverse((int32_t)at(0), (int32_t)at(1), (int32_t)at(2), d, d + 1, d + 2);
          } else {
            for (int c = 0; c < 3; c++) d[c] = clamp8((int32_t)at(c) + 128);
          }
        } else if (t.mct) {
          ict_inverse(f(at(0)), f(at(1)), f(at(2)), d, d + 1, d + 2);
        } else {
          for (int c = 0; c < 3; c++) d[c] = clamp8(round_half_even(f(at(c))) + 128);
        }
      }
  }
  return bytes;
}

// The pair-at-a-time lifting (j2k_dwt.h, the device kernels' form) against
// the sequential in-place lifting for every line length 1..nmax, both
// parities, 5/3 both ways and 9/7 inverse, on seeded data; returns the
// number of mismatching samples.
int64_t j2k_dwt_check(int nmax, uint32_t seed) {
  int64_t bad = 0;
  uint32_t rs = seed;
  auto rnd = [&]() { rs = rs * 1664525u + 1013904223u; return rs >> 8; };
  for (int n = 1; n <= nmax; n++)
    for (int cas = 0; cas < 2; cas++) {
      std::vector<int32_t> a(n), nat(n), m(n);
      std::vector<float> fa(n), fnat(n);
      for (int i = 0; i < n; i++) {
        a[i] = (int32_t)(rnd() % 2001) - 1000;
        fa[i] = (float)((int32_t)(rnd() % 20001) - 10000) * 0.037f;
      }
      // inverse 5/3 and 9/7: Mallat -> natural
      std::vector<int32_t> ref(n);
      std::vector<float> fref(n);
      interleave(a.data(), 1, n, cas, ref.data(), 1);
      idwt53_line(ref.data(), n, cas, 1);
      interleave(fa.data(), 1, n, cas, fref.data(), 1);
      idwt97_line(fref.data(), n, cas, 1);
      for (int t = 0; 2 * t < n; t++) {
        int32_t o0 = 0, o1 = 0;
        float f0 = 0, f1 = 0;
        if (cas) {
          idwt_pair<int32_t, 1>(a.data(), 1, n, t, &o0, &o1);
          idwt_pair<float, 1>(fa.data(), 1, n, t, &f0, &f1);
        } else {
          idwt_pair<int32_t, 0>(a.data(), 1, n, t, &o0, &o1);
          idwt_pair<float, 0>(fa.data(), 1, n, t, &f0, &f1);
        }
        bad += o0 != ref[2 * t];
        bad += memcmp(&f0, &fref[2 * t], 4) != 0;
        if (2 * t + 1 < n) {
          bad += o1 != ref[2 * t + 1];
          bad += memcmp(&f1, &fref[2 * t + 1], 4) != 0;
        }
      }
      // forward 5/3: natural -> Mallat
      std::vector<int32_t> fw(a);
      fdwt53_line(fw.data(), n, cas, 1);
      std::vector<int32_t> fm(n);
      deinterleave(fw.data(), 1, n, cas, fm.data(), 1);
      for (int t = 0; 2 * t < n; t++) {
        int32_t o0 = 0, o1 = 0;
        if (cas) fdwt53_pair<1>(a.data(), 1, n, t, &o0, &o1);
        else fdwt53_pair<0>(a.data(), 1, n, t, &o0, &o1);
        bad += o0 != fm[mallat_index(2 * t, n, cas)];
        if (2 * t + 1 < n) bad += o1 != fm[mallat_index(2 * t + 1, n, cas)];
      }
    }
  return bad;
}

// The device's forward transforms on the CPU (k_j2k_in, k_j2k_fcol /
// k_j2k_frow through the pair functions) into img's coefficient planes.
static bool emul_forward(const uint8_t* src, int32_t w, int32_t h, int32_t ncomp, Image* img,
                         std::vector<uint32_t>* coefp) {
  if (!encode_geometry(w, h, ncomp, img)) return false;
  std::vector<uint32_t>& coef = *coefp;
  coef.assign((size_t)img->coef_elems, 0u);
  const int64_t n = (int64_t)w * h;
  for (int64_t i = 0; i < n; i++) {  // k_j2k_in
    const uint8_t* s = src + i * ncomp;
    if (ncomp == 1) {
      coef[(size_t)i] = (uint32_t)((int32_t)s[0] - 128);
      continue;
    }
    const int32_t R = s[0] - 128, G = s[1] - 128, B = s[2] - 128;
    coef[(size_t)i] = (uint32_t)((R + 2 * G + B) >> 2);
    coef[(size_t)(n + i)] = (uint32_t)(B - G);
    coef[(size_t)(2 * n + i)] = (uint32_t)(R - G);
  }
  const Tile& t = img->tiles[0];
  for (int c = 0; c < ncomp; c++) {
    const TileComp& tc = t.tc[c];
    int32_t* plane = (int32_t*)(coef.data() + tc.off);
    for (int r = tc.nlevels; r >= 1; r--) {
      const int rw = tc.rx1[r] - tc.rx0[r], rh = tc.ry1[r] - tc.ry0[r];
      std::vector<int32_t> t2((size_t)tc.stride * rh);
      const int cx = tc.rx0[r] & 1, cy = tc.ry0[r] & 1;
      for (int x = 0; x < rw; x++)  // k_j2k_fcol: plane -> t2
        for (int t = 0; 2 * t < rh; t++) {
          int32_t o0, o1;
          if (cy) fdwt53_pair<1>(plane + x, tc.stride, rh, t, &o0, &o1);
          else fdwt53_pair<0>(plane + x, tc.stride, rh, t, &o0, &o1);
          t2[(size_t)mallat_index(2 * t, rh, cy) * tc.stride + x] = o0;
          if (2 * t + 1 < rh) t2[(size_t)mallat_index(2 * t + 1, rh, cy) * tc.stride + x] = o1;
        }
      for (int y = 0; y < rh; y++)  // k_j2k_frow: t2 -> plane
        for (int t = 0; 2 * t < rw; t++) {
          int32_t o0, o1;
          const int32_t* line = t2.data() + (size_t)y * tc.stride;
          if (cx) fdwt53_pair<1>(line, 1, rw, t, &o0, &o1);
          else fdwt53_pair<0>(line, 1, rw, t, &o0, &o1);
          plane[(int64_t)y * tc.stride + mallat_index(2 * t, rw, cx)] = o0;
          if (2 * t + 1 < rw) plane[(int64_t)y * tc.stride + mallat_index(2 * t + 1, rw, cx)] = o1;
        }
    }
  }
  return true;
}

static int64_t give(const std::vector<uint8_t>& file, uint8_t* out, int64_t cap) {
  if (out && cap >= (int64_t)file.size()) memcpy(out, file.data(), file.size());
  return (int64_t)file.size();
}

// Encodes `src` (rows of w * ncomp bytes) as the device path would, the
// code-blocks coded by j2k_t1.h's host coder; returns the file size
// (written when cap suffices) or -1.
int64_t j2k_emulate_encode(const uint8_t* src, int32_t w, int32_t h, int32_t ncomp, uint8_t* out,
                           int64_t cap) {
  Image img;
  std::vector<uint32_t> coef;
  std::vector<uint8_t> file;
  if (!emul_forward(src, w, h, ncomp, &img, &coef) || !encode_host(img, coef.data(), &file)) return -1;
  return give(file, out, cap);
}

// The same with the code-blocks through the device encoder's lane code
// (j2k_t1_lane.h, LS = 1) in 64-block groups, as k_j2k_t1enc runs them.
int64_t j2k_emulate_encode_lane(const uint8_t* src, int32_t w, int32_t h, int32_t ncomp,
                                uint8_t* out, int64_t cap) {
  Image img;
  std::vector<uint32_t> coef;
  std::vector<T1EncJob> jobs;
  size_t obytes = 0;
  if (!emul_forward(src, w, h, ncomp, &img, &coef) || !encode_jobs(img, &jobs, &obytes)) return -1;
  MqState qe[47];
  for (int i = 0; i < 47; i++) qe[i] = kMq[i];
  uint8_t zct[kZcTable];
  zc_table(zct);
  std::vector<uint8_t> odata(obytes + 16);
  const int njobs = (int)jobs.size();
  std::vector<uint32_t> off(njobs), len(njobs);
  std::vector<uint8_t> nbv(njobs);
  std::vector<uint16_t> fl;
  std::vector<uint64_t> mg;
  uint8_t cx[kNumCtx];
  for (int g0 = 0; g0 < njobs; g0 += 64) {
    const int g1 = std::min(njobs, g0 + 64);
    int Wg = 0, Hg = 0, P = 0;
    std::vector<int> nbs;
    for (int j = g0; j < g1; j++) {
      const T1EncJob& jb = jobs[(size_t)j];
      uint32_t m = 0;
      for (int y = 0; y < jb.h; y++)
        for (int x = 0; x < jb.w; x++) {
          const int32_t v = (int32_t)coef[(size_t)(jb.in + (int64_t)y * jb.stride + x)];
          m |= (uint32_t)(v < 0 ? -v : v);
        }
      int nb = 0;
      while (m) {
        nb++;
        m >>= 1;
      }
      nbs.push_back(nb);
      Wg = std::max(Wg, (int)jb.w);
      Hg = std::max(Hg, (int)jb.h);
      P = std::max(P, nb > 0 ? 3 * nb - 2 : 0);
    }
    const int Sg = (Hg + 3) / 4;
    for (int j = g0; j < g1; j++) {
      const T1EncJob& jb = jobs[(size_t)j];
      const int nb = nbs[(size_t)(j - g0)];
      fl.assign((size_t)(Sg + 2) * (Wg + 2), 0);
      mg.assign((size_t)Sg * Wg, 0);
      T1EncLane<1> L;
      L.WS = Wg + 2;
      L.Wg = Wg;
      L.fl = fl.data();
      L.mg = mg.data();
      for (int y = 0; y < jb.h; y++)
        for (int x = 0; x < jb.w; x++) {
          const int32_t v = (int32_t)coef[(size_t)(jb.in + (int64_t)y * jb.stride + x)];
          const uint32_t a = (uint32_t)(v < 0 ? -v : v);
          mg[(size_t)((y >> 2) * Wg + x)] |= (uint64_t)a << (16 * (y & 3));
          if (v < 0) L.F(y >> 2, x) |= (uint16_t)(2u << (4 * (y & 3)));
        }
      L.cx = cx;
      L.qe = qe;
      L.zct = zct;
      L.w = jb.w;
      L.h = jb.h;
      L.orient = jb.orient;
      L.out = odata.data() + jb.out;
      L.cap = (int32_t)t1_enc_cap(jb.w, jb.h);
      L.over = false;
      const int32_t n = t1_encode_lane(L, nb > 0, nb, Sg, P, [](bool b) { return b; });
      if (L.over) return -1;
      off[(size_t)j] = jb.out;
      len[(size_t)j] = (uint32_t)n;
      nbv[(size_t)j] = (uint8_t)nb;
    }
  }
  std::vector<uint8_t> file;
  if (!encode_host_coded(img, off.data(), len.data(), nbv.data(), odata.data(), &file)) return -1;
  return give(file, out, cap);
}

}  // extern "C"
