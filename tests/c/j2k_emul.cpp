// j2k_emul.cpp — TEST INFRASTRUCTURE: the JPEG 2000 decode with the device
// half (csrc/kernels_j2k.hip: inverse wavelet per level, rows then columns,
// inverse component transform, DC shift) replayed on the CPU with the same
// line functions (csrc/j2k_dwt.h), after the library's host half
// (j2k::decode_host), so that the CPU suite checks the decoder against PIL
// (OpenJPEG) without a GPU; likewise the lossless encode (the device's
// forward transforms replayed, then j2k::encode_host).  Built by
// `make j2k_emul`.
#include <cstdint>
#include <cstring>
#include <vector>

#include "j2k.h"
#include "j2k_dwt.h"

using namespace uph::j2k;

extern "C" {

// Decodes `file` into out (rows of width * ncomp bytes); returns the byte
// count (written when cap suffices) or -1 (uphip_last_error); info3 =
// {width, height, ncomp}.
int64_t j2k_emulate(const uint8_t* file, size_t n, uint8_t* out, int64_t cap, int32_t* info3) {
  Image img;
  std::vector<uint32_t> coef;
  if (!decode_host(file, n, "<emul>", &img, &coef)) return -1;
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

// Encodes `src` (rows of w * ncomp bytes) as the device path would; returns
// the file size (written when cap suffices) or -1.
int64_t j2k_emulate_encode(const uint8_t* src, int32_t w, int32_t h, int32_t ncomp, uint8_t* out,
                           int64_t cap) {
  Image img;
  if (!encode_geometry(w, h, ncomp, &img)) return -1;
  std::vector<uint32_t> coef((size_t)img.coef_elems);
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
  std::vector<int32_t> tmp((size_t)n);
  const Tile& t = img.tiles[0];
  for (int c = 0; c < ncomp; c++) {
    const TileComp& tc = t.tc[c];
    int32_t* plane = (int32_t*)(coef.data() + tc.off);
    for (int r = tc.nlevels; r >= 1; r--) {
      const int rw = tc.rx1[r] - tc.rx0[r], rh = tc.ry1[r] - tc.ry0[r];
      for (int x = 0; x < rw; x++) {  // k_j2k_fcols
        for (int i = 0; i < rh; i++) tmp[(size_t)i * rw + x] = plane[(int64_t)i * tc.stride + x];
        fdwt53_line(tmp.data() + x, rh, tc.ry0[r] & 1, rw);
        deinterleave(tmp.data() + x, rw, rh, tc.ry0[r] & 1, plane + x, tc.stride);
      }
      for (int y = 0; y < rh; y++) {  // k_j2k_frows
        int32_t* row = plane + (int64_t)y * tc.stride;
        int32_t* tl = tmp.data() + (int64_t)y * rw;
        memcpy(tl, row, 4 * (size_t)rw);
        fdwt53_line(tl, rw, tc.rx0[r] & 1, 1);
        deinterleave(tl, 1, rw, tc.rx0[r] & 1, row, 1);
      }
    }
  }
  std::vector<uint8_t> file;
  if (!encode_host(img, coef.data(), &file)) return -1;
  if (out && cap >= (int64_t)file.size()) memcpy(out, file.data(), file.size());
  return (int64_t)file.size();
}

}  // extern "C"
