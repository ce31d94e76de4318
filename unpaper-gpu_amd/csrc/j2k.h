// j2k.h — JPEG 2000 (ISO/IEC 15444-1) decode and encode: the JP2 half of
// the reference's nvImageCodec peer (imageprocess/nvimgcodec.c:168-179
// format detection, :840 JPEG2000 decode, :1133-1165 nvimgcodec_encode_jp2).
//
// Decode: the host parses the codestream (JP2 boxes, main and tile-part
// headers), reads the packet headers (tag trees, pass counts, lengths) and
// runs the EBCOT code-block decoder (MQ arithmetic decoder, the three coding
// passes) into per-tile-component coefficient planes laid out by subband
// (each resolution's LL | HL over LH | HH, the layout the inverse wavelet
// transform works in place on); the device runs the inverse wavelet
// transforms (5/3 reversible, 9/7 irreversible), the inverse component
// transform, the DC level shift and the store into the destination image.
//
// Encode (lossless): the device runs the forward component and wavelet
// transforms; the host codes the code-blocks and writes the JP2 file (one
// tile, one quality layer, LRCP, 64x64 code-blocks, reversible 5/3).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "unpaper_hip.h"

namespace uph {
namespace j2k {

constexpr int kMaxComps = 3;
constexpr int kMaxLevels = 32;

// A tile-component's coefficient plane and what the device needs to turn it
// into pixels: level geometry for the inverse transform (resolution r spans
// [rx0, rx1) x [ry0, ry1) in the tile-component's reference grid of that
// resolution; its plane region is [0, rx1 - rx0) x [0, ry1 - ry0)).
struct TileComp {
  int32_t x0, y0, x1, y1;          // tile-component region (reference grid = image grid)
  int32_t nlevels;                  // decomposition levels
  int32_t rx0[kMaxLevels + 1], ry0[kMaxLevels + 1], rx1[kMaxLevels + 1], ry1[kMaxLevels + 1];
  int64_t off;                      // plane offset in the coefficient buffer (elements)
  int32_t stride;                   // plane row stride (elements)
};

struct Tile {
  int32_t x0, y0, x1, y1;  // tile region in the image grid
  int32_t mct;             // inverse component transform after the wavelet
  TileComp tc[kMaxComps];
};

struct Image {
  int32_t width, height, ncomp;
  int32_t x0, y0;          // image origin on the reference grid (XOsiz, YOsiz)
  int32_t reversible;      // 5/3 integer (coefficients int32) or 9/7 (float)
  std::vector<Tile> tiles;
  int64_t coef_elems;      // elements of the coefficient buffer (all tiles)
};

// Decodes a JP2 / J2K file in memory: header, packet headers and code-blocks
// on the host; `coef` receives the coefficient planes (int32 for reversible
// files, float otherwise; 4 bytes each).  Fails (fail()) on what the
// decoder does not take: precision other than 8 unsigned, subsampled
// components, 2 or 4+ components, code-block styles other than 0, region of
// interest, progression order changes, packed packet headers.
struct T1Job;
// The code-blocks of a file for the device decoder (k_j2k_t1): jobs sorted
// by shape and pass count, their codewords back to back (each followed by
// 0xFF 0xFF, offsets 4-byte aligned, 16 bytes of read-ahead at the end).
struct T1Batch {
  std::vector<T1Job> jobs;
  std::vector<uint8_t> data;
  int maxw = 0, maxh = 0;
};
// With `t1`, the code-blocks are not decoded here: they are appended to *t1
// (coef is then not touched and may be null); the device decodes them into a
// zeroed coefficient buffer (t1_launch) before decode_launch.
bool decode_host(const uint8_t* data, size_t size, const char* name, Image* img,
                 std::vector<uint32_t>* coef, T1Batch* t1 = nullptr);
// Geometry only (width, height, GRAY8 / RGB24).
bool probe(const uint8_t* data, size_t size, const char* name, UphipPnmInfo* info);
// Whether the bytes start a JP2 file or a J2K codestream.
bool is_j2k(const uint8_t* data, size_t size);

// Device half of the decode: the coefficient buffer `dcoef` (device, as
// decode_host filled it) into the image at `dst` (rows `pitch` apart, GRAY8
// or RGB24), on stream st; `tmp` (device, decode_tmp_bytes) holds the lanes'
// lines.  Both buffers are stream-ordered: reusable once st passes.
size_t decode_tmp_bytes(const Image& img);
bool decode_launch(const Image& img, uint32_t* dcoef, uint8_t* dst, int64_t pitch, void* tmp,
                   hipStream_t st);

// The device code-block decoder: one wave (a workgroup of 64) per 64 jobs,
// `nslots` workgroups walking the groups, each with a scratch slot of
// t1_slot_bytes(maxw, maxh) bytes; writes every sample of every job's block
// into dcoef (samples of blocks without passes stay as they are: zero them
// first).
size_t t1_slot_bytes(int maxw, int maxh);
bool t1_launch(const T1Job* djobs, int njobs, const uint8_t* ddata, uint32_t* dcoef, void* dscr,
               int nslots, int maxw, int maxh, hipStream_t st);

// Lossless encode: the device transforms `src` (GRAY8 or RGB24) into the
// coefficient planes (`dcoef`, laid out as decode_host's for the encoder's
// geometry), the host codes them.
bool encode_geometry(int32_t w, int32_t h, int32_t ncomp, Image* img);
// (tmp: coef_elems * 4 bytes of device line buffer)
bool encode_launch(const Image& img, const uint8_t* src, int64_t pitch, uint32_t* dcoef, void* tmp,
                   hipStream_t st);
bool encode_host(const Image& img, const uint32_t* coef, std::vector<uint8_t>* out);
// The device-coded variant: the code-blocks in encode_jobs' order (their
// codewords at data + off[i], len[i] bytes, nb[i] magnitude planes).
struct T1EncJob;
bool encode_jobs(const Image& img, std::vector<T1EncJob>* jobs, size_t* out_bytes);
bool encode_host_coded(const Image& img, const uint32_t* off, const uint32_t* len,
                       const uint8_t* nb, const uint8_t* data, std::vector<uint8_t>* out);
// device code-block encoder: every job's codeword into its output region,
// lengths and plane counts per job (coef: the forward transform's planes)
size_t t1enc_slot_bytes(int maxw, int maxh);
bool t1enc_launch(const T1EncJob* djobs, int njobs, const uint32_t* dcoef, uint8_t* dout,
                  uint32_t* dlen, uint8_t* dnb, void* dscr, int nslots, int maxw, int maxh,
                  hipStream_t st);
// the codewords packed: doff[i] = exclusive prefix sum of dlen (doff[njobs]
// = total; chained: the sums start at doff[0]'s value, the previous
// sub-batch's total), each job's bytes at dpacked + doff[i]; a job past
// `cap` packed bytes sets *derr instead
bool t1enc_pack(const T1EncJob* djobs, int njobs, const uint8_t* dout, const uint32_t* dlen,
                uint32_t* doff, uint8_t* dpacked, uint64_t cap, int32_t* derr, bool chained,
                hipStream_t st);

}  // namespace j2k
}  // namespace uph
