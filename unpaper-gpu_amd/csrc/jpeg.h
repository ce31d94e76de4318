// jpeg.h — the JPEG decode peer: the layout shared by the
// host entropy decoder (jpeg.cpp) and the device kernels (kernels_jpeg.hip).
//
// The reference decodes JPEG pages through FFmpeg on the CPU path
// (file.c:29-128 loadImage; the batch decode queue converts YUV frames to
// RGB24 with swscale, sheet_stages.c:99-122) and through nvImageCodec on the
// GPU path (imageprocess/nvimgcodec.c:679-1007).  Here the sequential part --
// marker parsing and Huffman decoding -- runs on the host, and the data-
// parallel part -- dequantisation, the inverse DCT, chroma upsampling and
// YCbCr->RGB -- runs on the device, straight into a page buffer (a batch's
// input slot in the runner).
//
// What is decoded: baseline and extended-sequential Huffman JPEG, 8-bit, one
// component (-> GRAY8) or three (YCbCr -> RGB24, or RGB when the file says
// so), sampling factors 1 or 2, restart intervals, any number of sequential
// scans.  Progressive, arithmetic-coded, 12-bit, lossless and CMYK files are
// refused with an error.  Pixel arithmetic follows libjpeg's defaults
// (jidctint.c islow IDCT, jdsample.c fancy upsampling, jdcolor.c
// ycc_rgb_convert) -- checked against PIL's libjpeg-turbo; FFmpeg's decoder
// (the reference's) has its own IDCT and swscale conversion: parity with it
// is unpinned.
//
// Packed layout (one contiguous buffer, uploaded as is):
//   JpegHeader | counts (u8 per block, decode order) | group offsets (u32 per
//   group + 1, int16 units into coefs) | coefs (int16, each block's zigzag
//   prefix up to its last non-zero coefficient, pre-multiplied by nothing:
//   the device dequantises)
// A group is one MCU row of one scan (the unit the device prefix-sums).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "unpaper_hip.h"

namespace uph {

constexpr int kJpegMaxScans = 8;

struct JpegComp {
  int32_t h, v;          // sampling factors
  int32_t bw, bh;        // blocks allocated in the component plane (MCU-padded)
  int32_t dw, dh;        // downsampled width/height in samples (libjpeg's downsampled_*)
  int64_t plane_off;     // byte offset of the plane in the device scratch (colour)
  int32_t pitch;         // plane pitch = bw * 8
  uint16_t qzz[64];      // quantisation table in zigzag order
};

struct JpegScan {
  int32_t ncomp;          // components in the scan (1 = non-interleaved)
  int32_t comp[4];        // their indices
  int32_t mcus_x, mcus_y; // MCUs (or, non-interleaved, blocks) across / down
  int32_t blocks_per_mcu;
  int64_t first_block;    // index of the scan's first block in decode order
  int32_t first_group;    // index of the scan's first group (MCU row)
};

struct JpegHeader {
  int32_t width, height;
  int32_t ncomp;          // 1 or 3
  int32_t color;          // 0 gray, 1 YCbCr -> RGB, 2 RGB (no transform)
  int32_t hmax, vmax;
  JpegComp comp[3];
  int32_t nscans;
  JpegScan scan[kJpegMaxScans];
  int64_t nblocks, ngroups;
  int64_t counts_off, groups_off, coefs_off, total_bytes;  // within the packed buffer
  int64_t scratch_bytes;  // device planes needed (colour; 0 for gray)
};

// jpeg_natural_order: zigzag index -> natural (row-major) index
constexpr uint8_t kJpegNatural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ---------------------------------------------------------------------------
// Device entropy decoding (kernels_jpeg_huff.hip).  For a sequential file
// with one scan the host only parses the markers and copies the entropy-coded
// data with the byte stuffing and restart markers removed; the device decodes
// the Huffman codes itself, in parallel over fixed-size subsequences of the
// bit stream that synchronise by iteration (a decoder started at an arbitrary
// bit falls into step with the true code boundaries after a few codes, and
// the iteration carries each subsequence's exact exit state to the next until
// none changes), then writes the packed layout above for the IDCT kernel.
// Progressive and multi-scan files keep the host entropy decoder.
// ---------------------------------------------------------------------------
constexpr int kJdecSubBits = 1024;   // subsequence length (the count / write passes' unit)
constexpr int kJdecMacro = 8;        // subsequences a synchronisation pass decodes in a row
constexpr int kJdecLook = 10;        // lookahead bits of the decode tables (jpeg.cpp kLook)
// entropy-coded bytes the device decoder takes (bit positions are int32)
constexpr size_t kJdecMaxBytes = (size_t)1 << 27;

struct JdecTable {
  uint16_t look[1 << kJdecLook];     // len << 8 | symbol, 0 = a longer code
  int32_t maxcode[18];               // largest code of each length, -1 if none; [17] sentinel
  int32_t valoff[17];                // vals index of code c of length l: c + valoff[l]
  uint8_t vals[256];
};

// The uploaded stream: JdecHeader | segment start bits (int32, nseg + 1) |
// segment subsequence prefix (int32, nseg + 1) | segment macro prefix
// (int32, nseg + 1; a macro = kJdecMacro subsequences of one segment) | data
// (unstuffed, 48 zero bytes of slack).  h describes the frame, its one scan and the offsets of
// the packed layout the device writes (upper bound of 64 coefficients a block).
struct JdecHeader {
  JpegHeader h;
  int32_t restart;        // MCUs per restart interval (0: none)
  int32_t nseg;           // restart segments (>= 1)
  int64_t nsub;           // subsequences
  int64_t nmac;           // macros
  int64_t nbits;          // data bits
  int32_t tdc[4], tac[4]; // table slots of the scan's components
  int32_t bcomp[10];      // scan component of each block of an MCU
  JdecTable dc[4], ac[4];
  int64_t seg_off, segsub_off, segmac_off, data_off, total_bytes;
};

// One image of a batched device decode (kernels read job blockIdx.y).
struct JdecJob {
  const uint8_t* stream;  // device copy of the uploaded stream
  uint8_t* packed;        // packed coefficient layout (JdecHeader::h.total_bytes)
  uint8_t* scratch;       // jdec_scratch_bytes
  int32_t* status;        // non-zero: corrupt data
};

struct JdecStreamHost {
  JdecHeader hd{};
  std::vector<int32_t> seg;     // segment start bits, + the end
  std::vector<int32_t> segsub;  // subsequences before each segment, + the total
  std::vector<int32_t> segmac;  // macros before each segment, + the total
  std::vector<uint8_t> data;
};

// Marker parse + unstuffing for the device decoder.  Returns 1 when the file
// is a one-scan sequential JPEG (out filled), 0 when it needs the host
// entropy decoder (progressive or several scans; no error set), -1 on error.
int jpeg_stream_prepare(const uint8_t* data, size_t size, const char* name, JdecStreamHost* out);
// Writes the uploaded layout (hd.total_bytes bytes).
void jpeg_stream_pack(const JdecStreamHost& s, uint8_t* dst);
// Device scratch of the decode phases for one image (jdec_launch needs
// sizeof(JdecJob) more).
size_t jdec_scratch_bytes(const JdecHeader& hd);
// One image: the stream at `dstream` (device copy of jpeg_stream_pack's
// bytes), its header `hd`, into the packed coefficient layout at `dpacked`
// (hd.h.total_bytes), using `scratch` (jdec_scratch_bytes), on stream st;
// jpeg_launch then turns the packed layout into pixels.
// A corrupt stream (an invalid code, a coefficient past 63, segments or
// blocks that do not add up) sets *dstatus (device int32) non-zero.
bool jdec_launch(const JdecHeader& hd, const uint8_t* dstream, uint8_t* dpacked, uint8_t* scratch,
                 int32_t* dstatus, hipStream_t st);
// Several images in one set of launches: jobs[n] in device memory (statuses
// zeroed by the caller); max_nsub / max_nmac over the images.
bool jdec_launch_batch(const JdecJob* djobs, int n, int64_t max_nsub, int64_t max_nmac,
                       hipStream_t st);

// Host half: a decoded file's coefficients before packing.
struct JpegDecoded {
  JpegHeader h{};
  std::vector<uint8_t> counts;    // per block: length of the zigzag prefix kept
  std::vector<uint32_t> groups;   // per group (MCU row of a scan) + 1: coefficient offset
  std::vector<int16_t> coefs;
};

// Marker parse + Huffman decode of a whole file image (thread-safe; errors
// through fail()).  Sets the packed offsets (h.*_off, h.total_bytes).
bool jpeg_entropy_decode(const uint8_t* data, size_t size, const char* name, JpegDecoded* out);
// Writes the packed layout (h.total_bytes bytes) to dst.
void jpeg_pack(const JpegDecoded& j, uint8_t* dst);
// Device half: the packed image `dpacked` (device memory) into dst (rows dpitch
// apart) on stream st; scratch holds h.scratch_bytes (colour planes).
bool jpeg_launch(const JpegHeader& h, const uint8_t* dpacked, uint8_t* scratch, uint8_t* dst,
                 int64_t dpitch, hipStream_t st);
bool jpeg_read_file(const char* path, std::vector<uint8_t>* buf);
// The frame header alone (geometry, pixel format), no entropy decoding.
bool jpeg_probe_mem(const uint8_t* d, size_t n, const char* name, UphipPnmInfo* info);
// the pixel format a decoded header yields (GRAY8 or RGB24)
inline int jpeg_format(const JpegHeader& h) { return h.ncomp == 1 ? UPHIP_FMT_GRAY8 : UPHIP_FMT_RGB24; }

}  // namespace uph
