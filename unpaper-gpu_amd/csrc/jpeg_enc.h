// jpeg_enc.h — the JPEG encode peer (the GPU output branch):
// layout shared by the host half (jpeg_enc.cpp: tables, file header, batch
// and single-image entry points) and the device kernels (kernels_jpeg_enc.hip).
//
// The reference hands a finished device sheet to nvImageCodec instead of
// copying it back (src/core/sheet_stages.c:554-581 -> encode_queue_submit_gpu,
// lib/encode_queue.c:860-990 -> nvimgcodec_encode, imageprocess/nvimgcodec.c:
// 1007-1212; quality from --jpeg-quality, default 85).  Here the whole encode
// runs on the device, on the batch's stream right after its pipeline, and
// only the finished file images cross PCIe:
//
//   A  k_jenc_count  per tile of 256 MCUs (8 rounds of 32 MCUs, 8 lanes per
//                    MCU): colour conversion + downsampling (jccolor.c,
//                    jcsample.c), islow forward DCT (jfdctint.c) with a
//                    uniform-block shortcut, quantisation by reciprocal
//                    (jcdctmgr.c), Huffman code lengths (jchuff.c): the
//                    tile's bit count and its first / last DC per component
//   B  k_jenc_scan   per image: tile bit offsets (+ the DC differences that
//                    cross tiles), overflow check against the bit buffer
//   C  k_jenc_emit   per tile again (DCT recomputed: cheaper than storing
//                    2 B per coefficient): each lane ORs its codes into an
//                    LDS window of the bit stream at its exact offset; whole
//                    words go to HBM, a tile's first and last (shared) words
//                    to an edge record
//   D  k_jenc_fix    per tile: the shared words assembled from the edge
//                    records, the 0xFF bytes of the tile counted
//   E  k_jenc_layout per image: stuffed byte offsets of the tiles, file size;
//      k_jenc_pack   image offsets in the packed output (one small launch)
//   F  k_jenc_write  per tile: bytes with 0x00 stuffed after 0xFF, the file
//                    header (tile 0) and EOI (last tile)
//
// Output equals libjpeg-turbo's (PIL) byte for byte: baseline, standard
// Annex K tables scaled by jpeg_set_quality, JFIF 1.01 header, 1 component
// for GRAY8 sheets, YCbCr 4:4:4 (nvImageCodec's default) / 4:2:2 / 4:2:0 for
// RGB24 ones.  Parity with nvImageCodec's own encoder is unpinned.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "unpaper_hip.h"

namespace uph {

constexpr int kJencRoundMcus = 32;                          // 8 lanes per MCU, 256 threads
constexpr int kJencTileRounds = 8;
constexpr int kJencTileMcus = kJencRoundMcus * kJencTileRounds;
constexpr int kJencWinWords = 2048;                         // LDS bit window (8 KiB)

enum JencMode : int32_t { JENC_GRAY = 0, JENC_444 = 1, JENC_422 = 2, JENC_420 = 3 };

struct JencTables {
  uint16_t recip[2][64];  // jcdctmgr.c compute_reciprocal (16-bit DCTELEM), natural order
  uint16_t corr[2][64];
  uint8_t shift[2][64];
  uint32_t dc[2][16];     // len << 16 | code, by DC category (jchuff.c ehufco/ehufsi)
  uint32_t ac[2][256];    // len << 16 | code, by run/size symbol
};

struct JencGeom {
  int32_t w, h;
  int32_t mode;           // JencMode
  int32_t ncomp, bpm;     // components, blocks per MCU
  int32_t mcux, mcuy;     // MCUs across / down
  int32_t wb[3], hb[3];   // width_in_blocks / height_in_blocks per component
  int32_t ch[3];          // component heights in samples (downsampled_height)
  int32_t tiles;          // tiles of kJencTileMcus MCUs per image
  int32_t header_bytes;   // file header (SOI .. SOS) length
  int64_t cap_words;      // bit buffer words per image
  int64_t out_cap;        // packed output bytes (all images)
};

struct JencImage {
  const uint8_t* src;     // top-left pixel (GRAY8 or RGB24 rows)
  int64_t pitch;
};

// Device buffers of one encode of `n` images of one geometry.
struct JencBuffers {
  JencImage* images;      // [n]
  uint32_t* tile_bits;    // [n][tiles]   bits of the tile except the DCs that cross tiles
  int16_t* tile_dc;       // [n][tiles][2][3] first / last quantised DC per component
  uint64_t* tile_off;     // [n][tiles + 1] bit offsets (last = image total)
  uint32_t* edges;        // [n][tiles][2] the tile's first / last (shared) words
  uint32_t* tile_ff;      // [n][tiles]   0xFF bytes among the tile's bytes
  uint64_t* tile_out;     // [n][tiles]   stuffed byte offset of the tile in the image
  int64_t* sizes;         // [n] file size; -1 bit buffer overflow, -2 output overflow
  int64_t* offs;          // [n] file offset in `out`
  uint32_t* bits;         // [n][cap_words] bit streams
  uint8_t* out;           // packed files
  const uint8_t* header;  // [header_bytes]
  const JencTables* tables;
};

// The device buffers of one encoder (a batch's, or a thread's for
// uphip_jpeg_encode), grown on demand and reused; setup() waits for the
// stream only when buffers grow or the tables change.
struct JencContext {
  int device = -1;
  JencGeom g{};
  int quality = -1, n = 0;
  JencTables* tables = nullptr;
  uint8_t* header = nullptr;
  uint8_t* meta = nullptr;
  uint32_t* bits = nullptr;
  uint8_t* out = nullptr;
  size_t meta_cap = 0, bits_cap = 0, out_cap = 0;
  int64_t* host_sizes = nullptr;  // pinned: sizes[n] then offsets[n] of the last encode
  int sizes_cap = 0;
  JencBuffers B{};
  ~JencContext();
  void release();
  // geometry, tables and buffers for nimg images; B.images is left to the caller
  bool setup(int32_t w, int32_t h, int32_t fmt, int32_t sampling, int32_t quality, int nimg,
             int64_t cap_words, int64_t out_bytes, hipStream_t st);
  // queues the encode and the copy of sizes / offsets into host_sizes
  bool encode_async(hipStream_t st);
};

// Queues passes A-F for n images on stream st.
bool jenc_launch(const JencGeom& g, const JencBuffers& b, int n, hipStream_t st);

// Host half (jpeg_enc.cpp).
bool jenc_geometry(int32_t w, int32_t h, int32_t fmt, int32_t sampling, JencGeom* g);
void jenc_tables(int32_t quality, JencTables* t);
// The file header libjpeg writes for these parameters; returns its length.
int jenc_header(const JencGeom& g, int32_t quality, uint8_t* out, int cap);
// Device bytes of the per-tile arrays for n images.
size_t jenc_meta_bytes(const JencGeom& g, int n);
// Carves the per-tile arrays out of `meta` (jenc_meta_bytes).
void jenc_carve(const JencGeom& g, int n, uint8_t* meta, JencBuffers* b);

}  // namespace uph
