// PDF container: a reader for scanned documents (each page one image
// XObject) and a writer of image-per-page documents.
//
// The reference reads and writes PDFs through MuPDF (pdf/pdf_reader.c,
// pdf/pdf_writer.c); MuPDF is not in this image and the hot path never needs
// a rasteriser, so this is a self-contained container codec: the reader
// parses the file structure (classic xref tables, xref streams, object
// streams, incremental updates, a scan of the file when the xref is broken),
// walks the page tree and hands back the raw bytes of a page's largest image
// (pdf_reader.c:290-396) for the device JPEG / JPEG 2000 decoders or the host
// Flate path; the writer embeds encoded pages untouched (DCTDecode /
// JPXDecode, pdf_writer.c:141-193) or Flate-compresses pixels
// (pdf_writer.c:357-433), streaming each page to disk as it arrives.
//
// Not here: rendering of vector / text pages (pdf_reader.c:443-775, MuPDF's
// rasteriser) and decryption (pdf_doc_authenticate).  Pages that need them
// fail loudly.  JBIG2 and CCITT fax pages decode on the host (jbig2.h,
// ccitt.h).
#pragma once

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "ccitt.h"
#include "unpaper_hip.h"

namespace uph {
namespace pdf {

// pdf_reader.h:19-28
enum ImageFormat : int32_t {
  kUnknown = 0,
  kJpeg = 1,
  kJp2 = 2,
  kJbig2 = 3,
  kCcitt = 4,
  kPng = 5,  // Flate with a PNG predictor
  kRaw = 6,
  kFlate = 7,
};

enum class T : uint8_t { Null, Bool, Int, Real, Name, Str, Arr, Dict, Ref, Stream };

struct Obj {
  T t = T::Null;
  int64_t i = 0;   // Bool / Int; Ref: object number
  int32_t gen = 0;
  double r = 0;    // Real
  std::string s;   // Name (no '/') or String bytes
  std::vector<Obj> a;                          // Arr
  std::vector<std::pair<std::string, Obj>> d;  // Dict, Stream's dictionary
  size_t soff = 0, slen = 0;                   // Stream: bytes [soff, soff + slen) of the file
  const Obj* get(const char* key) const;
  bool is_num() const { return t == T::Int || t == T::Real; }
  double num() const { return t == T::Int ? (double)i : t == T::Real ? r : 0.0; }
  bool is_name(const char* n) const { return t == T::Name && s == n; }
};

// A page's image as stored (PdfImage, pdf_reader.h:31-44) plus what the
// pixel path needs from the image dictionary.
struct PageImage {
  std::vector<uint8_t> data, globals;
  int32_t width = 0, height = 0, components = 0, bpc = 0;
  int32_t format = kUnknown;
  bool mask = false;
  bool inverted = false;  // /Decode [1 0] on a one-component image
  bool indexed = false;   // /Indexed colour space: expanded through `palette`
  std::vector<uint8_t> palette;  // (hival + 1) entries of palette_comps bytes
  int32_t palette_comps = 0;     // 1 (gray base) or 3 (RGB base); 0 = not expandable
  int32_t predictor = 1, colors = 1, pbpc = 8, columns = 1;  // Flate /DecodeParms
  ccitt::Params fax;                                          // CCITTFaxDecode /DecodeParms
  int32_t object = 0;  // its object number (diagnostics)
};

struct Meta {
  std::string title, author, subject, keywords, creator, producer, creation_date, modification_date;
  bool has[8] = {};
};

struct PageBox {
  float width = 0, height = 0;  // points, the page bounds after /Rotate (fz_bound_page)
  int32_t rotation = 0;         // the page object's own /Rotate (pdf_reader.c:250-255)
};

class Document {
 public:
  // Takes the file's bytes (open) or a caller buffer that outlives the
  // document (open_view).  `name` appears in error messages.
  bool open(std::vector<uint8_t>&& bytes, const char* name);
  bool open_view(const uint8_t* p, size_t n, const char* name);
  int page_count() const { return (int)pages_.size(); }
  bool encrypted() const { return encrypted_; }
  bool page_box(int page, PageBox* out);
  // The page's largest image XObject; false (with the error set) when the
  // page has none.
  bool extract_image(int page, PageImage* out);
  bool metadata(Meta* out);
  const std::string& name() const { return name_; }

 private:
  struct XEnt {
    uint8_t type = 0;  // 0 free / absent, 1 at offset a, 2 in object stream a at index b
    int64_t a = 0;
    int64_t b = 0;
  };
  const uint8_t* p_ = nullptr;
  size_t n_ = 0;
  std::vector<uint8_t> own_;
  std::string name_;
  std::vector<XEnt> xref_;
  std::vector<bool> seen_;
  Obj trailer_;
  bool encrypted_ = false;
  struct PageRec {
    Obj dict;            // the page dictionary with the inheritable keys filled in
    int32_t own_rotate;  // its own /Rotate
  };
  std::vector<PageRec> pages_;
  std::unordered_map<int64_t, std::unique_ptr<Obj>> cache_;
  std::unordered_map<int64_t, int> loading_;
  bool reconstructed_ = false;
  std::recursive_mutex mu_;

  bool init();
  bool read_xref_chain(int64_t off);
  bool read_xref_table(size_t pos, Obj* trailer);
  bool read_xref_stream(size_t pos, Obj* trailer);
  bool reconstruct();
  bool build_pages();
  void set_entry(int64_t num, uint8_t type, int64_t a, int64_t b);
  bool parse_indirect_at(size_t pos, int64_t expect_num, Obj* out, int depth);
  bool load_objstm(int64_t stm, int depth);
  const Obj* load(int64_t num, int depth);

 public:
  // An object with references followed (nullptr = a dangling reference,
  // which PDF reads as null).
  const Obj* resolve(const Obj* o, int depth = 0);
  // A stream's data with its filters [first, last) applied (all of them by
  // default; `cap` bounds the output).
  bool stream_data(const Obj& stream, std::vector<uint8_t>* out, size_t cap, int depth = 0,
                   int first = 0, int last = -1);
  const uint8_t* bytes() const { return p_; }
  size_t size() const { return n_; }
};

// Filters (also used by the pixel path).  inflate: zlib stream; false on
// corrupt data or when the output would pass `cap`.
bool inflate_bytes(const uint8_t* p, size_t n, std::vector<uint8_t>* out, size_t cap);
bool unpredict(std::vector<uint8_t>* data, int predictor, int colors, int bpc, int columns);

// The pixel format a Flate / raw image maps to (UPHIP_FMT_*), -1 if none.
int pixel_format(const PageImage& im);
// Flate / PNG / raw page images to pixels of pixel_format(im).
bool decode_pixels(const PageImage& im, uint8_t* dst, int64_t linesize, const char* name);

// The page's image and the pixel geometry it decodes to (JPEG / JPEG 2000 by
// their headers, Flate / raw by pixel_format); dpi > 0 applies the
// reference's page-size check (pdf_pipeline_decode.c:69-111).
bool page_geometry(Document& doc, int page, int32_t dpi, PageImage* im, UphipPnmInfo* info);

// The image-per-page writer (PdfWriter, pdf_writer.h).  Pages stream to
// "<path>.part" as they are added, in any order: a page reserves its byte
// range and object numbers under the lock, then writes its objects with one
// positioned write outside it, so store tasks write concurrently.  close()
// waits for those writes, writes the page tree in page-index order, the
// cross-reference table and trailer, and renames the file into place;
// abort() (or destruction without close) removes it.  Thread-safe.
class Writer {
 public:
  ~Writer();
  bool create(const char* path, const Meta* meta, int dpi);
  // kind: kJpeg, kJp2 or kRaw (pixels: components 1 or 3, `stride` apart)
  bool add_page(int64_t index, int kind, const uint8_t* data, size_t len, int width, int height,
                int stride, int components, int dpi);
  bool add_page_next(int kind, const uint8_t* data, size_t len, int width, int height, int stride,
                     int components, int dpi);
  int page_count();
  bool close();
  void abort();

 private:
  std::mutex mu_;
  int fd_ = -1;
  std::string path_, part_;
  int dpi_ = 72;
  int64_t pos_ = 0;                                   // bytes reserved so far
  std::vector<int64_t> offsets_;                      // by object number (0 unused)
  std::vector<std::pair<int64_t, int64_t>> pages_;    // (page index, page object)
  int64_t next_index_ = 0;
  std::atomic<int> inflight_{0};                      // page writes outside the lock
  std::atomic<bool> failed_{false};
  Meta meta_;
  bool has_meta_ = false;
  bool put(const void* p, size_t n);  // at pos_, under the lock
  bool putf(const char* fmt, ...) __attribute__((format(printf, 2, 3)));
  void drain();
};

}  // namespace pdf
}  // namespace uph
