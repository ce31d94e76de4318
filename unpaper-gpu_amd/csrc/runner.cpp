// runner.cpp — multi-device batch scheduler: the MI355X peer of the reference's
// lib/batch_worker.c + lib/threadpool.c + the decode/encode queues
// (lib/decode_queue.c, lib/encode_queue.c) and the pinned per-stream staging of
// src/pipeline/image_pipeline.c:226-376.
//
// Reference: batch_process_parallel (batch_worker.c:273) submits every job to
// a thread pool; each worker binds a CUDA stream from the pool
// (batch_worker.c:197-212) and runs process_sheet on one sheet.  Jobs are
// independent (fresh SheetProcessState per job, sheet_process.c:29-84), so
// pages shard across devices with no collective.
//
// Here: one host thread per device, each owning K batches (= K HIP streams,
// K in-flight launch sequences of S sheets).  Jobs are pulled in chunks of S
// from one shared counter (BatchQueue peer), so a faster device takes more.
// Host-fed runs move every chunk through a slot's pinned staging:
//   load (host pool: source -> pinned in)   [decode queue peer]
//   H2D + pipeline + D2H on the slot stream [DMA engines + CUs]
//   store (host pool: pinned out -> sink)   [encode queue peer]
// with K slots per device in flight, so the host work of one slot overlaps the
// device work of the others.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "j2k.h"
#include "j2k_t1_lane.h"
#include "jpeg.h"
#include "pdf.h"
#include "runtime.h"

using Clock = std::chrono::steady_clock;

namespace uph {
namespace {

double secs(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

// Fixed-size host thread pool with a blocking parallel-for; the calling
// thread works too, so a pool shared by several device threads cannot
// deadlock.
class HostPool {
 public:
  // aff: the CPUs the workers run on (a device's NUMA node), or null
  explicit HostPool(int n, const cpu_set_t* aff = nullptr) {
    if (aff) {
      aff_ = *aff;
      pinned_ = true;
    }
    for (int i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size(); }
  // fire-and-forget task (the caller tracks completion itself)
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  void parallel_for(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    struct Group {
      std::atomic<int> next{0};
      std::atomic<int> left;
      std::mutex mu;
      std::condition_variable cv;
    };
    auto g = std::make_shared<Group>();
    g->left = n;
    auto body = [g, n, &fn] {
      for (;;) {
        const int i = g->next.fetch_add(1);
        if (i >= n) return;
        fn(i);
        if (g->left.fetch_sub(1) == 1) {
          std::lock_guard<std::mutex> lk(g->mu);
          g->cv.notify_all();
        }
      }
    };
    const int helpers = std::min<int>(n - 1, (int)th_.size());
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (int i = 0; i < helpers; i++) q_.push_back(body);
    }
    cv_.notify_all();
    body();
    std::unique_lock<std::mutex> lk(g->mu);
    g->cv.wait(lk, [&] { return g->left.load() == 0; });
    // queued helpers that start after this point find no index left and
    // return without touching `fn`
  }

 private:
  void loop() {
    if (pinned_) pthread_setaffinity_np(pthread_self(), sizeof(aff_), &aff_);
    for (;;) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        t = std::move(q_.front());
        q_.pop_front();
      }
      t();
    }
  }
  std::vector<std::thread> th_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  cpu_set_t aff_;
  bool pinned_ = false;
};

// The CPUs of a device's NUMA node (sysfs via its PCI bus id), within the
// CPUs this process may use.  False when the node is unknown (no NUMA, a
// virtual device) or shares no CPU with the process.
bool device_node_cpus(int device, int* node, cpu_set_t* cpus) {
  *node = -1;
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, device) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  for (char* c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
  char path[256];
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  const bool got = fscanf(f, "%d", node) == 1;
  fclose(f);
  if (!got || *node < 0) return false;
  snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", *node);
  f = fopen(path, "r");
  if (!f) return false;
  char list[4096] = {0};
  const bool read = fgets(list, sizeof(list), f) != nullptr;
  fclose(f);
  if (!read) return false;
  cpu_set_t allowed;
  CPU_ZERO(cpus);
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  for (char* p = list; *p && *p != '\n';) {  // "a-b,c,d-e"
    char* e;
    const long a = strtol(p, &e, 10);
    long b = a;
    if (e == p) break;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; c++)
      if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, cpus);
    p = *e == ',' ? e + 1 : e;
  }
  return CPU_COUNT(cpus) > 0;
}

}  // namespace
}  // namespace uph

using namespace uph;

// ---------------------------------------------------------------------------
// sources and sinks
// ---------------------------------------------------------------------------
// Memory sources and sinks are page-locked (hipHostRegister) on their first
// run, so the runner's DMA copies read and write the caller's buffers
// directly instead of going through pinned staging and a host memcpy each way
// (image_pipeline.c:226-376 stages through pinned buffers because its decode
// produces frames in pageable memory).  Unregistered on destroy.
struct HostRegistration {
  void* ptr = nullptr;
  size_t bytes = 0;
  bool tried = false;
  bool ok = false;
  std::mutex mu;  // a source or sink may be shared by runners on other threads
  // Registers [p, p + n) once; n is the extent the runner reads or writes,
  // not a whole number of strides (the caller's last page need not be padded).
  bool ensure(const void* p, size_t n) {
    std::lock_guard<std::mutex> lk(mu);
    if (tried) return ok;
    tried = true;
    ok = hipHostRegister(const_cast<void*>(p), n, hipHostRegisterDefault) == hipSuccess;
    if (ok) {
      ptr = const_cast<void*>(p);
      bytes = n;
    } else {
      (void)hipGetLastError();  // registration is an optimisation: staged copies otherwise
    }
    return ok;
  }
  ~HostRegistration() {
    if (ok) hipHostUnregister(ptr);
  }
};

struct UphipSource {
  UphipLoadFn load = nullptr;
  void* user = nullptr;
  // built-ins
  const uint8_t* base = nullptr;
  int64_t linesize = 0, page_stride = 0, npages = 0;
  std::vector<std::string> paths;
  // a PDF document: page i of it is input page i (uphip_source_pdf)
  std::shared_ptr<uph::pdf::Document> pdf;
  int32_t pdf_dpi = 0;
  HostRegistration reg;
};

struct UphipSink {
  UphipStoreFn store = nullptr;
  void* user = nullptr;
  uint8_t* base = nullptr;
  int64_t linesize = 0, sheet_stride = 0, nsheets = 0;
  std::string pattern;
  int64_t wrap = 0;
  // JPEG files encoded on the device (uphip_sink_jpeg)
  bool jpeg = false;
  int32_t quality = UPHIP_JPEG_DEFAULT_QUALITY, sampling = UPHIP_JPEG_444;
  // lossless JPEG 2000 files (uphip_sink_jp2): transforms on the device from
  // the batch's output planes, code-blocks on the store tasks
  bool jp2 = false;
  // one PDF of all the output pages (uphip_sink_pdf): the encoded pages go
  // to the writer instead of files
  std::unique_ptr<uph::pdf::Writer> pdfw;
  int32_t pdf_dpi = 300;
  HostRegistration reg;
};

namespace {

int mem_load(const UphipSource* s, int64_t idx, void* dst, int64_t linesize,
             const UphipPnmInfo& geo) {
  if (idx < 0 || idx >= s->npages) return fail("source_memory: page %lld out of range", (long long)idx), -1;
  const int64_t rb = row_bytes(geo.width, geo.format);
  const uint8_t* src = s->base + idx * s->page_stride;
  uint8_t* d = (uint8_t*)dst;
  if (linesize == s->linesize && linesize == rb) {
    memcpy(d, src, (size_t)(rb * geo.height));
  } else {
    for (int32_t y = 0; y < geo.height; y++)
      memcpy(d + (int64_t)y * linesize, src + (int64_t)y * s->linesize, (size_t)rb);
  }
  return 0;
}

int pnm_load(const UphipSource* s, int64_t idx, void* dst, int64_t linesize,
             const UphipPnmInfo& geo) {
  if (idx < 0 || idx >= (int64_t)s->paths.size())
    return fail("source_pnm: page %lld out of range", (long long)idx), -1;
  return uphip_image_read(s->paths[(size_t)idx].c_str(), dst, linesize, &geo);
}

// The reference names output files with sprintf(buf, pattern, outputNr++)
// (image_pipeline.c:742): an int conversion such as "out%04d.pbm".  The
// pattern becomes a format string here, so it may hold at most one integer
// conversion (flags, width and precision kept, any length modifier replaced
// by ll to match the int64_t page number) and "%%"; anything else (%s, %n,
// a second conversion) is refused.
bool output_pattern(const char* p, std::string* out) {
  int nconv = 0;
  out->clear();
  for (const char* c = p; *c; c++) {
    if (*c != '%') {
      out->push_back(*c);
      continue;
    }
    if (c[1] == '%') {
      out->append("%%");
      c++;
      continue;
    }
    std::string spec = "%";
    const char* q = c + 1;
    while (*q && strchr("-+ #0", *q)) spec.push_back(*q++);
    while (*q >= '0' && *q <= '9') spec.push_back(*q++);
    if (*q == '.') {
      spec.push_back(*q++);
      while (*q >= '0' && *q <= '9') spec.push_back(*q++);
    }
    while (*q && strchr("hljzt", *q)) q++;  // length modifiers: replaced below
    if (!*q || !strchr("diuoxX", *q))
      return fail("sink_pnm: pattern \"%s\": only one integer conversion (%%d, %%05d, ...) "
                  "is allowed", p);
    if (++nconv > 1) return fail("sink_pnm: pattern \"%s\" has more than one conversion", p);
    spec.append("ll");
    spec.push_back(*q);
    out->append(spec);
    c = q;
  }
  return true;
}

}  // namespace

extern "C" {

UphipSource* uphip_source_callback(UphipLoadFn load, void* user) {
  if (!load) return fail("source_callback: null function"), nullptr;
  UphipSource* s = new UphipSource();
  s->load = load;
  s->user = user;
  return s;
}

UphipSource* uphip_source_memory(const void* base, int64_t linesize, int64_t page_stride,
                                 int64_t npages) {
  if (!base || npages <= 0) return fail("source_memory: bad arguments"), nullptr;
  UphipSource* s = new UphipSource();
  s->base = (const uint8_t*)base;
  s->linesize = linesize;
  s->page_stride = page_stride;
  s->npages = npages;
  return s;
}

UphipSource* uphip_source_pnm(const char* const* paths, int64_t npaths) {
  if (!paths || npaths <= 0) return fail("source_pnm: no files"), nullptr;
  UphipSource* s = new UphipSource();
  for (int64_t i = 0; i < npaths; i++) s->paths.emplace_back(paths[i] ? paths[i] : "");
  return s;
}

UphipSource* uphip_source_pdf(const char* path, int32_t dpi) {
  if (!path) return fail("source_pdf: null path"), nullptr;
  if (dpi < 0) return fail("source_pdf: dpi %d", dpi), nullptr;
  std::vector<uint8_t> bytes;
  if (!uph::jpeg_read_file(path, &bytes)) return nullptr;
  auto doc = std::make_shared<uph::pdf::Document>();
  if (!doc->open(std::move(bytes), path)) return nullptr;
  if (doc->encrypted()) return fail("source_pdf: %s is encrypted (decryption is not supported)", path), nullptr;
  if (doc->page_count() <= 0) return fail("source_pdf: %s has no pages", path), nullptr;
  UphipSource* s = new UphipSource();
  s->pdf = std::move(doc);
  s->pdf_dpi = dpi;
  return s;
}

int64_t uphip_source_page_count(UphipSource* s) {
  if (!s) return fail("source_page_count: null source"), -1;
  if (s->pdf) return s->pdf->page_count();
  if (s->base) return s->npages;
  if (!s->paths.empty()) return (int64_t)s->paths.size();
  return fail("source_page_count: a callback source has no page count"), -1;
}

void uphip_source_destroy(UphipSource* s) { delete s; }

UphipSink* uphip_sink_callback(UphipStoreFn store, void* user) {
  if (!store) return fail("sink_callback: null function"), nullptr;
  UphipSink* k = new UphipSink();
  k->store = store;
  k->user = user;
  return k;
}

UphipSink* uphip_sink_memory(void* base, int64_t linesize, int64_t sheet_stride, int64_t nsheets) {
  if (!base || nsheets <= 0) return fail("sink_memory: bad arguments"), nullptr;
  UphipSink* k = new UphipSink();
  k->base = (uint8_t*)base;
  k->linesize = linesize;
  k->sheet_stride = sheet_stride;
  k->nsheets = nsheets;
  return k;
}

UphipSink* uphip_sink_pnm(const char* pattern, int64_t wrap) {
  if (!pattern) return fail("sink_pnm: null pattern"), nullptr;
  std::string fmt;
  if (!output_pattern(pattern, &fmt)) return nullptr;
  UphipSink* k = new UphipSink();
  k->pattern = fmt;
  k->wrap = wrap;
  return k;
}

UphipSink* uphip_sink_jpeg(const char* pattern, int64_t wrap, int32_t quality, int32_t sampling) {
  if (!pattern) return fail("sink_jpeg: null pattern"), nullptr;
  if (quality == 0) quality = UPHIP_JPEG_DEFAULT_QUALITY;
  if (quality < 1 || quality > 100) return fail("sink_jpeg: quality %d outside 1..100", quality), nullptr;
  if (sampling < UPHIP_JPEG_444 || sampling > UPHIP_JPEG_420)
    return fail("sink_jpeg: unknown sampling %d", sampling), nullptr;
  std::string fmt;
  if (!output_pattern(pattern, &fmt)) return nullptr;
  UphipSink* k = new UphipSink();
  k->pattern = fmt;
  k->wrap = wrap;
  k->jpeg = true;
  k->quality = quality;
  k->sampling = sampling;
  return k;
}

UphipSink* uphip_sink_jp2(const char* pattern, int64_t wrap) {
  if (!pattern) return fail("sink_jp2: null pattern"), nullptr;
  std::string fmt;
  if (!output_pattern(pattern, &fmt)) return nullptr;
  UphipSink* k = new UphipSink();
  k->pattern = fmt;
  k->wrap = wrap;
  k->jp2 = true;
  return k;
}

UphipSink* uphip_sink_discard(void) { return new UphipSink(); }

UphipSink* uphip_sink_pdf(const char* path, const UphipPdfMetadata* meta, int32_t dpi, int32_t quality,
                          int32_t mode) {
  if (!path) return fail("sink_pdf: null path"), nullptr;
  if (mode != UPHIP_PDF_FAST && mode != UPHIP_PDF_HIGH) return fail("sink_pdf: unknown mode %d", mode), nullptr;
  if (quality == 0) quality = UPHIP_JPEG_DEFAULT_QUALITY;
  if (quality < 1 || quality > 100) return fail("sink_pdf: quality %d outside 1..100", quality), nullptr;
  if (dpi < 0 || dpi > 1200) return fail("sink_pdf: dpi %d outside 0..1200", dpi), nullptr;
  uph::pdf::Meta m;
  if (meta) {
    const char* f[8] = {meta->title,   meta->author,   meta->subject,       meta->keywords,
                        meta->creator, meta->producer, meta->creation_date, meta->modification_date};
    std::string* o[8] = {&m.title,   &m.author,   &m.subject,       &m.keywords,
                         &m.creator, &m.producer, &m.creation_date, &m.modification_date};
    for (int i = 0; i < 8; i++)
      if (f[i]) {
        *o[i] = f[i];
        m.has[i] = true;
      }
  }
  std::unique_ptr<uph::pdf::Writer> w(new uph::pdf::Writer());
  if (!w->create(path, meta ? &m : nullptr, dpi ? dpi : 300)) return nullptr;
  UphipSink* k = new UphipSink();
  k->pdfw = std::move(w);
  k->pdf_dpi = dpi ? dpi : 300;  // PDF_RENDER_DPI (pdf_pipeline_cpu_batch.c:41)
  k->quality = quality;
  k->sampling = UPHIP_JPEG_444;
  if (mode == UPHIP_PDF_HIGH)
    k->jp2 = true;
  else
    k->jpeg = true;
  return k;
}

int uphip_sink_finish(UphipSink* k) {
  if (!k) return fail("sink_finish: null sink"), -1;
  if (!k->pdfw) return 0;
  const bool ok = k->pdfw->close();
  k->pdfw.reset();
  return ok ? 0 : -1;
}

void uphip_sink_destroy(UphipSink* k) { delete k; }

}  // extern "C"

// ---------------------------------------------------------------------------
// runner
// ---------------------------------------------------------------------------
namespace {

// A JPEG page of a chunk: entropy-decoded by a load task into pinned memory
// (jpeg.h packed layout); the device thread uploads it and decodes it on the
// slot's stream straight into the batch's input slot before the run.
struct JpegPage {
  uint8_t* host = nullptr;  // pinned, grown on demand
  size_t cap = 0;
  bool on = false;          // this chunk's page is a JPEG waiting for the device
  bool dev = false;         // Huffman-decoded on the device (host holds a JdecHeader stream)
  size_t bytes = 0;         // bytes to upload
  JpegHeader h{};
  // a JPEG 2000 page instead: host holds its code-block jobs (j2k_t1_lane.h;
  // offsets relative to the page) then their codewords; the device decodes
  // the code-blocks of all the chunk's JPEG 2000 pages in one launch, then
  // runs each page's inverse transforms into its input slot
  bool j2k = false;
  j2k::Image img;
  int32_t njobs = 0;
  size_t jobs_bytes = 0;  // 256-aligned
  int maxw = 0, maxh = 0;
};

struct Slot {
  std::vector<JpegPage> jpg;  // per page of the chunk (sheet * input_count + page)
  uint8_t* djpg = nullptr;    // device copies of the chunk's packed JPEG pages
  size_t djpg_cap = 0;
  j2k::T1Job* hj2j = nullptr; // the chunk's JPEG 2000 jobs, offsets made chunk-wide (pinned)
  size_t hj2j_cap = 0;
  j2k::T1Job* dj2j = nullptr; // their device copy
  size_t dj2j_cap = 0;
  uint32_t* dj2c = nullptr;   // the JPEG 2000 pages' coefficient planes
  size_t dj2c_cap = 0;
  uint8_t* dj2t = nullptr;    // k_j2k_t1 scratch slots
  size_t dj2t_cap = 0;
  uint8_t* dscr = nullptr;    // colour planes (one page at a time on the stream)
  size_t dscr_cap = 0;
  uint8_t* djpk = nullptr;    // packed coefficients of the device-decoded pages
  size_t djpk_cap = 0;
  uint8_t* djsc = nullptr;    // their device Huffman scratch
  size_t djsc_cap = 0;
  int32_t* djst = nullptr;    // per page: device Huffman status
  size_t djst_cap = 0;
  JdecJob* djob = nullptr;    // the decode jobs (device) and their pinned source
  JdecJob* hjob = nullptr;
  size_t djob_cap = 0;
  bool jdev = false;          // the chunk has device-decoded pages (statuses to read)
  UphipBatch* b = nullptr;
  uint8_t* hin = nullptr;   // pinned input staging (count * input_count pages)
  uint8_t* hout = nullptr;  // pinned output staging (count sheets)
  uint8_t* din = nullptr;   // device copy of a registered memory source's chunk
  size_t din_bytes = 0;
  bool direct_out = false;  // this chunk's D2H went straight into the sink
  int64_t first = 0;        // first job of the chunk in flight
  int32_t count = 0;
  int64_t last_first = -1;  // the chunk whose outputs the batch holds (uphip_runner_slot_chunk)
  int32_t last_count = 0;
  std::vector<char> failed;  // per sheet of the chunk
  // JPEG sink: the chunk's packed files (pinned) and each page's size / offset
  uint8_t* hjpg = nullptr;
  size_t hjpg_cap = 0;
  std::vector<int64_t> jsize, joff;
  // JPEG 2000 sink: the chunk's pages coded on the device (jp2_chunk_submit):
  // one device arena (coefficients and code-block outputs of a sub-batch,
  // the coder's slots, jobs, lengths, offsets, planes, packed codewords)
  // and the pinned copies of the offsets / lengths / planes per job
  uint8_t* dj2e = nullptr;
  size_t dj2e_cap = 0;
  uint8_t* hj2e = nullptr;
  size_t hj2e_cap = 0;
  j2k::Image j2img;
  int32_t j2jobs = 0;         // code-blocks a page
  uint32_t* hj2off = nullptr; // pinned views into hj2e (npages * j2jobs + 1, ...)
  uint32_t* hj2len = nullptr;
  uint8_t* hj2nb = nullptr;
  int32_t* hj2err = nullptr;
  const uint8_t* dj2pk = nullptr;  // packed codewords (device)
};

struct DeviceCtx {
  int device = 0;
  std::vector<Slot> slots;
  // placement (image_pipeline.c:226-376 sizes pools per device; here each
  // device also gets its node's CPUs): the device thread and this device's
  // load/store pool run on the CPUs of the GPU's NUMA node; pinned staging
  // comes from hipHostMalloc, which places it on the node nearest the
  // current device
  int numa = -1;
  bool pinned = false;
  cpu_set_t cpus;
  HostPool* pool = nullptr;
  void bind() const {
    if (pinned) pthread_setaffinity_np(pthread_self(), sizeof(cpus), &cpus);
  }
  // per-run results
  int64_t done = 0, failed = 0;
  double busy_s = 0;
  std::string error;
};

}  // namespace

struct UphipRunner {
  UphipOptions opts;
  UphipBatchGeometry geo;  // capacity = sheets per batch
  UphipRunnerConfig cfg;
  std::vector<int> devices;
  std::vector<DeviceCtx> dev;
  int32_t out_w = 0, out_h = 0, out_fmt = 0;
  int64_t in_pitch = 0, in_page_stride = 0;   // batch input slot layout (= staging layout)
  int64_t out_linesize = 0, out_sheet_stride = 0;
  bool staged = false;  // pinned staging allocated
  int64_t batch_bytes = 0;  // device memory of one batch
  UphipRunnerStats stats{};
};

namespace {

void store_sheet(UphipRunner* r, const UphipSink* k, int64_t job, const uint8_t* sheet, bool* ok) {
  const int oc = r->opts.output_count < 1 ? 1 : r->opts.output_count;
  if (k->store) {
    if (k->store(k->user, job, sheet, r->out_linesize, r->out_w, r->out_h, r->out_fmt) != 0) *ok = false;
    return;
  }
  const int64_t rb = row_bytes(r->out_w, r->out_fmt);
  if (k->base) {
    if (job < 0 || job >= k->nsheets) {
      *ok = fail("sink_memory: sheet %lld out of range", (long long)job);
      return;
    }
    uint8_t* d = k->base + job * k->sheet_stride;
    for (int32_t y = 0; y < r->out_h; y++)
      memcpy(d + (int64_t)y * k->linesize, sheet + (int64_t)y * r->out_linesize, (size_t)rb);
    return;
  }
  if (k->pattern.empty()) return;  // discard
  // output pages side by side in the sheet (sheet_stages.c:606-624)
  const int32_t pw = r->out_w / oc;
  const int64_t prb = row_bytes(pw, r->out_fmt);
  std::vector<uint8_t> tmp;
  for (int j = 0; j < oc; j++) {
    int64_t idx = job * oc + j;
    if (k->wrap > 0) idx %= k->wrap;
    char path[4096];
    // the pattern holds at most one ll integer conversion (output_pattern)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wformat-nonliteral"
    snprintf(path, sizeof(path), k->pattern.c_str(), (long long)idx);
#pragma GCC diagnostic pop
    const uint8_t* src = sheet;
    int64_t ls = r->out_linesize;
    const bool mono = r->out_fmt == UPHIP_FMT_MONOWHITE || r->out_fmt == UPHIP_FMT_MONOBLACK;
    if (j > 0 || (oc > 1 && mono && (pw & 7))) {  // a page of its own (fresh padding bits)
      const int64_t x0 = (int64_t)j * pw;
      tmp.assign((size_t)(prb * r->out_h), 0);
      for (int32_t y = 0; y < r->out_h; y++) {
        const uint8_t* row = sheet + (int64_t)y * r->out_linesize;
        uint8_t* t = tmp.data() + (int64_t)y * prb;
        if (mono) {
          for (int32_t x = 0; x < pw; x++) {
            const int64_t sx = x0 + x;
            if (row[sx >> 3] & (0x80 >> (sx & 7))) t[x >> 3] |= (uint8_t)(0x80 >> (x & 7));
          }
        } else {
          const int64_t bpp = row_bytes(1, r->out_fmt);
          memcpy(t, row + x0 * bpp, (size_t)prb);
        }
      }
      src = tmp.data();
      ls = prb;
    }
    if (uphip_pnm_write(path, src, ls, pw, r->out_h, r->out_fmt) != 0) *ok = false;
  }
}

std::string sink_path(const UphipSink* k, int64_t idx) {
  if (k->wrap > 0) idx %= k->wrap;
  char path[4096];
  // the pattern holds at most one ll integer conversion (output_pattern)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wformat-nonliteral"
  snprintf(path, sizeof(path), k->pattern.c_str(), (long long)idx);
#pragma GCC diagnostic pop
  return path;
}

bool write_file(const std::string& path, const uint8_t* p, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return fail("sink_jpeg: cannot create %s", path.c_str());
  const bool ok = fwrite(p, 1, n, f) == n;
  return (fclose(f) == 0 && ok) || fail("sink_jpeg: cannot write %s", path.c_str());
}

// An encoded output page `idx` (job * output_count + page): its file, or its
// page of the sink's PDF (the page accumulator's writes,
// pdf_page_accumulator.c:44-62; here straight from the store task, the
// writer orders the page tree).
bool sink_write(const UphipSink* k, int64_t idx, const uint8_t* p, size_t n) {
  if (!k->pdfw) return write_file(sink_path(k, idx), p, n);
  UphipPnmInfo g{0, 0, 0};
  if (k->jpeg ? !uph::jpeg_probe_mem(p, n, "output page", &g) : !uph::j2k::probe(p, n, "output page", &g))
    return false;
  return k->pdfw->add_page(idx, k->jpeg ? uph::pdf::kJpeg : uph::pdf::kJp2, p, n, g.width, g.height, 0, 0,
                           k->pdf_dpi);
}

// The JPEG pages of sheet s of a slot's chunk into their files: from the
// chunk's packed download, or -- a page the batch's encode buffers could not
// hold -- encoded again on its own, on the device, from the batch's sheet.
void store_jpeg_sheet(UphipRunner* r, const UphipSink* k, int device, UphipBatch* b, int64_t job,
                      int s, const uint8_t* packed, const std::vector<int64_t>& size,
                      const std::vector<int64_t>& off, bool* ok) {
  const int oc = r->opts.output_count < 1 ? 1 : r->opts.output_count;
  for (int j = 0; j < oc; j++) {
    const int i = s * oc + j;
    if (size[(size_t)i] > 0) {
      if (!sink_write(k, job * oc + j, packed + off[(size_t)i], (size_t)size[(size_t)i])) *ok = false;
      continue;
    }
    const void* src = nullptr;
    int64_t pitch = 0;
    int32_t w = 0, h = 0, fmt = 0;
    if (uphip_set_device(device) != 0 ||
        uphip_batch_jpeg_page(b, i, &src, &pitch, &w, &h, &fmt) != 0) {
      *ok = false;
      continue;
    }
    const int64_t n = uphip_jpeg_encode(src, pitch, w, h, fmt, k->quality, k->sampling, nullptr, 0);
    std::vector<uint8_t> file(n > 0 ? (size_t)n : 0);
    if (n <= 0 ||
        uphip_jpeg_encode(src, pitch, w, h, fmt, k->quality, k->sampling, file.data(), n) != n ||
        !sink_write(k, job * oc + j, file.data(), file.size()))
      *ok = false;
  }
}

constexpr int kJ2kSubBatch = 16;  // pages coded per k_j2k_t1enc launch (bounds the arena)

// The chunk's output pages as lossless JPEG 2000 code-blocks, queued on the
// batch's stream once its run has finished: per sub-batch of pages the
// forward transforms of each page, one code-block launch, the packing into
// one buffer (offsets chained across sub-batches); then the offsets, lengths
// and plane counts to pinned memory.  The store tasks copy each page's
// packed bytes and write its packets and file.
bool jp2_chunk_submit(UphipRunner* r, Slot* sl, int npg) {
  if (npg <= 0) return true;
  std::vector<const uint8_t*> src((size_t)npg);
  int64_t pitch = 0;
  int32_t w = 0, h = 0, fmt = 0;
  for (int i = 0; i < npg; i++) {
    const void* p = nullptr;
    if (uphip_batch_jpeg_page(sl->b, i, &p, &pitch, &w, &h, &fmt) != 0) return false;
    src[(size_t)i] = (const uint8_t*)p;
  }
  if (fmt != UPHIP_FMT_GRAY8 && fmt != UPHIP_FMT_RGB24) return fail("sink_jp2: GRAY8 or RGB24 sheets only");
  j2k::Image& img = sl->j2img;
  std::vector<j2k::T1EncJob> page;
  size_t obytes = 0;
  if (!j2k::encode_geometry(w, h, fmt == UPHIP_FMT_GRAY8 ? 1 : 3, &img) ||
      !j2k::encode_jobs(img, &page, &obytes))
    return false;
  const int J = (int)page.size();
  sl->j2jobs = J;
  int maxw = 1, maxh = 1;
  for (const j2k::T1EncJob& j : page) {
    maxw = std::max(maxw, (int)j.w);
    maxh = std::max(maxh, (int)j.h);
  }
  const int P = std::min(npg, kJ2kSubBatch);
  const int nslots = std::min((P * J + 63) / 64, 1024);
  auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
  const size_t cb = al((size_t)P * img.coef_elems * 4), tb = al((size_t)img.coef_elems * 4);
  const size_t ob = al((size_t)P * obytes), sb = al((size_t)nslots * j2k::t1enc_slot_bytes(maxw, maxh));
  const size_t jb = al(sizeof(j2k::T1EncJob) * (size_t)P * J);
  const size_t nj = (size_t)npg * J;
  const size_t lb = al(4 * nj), fb = al(4 * (nj + 1)), nb = al(nj), eb = 256;
  // packed codewords: the pages' raw bytes and a half more (lossless files
  // of 8-bit pages stay below their samples); a chunk past it fails loudly
  const uint64_t pk = (uint64_t)npg * ((uint64_t)img.coef_elems * 3 / 2 + 65536);
  const size_t need = cb + tb + ob + sb + jb + lb + fb + nb + eb + al(pk);
  auto grow = [](uint8_t** p, size_t* cap, size_t n, bool pinned) -> bool {
    if (*cap >= n) return true;
    if (*p) pinned ? hipHostFree(*p) : hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (!(pinned ? UPH_HIP(hipHostMalloc((void**)p, n, hipHostMallocDefault)) : UPH_HIP(hipMalloc((void**)p, n))))
      return false;
    *cap = n;
    return true;
  };
  const size_t hjobs = al(sizeof(j2k::T1EncJob) * (size_t)P * J);
  const size_t hneed = hjobs + 4 * (nj + 1) + 4 * nj + nj + 64;
  if (!grow(&sl->dj2e, &sl->dj2e_cap, need, false) || !grow(&sl->hj2e, &sl->hj2e_cap, hneed, true))
    return false;
  uint8_t* a = sl->dj2e;
  uint32_t* dcoef = (uint32_t*)a;
  void* dtmp = a + cb;
  uint8_t* dout = a + cb + tb;
  void* dscr = a + cb + tb + ob;
  j2k::T1EncJob* djobs = (j2k::T1EncJob*)(a + cb + tb + ob + sb);
  uint32_t* dlen = (uint32_t*)(a + cb + tb + ob + sb + jb);
  uint32_t* doff = (uint32_t*)(a + cb + tb + ob + sb + jb + lb);
  uint8_t* dnb = a + cb + tb + ob + sb + jb + lb + fb;
  int32_t* derr = (int32_t*)(a + cb + tb + ob + sb + jb + lb + fb + nb);
  uint8_t* dpk = a + cb + tb + ob + sb + jb + lb + fb + nb + eb;
  sl->dj2pk = dpk;
  hipStream_t st = (hipStream_t)uphip_batch_stream(sl->b);
  // the jobs of a sub-batch: page p's blocks with its coefficient and output
  // offsets (the same for every sub-batch: staged once)
  j2k::T1EncJob* sub = (j2k::T1EncJob*)sl->hj2e;  // pinned: the copy is asynchronous
  for (int p = 0; p < P; p++)
    for (int i = 0; i < J; i++) {
      j2k::T1EncJob t = page[(size_t)i];
      t.in += (int64_t)p * img.coef_elems;
      t.out += (uint32_t)((size_t)p * obytes);
      sub[(size_t)p * J + i] = t;
    }
  if (!UPH_HIP(hipMemcpyAsync(djobs, sub, sizeof(j2k::T1EncJob) * (size_t)P * J, hipMemcpyHostToDevice, st)) ||
      !UPH_HIP(hipMemsetAsync(doff, 0, 4, st)) || !UPH_HIP(hipMemsetAsync(derr, 0, 4, st)))
    return false;
  for (int p0 = 0; p0 < npg; p0 += P) {
    const int n = std::min(P, npg - p0);
    for (int p = 0; p < n; p++)
      if (!j2k::encode_launch(img, src[(size_t)(p0 + p)], pitch, dcoef + (size_t)p * img.coef_elems, dtmp, st))
        return false;
    const size_t j0 = (size_t)p0 * J;
    if (!j2k::t1enc_launch(djobs, n * J, dcoef, dout, dlen + j0, dnb + j0, dscr, nslots, maxw, maxh, st) ||
        !j2k::t1enc_pack(djobs, n * J, dout, dlen + j0, doff + j0, dpk, pk, derr, true, st))
      return false;
  }
  sl->hj2off = (uint32_t*)(sl->hj2e + hjobs);
  sl->hj2len = sl->hj2off + nj + 1;
  sl->hj2nb = (uint8_t*)(sl->hj2len + nj);
  sl->hj2err = (int32_t*)(((uintptr_t)(sl->hj2nb + nj) + 3) & ~(uintptr_t)3);
  return UPH_HIP(hipMemcpyAsync(sl->hj2off, doff, 4 * (nj + 1), hipMemcpyDeviceToHost, st)) &&
         UPH_HIP(hipMemcpyAsync(sl->hj2len, dlen, 4 * nj, hipMemcpyDeviceToHost, st)) &&
         UPH_HIP(hipMemcpyAsync(sl->hj2nb, dnb, nj, hipMemcpyDeviceToHost, st)) &&
         UPH_HIP(hipMemcpyAsync(sl->hj2err, derr, 4, hipMemcpyDeviceToHost, st));
}

// The pages of sheet s of a slot's chunk as JPEG 2000 files: each page's
// packed codewords from the device, its packets and boxes here.
void store_jp2_chunk_sheet(UphipRunner* r, const UphipSink* k, int device, const Slot* sl,
                           int64_t job, int s, bool* ok) {
  thread_local std::vector<uint8_t> data, file;
  thread_local std::vector<uint32_t> off;
  const int oc = r->opts.output_count < 1 ? 1 : r->opts.output_count;
  if (*sl->hj2err) {
    *ok = fail("sink_jp2: code-blocks larger than the packing buffer");
    return;
  }
  const int J = sl->j2jobs;
  for (int j = 0; j < oc; j++)
    for (int q = 0; q < J; q++)
      if (sl->hj2nb[(size_t)(s * oc + j) * J + q] > 16) {
        *ok = fail("sink_jp2: a code-block's codeword outgrew its region");
        return;
      }
  for (int j = 0; j < oc; j++) {
    const int i = s * oc + j;
    const uint32_t* po = sl->hj2off + (size_t)i * J;
    const uint32_t base = po[0], end = po[J];
    data.resize((size_t)(end - base) + 1);
    off.resize((size_t)J);
    for (int q = 0; q < J; q++) off[(size_t)q] = po[q] - base;
    if (uphip_set_device(device) != 0 ||
        (end > base && !UPH_HIP(hipMemcpy(data.data(), sl->dj2pk + base, end - base, hipMemcpyDeviceToHost))) ||
        !j2k::encode_host_coded(sl->j2img, off.data(), sl->hj2len + (size_t)i * J, sl->hj2nb + (size_t)i * J,
                                data.data(), &file) ||
        !sink_write(k, job * oc + j, file.data(), file.size()))
      *ok = false;
  }
}

bool is_jpeg_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  uint8_t sig[3];
  const bool yes = fread(sig, 1, 3, f) == 3 && sig[0] == 0xFF && sig[1] == 0xD8 && sig[2] == 0xFF;
  fclose(f);
  return yes;
}

// The host half of a JPEG page into the slot's pinned buffer `jp`.
bool jpeg_load_mem(UphipRunner* r, int device, const uint8_t* data, size_t size, const char* name,
                   JpegPage* jp) {
  thread_local JdecStreamHost S;
  // the frame header first: a file of the wrong geometry (or a crafted one
  // claiming a huge frame) is refused before anything is sized from it
  UphipPnmInfo info{0, 0, 0};
  if (!jpeg_probe_mem(data, size, name, &info)) return false;
  if (info.width != r->geo.page_width || info.height != r->geo.page_height ||
      info.format != r->geo.page_format)
    return fail("jpeg: %s is %dx%d format %d, expected %dx%d format %d", name, info.width,
                info.height, info.format, r->geo.page_width, r->geo.page_height,
                r->geo.page_format);
  // a one-scan sequential file goes to the device as its unstuffed entropy
  // data (Huffman decoding there too); progressive / multi-scan files are
  // entropy-decoded here
  const int dev = jpeg_stream_prepare(data, size, name, &S);
  if (dev < 0) return false;
  JpegDecoded d;
  if (!dev && !jpeg_entropy_decode(data, size, name, &d)) return false;
  // pinned memory for this device (the pool thread may have another current)
  if (uphip_set_device(device) != 0) return false;
  const size_t need = (size_t)(dev ? S.hd.total_bytes : d.h.total_bytes);
  if (jp->cap < need) {
    if (jp->host) hipHostFree(jp->host);
    jp->host = nullptr;
    jp->cap = 0;
    if (!UPH_HIP(hipHostMalloc((void**)&jp->host, need + need / 4, hipHostMallocDefault))) return false;
    jp->cap = need + need / 4;
  }
  if (dev)
    jpeg_stream_pack(S, jp->host);
  else
    jpeg_pack(d, jp->host);
  jp->h = dev ? S.hd.h : d.h;
  jp->dev = dev == 1;
  jp->j2k = false;
  jp->bytes = need;
  jp->on = true;
  return true;
}

bool jpeg_load(UphipRunner* r, int device, const std::string& path, JpegPage* jp) {
  // per pool thread, kept across pages: fresh multi-MB buffers per page would
  // page-fault (and contend on the address space) on every load
  thread_local std::vector<uint8_t> file;
  if (!jpeg_read_file(path.c_str(), &file)) return false;
  return jpeg_load_mem(r, device, file.data(), file.size(), path.c_str(), jp);
}

bool is_j2k_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  uint8_t sig[12];
  const size_t n = fread(sig, 1, 12, f);
  fclose(f);
  return j2k::is_j2k(sig, n);
}

// The host half of a JPEG 2000 page (headers, packet headers) into the
// slot's pinned buffer `jp`: its code-block jobs, then their codewords.
bool j2k_load_mem(UphipRunner* r, int device, const uint8_t* data, size_t size, const char* name,
                  JpegPage* jp) {
  thread_local j2k::T1Batch tb;
  UphipPnmInfo info{0, 0, 0};
  if (!j2k::probe(data, size, name, &info)) return false;
  if (info.width != r->geo.page_width || info.height != r->geo.page_height ||
      info.format != r->geo.page_format)
    return fail("jp2: %s is %dx%d format %d, expected %dx%d format %d", name, info.width,
                info.height, info.format, r->geo.page_width, r->geo.page_height,
                r->geo.page_format);
  if (!j2k::decode_host(data, size, name, &jp->img, nullptr, &tb)) return false;
  if (uphip_set_device(device) != 0) return false;
  jp->njobs = (int32_t)tb.jobs.size();
  jp->jobs_bytes = (sizeof(j2k::T1Job) * tb.jobs.size() + 255) & ~(size_t)255;
  jp->maxw = tb.maxw;
  jp->maxh = tb.maxh;
  const size_t need = jp->jobs_bytes + tb.data.size();
  if (jp->cap < need) {
    if (jp->host) hipHostFree(jp->host);
    jp->host = nullptr;
    jp->cap = 0;
    if (!UPH_HIP(hipHostMalloc((void**)&jp->host, need + need / 4, hipHostMallocDefault))) return false;
    jp->cap = need + need / 4;
  }
  memcpy(jp->host, tb.jobs.data(), sizeof(j2k::T1Job) * tb.jobs.size());
  memcpy(jp->host + jp->jobs_bytes, tb.data.data(), tb.data.size());
  jp->h = JpegHeader{};
  jp->h.scratch_bytes = (int64_t)j2k::decode_tmp_bytes(jp->img);  // the line buffer
  jp->j2k = true;
  jp->dev = false;
  jp->bytes = need;
  jp->on = true;
  return true;
}

bool j2k_load(UphipRunner* r, int device, const std::string& path, JpegPage* jp) {
  thread_local std::vector<uint8_t> file;
  if (!jpeg_read_file(path.c_str(), &file)) return false;
  return j2k_load_mem(r, device, file.data(), file.size(), path.c_str(), jp);
}

// Page `idx` of a PDF source (the decode queue of the PDF pipeline,
// pdf_pipeline_cpu_batch.c:381-496): its image's JPEG / JPEG 2000 bytes to
// the device decode like a file's, Flate / raw pixels decoded here.
bool pdf_load(UphipRunner* r, int device, const UphipSource* s, int64_t idx, uint8_t* dst, JpegPage* jp) {
  if (idx < 0 || idx >= s->pdf->page_count())
    return fail("source_pdf: page %lld out of range (%d pages)", (long long)idx, s->pdf->page_count());
  thread_local pdf::PageImage im;
  UphipPnmInfo g{0, 0, 0};
  if (!pdf::page_geometry(*s->pdf, (int)idx, s->pdf_dpi, &im, &g)) return false;
  char name[64];
  snprintf(name, sizeof(name), "pdf page %lld", (long long)idx);
  if (im.format == pdf::kJpeg) return jpeg_load_mem(r, device, im.data.data(), im.data.size(), name, jp);
  if (im.format == pdf::kJp2) return j2k_load_mem(r, device, im.data.data(), im.data.size(), name, jp);
  if (g.width != r->geo.page_width || g.height != r->geo.page_height || g.format != r->geo.page_format)
    return fail("pdf: %s is %dx%d format %d, expected %dx%d format %d", name, g.width, g.height, g.format,
                r->geo.page_width, r->geo.page_height, r->geo.page_format);
  return pdf::decode_pixels(im, dst, r->in_pitch, name);
}

bool load_page(UphipRunner* r, int device, const UphipSource* s, int64_t job, int32_t j,
               uint8_t* dst, JpegPage* jp) {
  const UphipPnmInfo geo{r->geo.page_width, r->geo.page_height, r->geo.page_format};
  const int64_t idx = job * r->opts.input_count + j;
  if (s->load) return s->load(s->user, job, j, dst, r->in_pitch) == 0;
  if (s->base) return mem_load(s, idx, dst, r->in_pitch, geo) == 0;
  if (s->pdf) return pdf_load(r, device, s, idx, dst, jp);
  if (idx >= 0 && idx < (int64_t)s->paths.size()) {
    const std::string& path = s->paths[(size_t)idx];
    if (is_jpeg_file(path)) return jpeg_load(r, device, path, jp);
    if (is_j2k_file(path)) return j2k_load(r, device, path, jp);
  }
  return pnm_load(s, idx, dst, r->in_pitch, geo) == 0;
}

// Queue the H2D copy of the slot's staged pages, skipping the JPEG pages (their
// decode writes the batch's input slots itself, after this copy): runs of
// other pages go as one copy each (the staging is laid out like the slots).
bool upload_staging(UphipRunner* r, Slot* sl, int npages) {
  bool any = false;
  for (int p = 0; p < npages; p++) any |= sl->jpg[(size_t)p].on;
  if (!any)
    return uphip_batch_upload_async(sl->b, sl->count, sl->hin, r->in_pitch, r->in_page_stride) == 0;
  hipStream_t st = (hipStream_t)uphip_batch_stream(sl->b);
  for (int p = 0; p < npages;) {
    if (sl->jpg[(size_t)p].on) {
      p++;
      continue;
    }
    int e = p;
    while (e < npages && !sl->jpg[(size_t)e].on) e++;
    int64_t pitch = 0;
    uint8_t* dst = (uint8_t*)uphip_batch_input_ptr(sl->b, p, &pitch);
    if (!dst || pitch != r->in_pitch ||
        !UPH_HIP(hipMemcpyAsync(dst, sl->hin + (int64_t)p * r->in_page_stride,
                                (size_t)((int64_t)(e - p) * r->in_page_stride),
                                hipMemcpyHostToDevice, st)))
      return false;
    p = e;
  }
  return true;
}

// Queue the chunk's JPEG and JPEG 2000 pages on the slot's stream: upload each
// packed page (JPEG 2000: its coefficient planes), then decode it into its
// input slot (after the staging upload, before the run).
size_t up256(size_t n) { return (n + 255) & ~(size_t)255; }

bool jpeg_submit(Slot* sl, int npages) {
  size_t total = 0, scr = 0, pk = 0, hs = 0;
  int ndev = 0;
  int64_t max_nsub = 0, max_nmac = 0;
  sl->jdev = false;
  for (int p = 0; p < npages; p++) {
    const JpegPage& jp = sl->jpg[(size_t)p];
    if (!jp.on) continue;
    total += up256(jp.bytes);  // page starts aligned (JPEG 2000 planes are int32)
    scr = std::max(scr, (size_t)jp.h.scratch_bytes);
    if (jp.dev) {
      const JdecHeader& hd = *(const JdecHeader*)jp.host;
      ndev++;
      pk += ((size_t)jp.h.total_bytes + 255) & ~(size_t)255;
      hs += (jdec_scratch_bytes(hd) + 255) & ~(size_t)255;
      max_nsub = std::max<int64_t>(max_nsub, hd.nsub);
      max_nmac = std::max<int64_t>(max_nmac, hd.nmac);
    }
  }
  if (!total) return true;
  // the slot's stream is idle here (the slot was free): old buffers can go
  auto grow = [](auto** p, size_t* cap, size_t need) -> bool {
    if (*cap >= need) return true;
    if (*p) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (!UPH_HIP(hipMalloc((void**)p, need + need / 4))) return false;
    *cap = need + need / 4;
    return true;
  };
  if (!grow(&sl->djpg, &sl->djpg_cap, total) || (scr && !grow(&sl->dscr, &sl->dscr_cap, scr)))
    return false;
  hipStream_t st = (hipStream_t)uphip_batch_stream(sl->b);
  if (ndev) {
    sl->jdev = true;
    if (!grow(&sl->djpk, &sl->djpk_cap, pk) || !grow(&sl->djsc, &sl->djsc_cap, hs) ||
        !grow(&sl->djst, &sl->djst_cap, 4 * (size_t)npages))
      return false;
    if (sl->djob_cap < (size_t)npages) {
      if (sl->djob) hipFree(sl->djob);
      if (sl->hjob) hipHostFree(sl->hjob);
      sl->djob = nullptr;
      sl->hjob = nullptr;
      sl->djob_cap = 0;
      if (!UPH_HIP(hipMalloc((void**)&sl->djob, sizeof(JdecJob) * (size_t)npages)) ||
          !UPH_HIP(hipHostMalloc((void**)&sl->hjob, sizeof(JdecJob) * (size_t)npages,
                                 hipHostMallocDefault)))
        return false;
      sl->djob_cap = (size_t)npages;
    }
    if (!UPH_HIP(hipMemsetAsync(sl->djst, 0, 4 * (size_t)npages, st))) return false;
  }
  // upload every page; the device-decoded ones as one batch of jobs
  size_t off = 0, poff = 0, soff = 0;
  int nj = 0;
  std::vector<int> jpage;
  for (int p = 0; p < npages; p++) {
    JpegPage& jp = sl->jpg[(size_t)p];
    if (!jp.on) continue;
    if (!UPH_HIP(hipMemcpyAsync(sl->djpg + off, jp.host, jp.bytes, hipMemcpyHostToDevice, st)))
      return false;
    if (jp.dev) {
      const JdecHeader& hd = *(const JdecHeader*)jp.host;
      sl->hjob[nj] = JdecJob{sl->djpg + off, sl->djpk + poff, sl->djsc + soff, sl->djst + p};
      jpage.push_back(p);
      nj++;
      poff += ((size_t)jp.h.total_bytes + 255) & ~(size_t)255;
      soff += (jdec_scratch_bytes(hd) + 255) & ~(size_t)255;
    }
    off += up256(jp.bytes);
  }
  if (nj) {
    if (!UPH_HIP(hipMemcpyAsync(sl->djob, sl->hjob, sizeof(JdecJob) * (size_t)nj,
                                hipMemcpyHostToDevice, st)) ||
        !jdec_launch_batch(sl->djob, nj, max_nsub, max_nmac, st))
      return false;
  }
  // JPEG 2000 pages: every code-block of the chunk in one launch (offsets
  // made chunk-wide), into one coefficient buffer
  {
    int64_t nj = 0, coefs = 0;
    int maxw = 0, maxh = 0;
    for (int p = 0; p < npages; p++) {
      const JpegPage& jp = sl->jpg[(size_t)p];
      if (!jp.on || !jp.j2k) continue;
      nj += jp.njobs;
      coefs += jp.img.coef_elems;
      maxw = std::max(maxw, jp.maxw);
      maxh = std::max(maxh, jp.maxh);
    }
    if (coefs > 0) {
      const int nslots = (int)std::min<int64_t>((nj + 63) / 64, 1024);
      if (!grow(&sl->dj2c, &sl->dj2c_cap, (size_t)coefs * 4) ||
          !grow(&sl->dj2t, &sl->dj2t_cap, (size_t)std::max(nslots, 1) * j2k::t1_slot_bytes(maxw, maxh)) ||
          !grow(&sl->dj2j, &sl->dj2j_cap, sizeof(j2k::T1Job) * (size_t)std::max<int64_t>(nj, 1)))
        return false;
      if (sl->hj2j_cap < (size_t)nj) {
        if (sl->hj2j) hipHostFree(sl->hj2j);
        sl->hj2j = nullptr;
        sl->hj2j_cap = 0;
        if (!UPH_HIP(hipHostMalloc((void**)&sl->hj2j, sizeof(j2k::T1Job) * (size_t)nj + 256,
                                   hipHostMallocDefault)))
          return false;
        sl->hj2j_cap = (size_t)nj;
      }
      size_t o = 0;
      int64_t q = 0, cb = 0;
      for (int p = 0; p < npages; p++) {
        const JpegPage& jp = sl->jpg[(size_t)p];
        if (!jp.on) continue;
        if (jp.j2k) {
          const j2k::T1Job* pj = reinterpret_cast<const j2k::T1Job*>(jp.host);
          for (int i = 0; i < jp.njobs; i++) {
            j2k::T1Job t = pj[i];
            t.data += (uint32_t)(o + jp.jobs_bytes);
            t.out += cb;
            sl->hj2j[q++] = t;
          }
          cb += jp.img.coef_elems;
        }
        o += up256(jp.bytes);
      }
      if (o > 0xFFFFFFF0u) return fail("jp2: chunk too large for 32-bit codeword offsets");
      if (!UPH_HIP(hipMemcpyAsync(sl->dj2j, sl->hj2j, sizeof(j2k::T1Job) * (size_t)nj,
                                  hipMemcpyHostToDevice, st)) ||
          !UPH_HIP(hipMemsetAsync(sl->dj2c, 0, (size_t)coefs * 4, st)) ||
          !j2k::t1_launch(sl->dj2j, (int)nj, sl->djpg, sl->dj2c, sl->dj2t, nslots, maxw, maxh, st))
        return false;
    }
  }
  // pixels: each page from its packed coefficients into its input slot
  off = 0;
  int k = 0;
  int64_t cb = 0;
  for (int p = 0; p < npages; p++) {
    JpegPage& jp = sl->jpg[(size_t)p];
    if (!jp.on) continue;
    int64_t pitch = 0;
    uint8_t* dst = (uint8_t*)uphip_batch_input_ptr(sl->b, p, &pitch);
    if (jp.j2k) {
      if (!dst || !j2k::decode_launch(jp.img, sl->dj2c + cb, dst, pitch, sl->dscr, st)) return false;
      cb += jp.img.coef_elems;
      off += up256(jp.bytes);
      continue;
    }
    const uint8_t* packed = jp.dev ? sl->hjob[k++].packed : sl->djpg + off;
    if (!dst || !jpeg_launch(jp.h, packed, sl->dscr, dst, pitch, st)) return false;
    off += up256(jp.bytes);
  }
  return true;
}

// per-sheet device status after a finished run: a failing wait names the
// sheets through their reports
void collect_failures(Slot& sl) {
  sl.failed.assign((size_t)sl.count, 0);
  if (uphip_batch_wait(sl.b) == 0) return;
  uphip_clear_error();
  for (int s = 0; s < sl.count; s++) {
    UphipSheetReport rep;
    if (uphip_batch_get_report(sl.b, s, &rep) != 0 || rep.flags) sl.failed[(size_t)s] = 1;
  }
}

// Sheets per batch when the caller leaves it to the runner: the sheet's
// input pages plus its two working planes (GRAY8 for gray inputs, RGB24
// otherwise, as the batch plans them) within 2 GiB, at most 64 (the batch
// size the A4 measurements use) and at least 1.
int32_t auto_capacity(const UphipOptions& o, const UphipBatchGeometry& g) {
  const int64_t w = g.page_width, h = g.page_height;
  const int n_in = o.input_count > 0 ? o.input_count : 1;
  const bool gray = g.page_format == UPHIP_FMT_GRAY8 || g.page_format == UPHIP_FMT_MONOWHITE ||
                    g.page_format == UPHIP_FMT_MONOBLACK;
  const int64_t in = round_pitch(row_bytes((int32_t)w, g.page_format)) * h * n_in;
  const int64_t plane = (gray ? 1 : 3) * w * n_in * h;
  const int64_t per_sheet = std::max<int64_t>(in + 2 * plane, 1);
  return (int32_t)std::max<int64_t>(1, std::min<int64_t>(64, (2ll << 30) / per_sheet));
}

}  // namespace

extern "C" {

UphipRunner* uphip_runner_create(const UphipOptions* options, const UphipBatchGeometry* geometry,
                                 const UphipRunnerConfig* config) {
  if (!options || !geometry || !config) return fail("runner_create: null argument"), nullptr;
  if (!runtime_ready()) return fail("runner_create: no HIP device"), nullptr;
  const int ndev_all = uphip_device_count();
  if (config->ndevices <= 0 || geometry->page_width <= 0 || geometry->page_height <= 0)
    return fail("runner_create: invalid configuration"), nullptr;
  UphipRunner* r = new UphipRunner();
  r->opts = *options;
  r->geo = *geometry;
  r->cfg = *config;
  if (r->geo.capacity <= 0) r->geo.capacity = auto_capacity(*options, *geometry);
  for (int i = 0; i < config->ndevices; i++) {
    const int d = config->devices ? config->devices[i] : i;
    if (d < 0 || d >= ndev_all) {
      delete r;
      return fail("runner_create: device %d out of range (%d devices)", d, ndev_all), nullptr;
    }
    r->devices.push_back(d);
  }
  const int caller_dev = uphip_get_device();
  r->dev.resize(r->devices.size());
  bool ok = true;
  for (size_t i = 0; ok && i < r->devices.size(); i++) {
    DeviceCtx& dc = r->dev[i];
    dc.device = r->devices[i];
    if (uphip_set_device(dc.device) != 0) {
      ok = false;
      break;
    }
    // the first batch measures the footprint the auto layout divides by
    if (i == 0) {
      UphipBatch* b = uphip_batch_create(options, &r->geo);
      if (!b) {
        ok = false;
        break;
      }
      int64_t bb = 0;
      uphip_batch_device_bytes(b, &bb);
      r->batch_bytes = bb;
      if (config->batches_per_device <= 0) {
        // per slot: the batch, plus the dense input chunk a direct memory
        // source is copied into (allocated at the first host run)
        int64_t ip = 0;
        uphip_batch_input_ptr(b, 0, &ip);
        const int64_t din = ip * r->geo.page_height * r->geo.capacity *
                            (options->input_count > 0 ? options->input_count : 1);
        size_t fr = 0, tot = 0;
        int n = 1;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && bb > 0)
          n = 1 + (int)std::min<int64_t>((int64_t)(fr / 2) / (bb + din), 15);
        r->cfg.batches_per_device = n;
      }
      dc.slots.resize((size_t)r->cfg.batches_per_device);
      dc.slots[0].b = b;
    } else {
      dc.slots.resize((size_t)r->cfg.batches_per_device);
    }
    for (Slot& sl : dc.slots) {
      if (!sl.b) sl.b = uphip_batch_create(options, &r->geo);
      if (!sl.b) {
        ok = false;
        break;
      }
      if (config->timing) uphip_batch_set_timing(sl.b, 1);
    }
  }
  uphip_set_device(caller_dev);
  if (!ok) {
    uphip_runner_destroy(r);
    return nullptr;
  }
  UphipBatch* b0 = r->dev[0].slots[0].b;
  int64_t bytes = 0;
  uphip_batch_output_info(b0, &r->out_w, &r->out_h, &r->out_fmt, &bytes);
  uphip_batch_input_ptr(b0, 0, &r->in_pitch);
  r->in_page_stride = r->in_pitch * r->geo.page_height;
  // output staging laid out like the batch's output rows, so a batch's
  // sheets come back as linear DMA copies
  {
    int64_t op = 0;
    UphipBatch* bb = r->dev[0].slots[0].b;
    r->out_linesize = round_pitch(row_bytes(r->out_w, r->out_fmt));
    if (uphip_batch_output_pitch(bb, &op) == 0 && op >= row_bytes(r->out_w, r->out_fmt))
      r->out_linesize = op;
  }
  r->out_sheet_stride = r->out_linesize * r->out_h;
  // load/store pools: one per device, its share of the host threads, on the
  // device's NUMA node (the decode/encode queues' workers, lib/decode_queue.c)
  const int nd = (int)r->devices.size();
  const int ht = config->host_threads > 0 ? config->host_threads : 4 * nd;
  for (int i = 0; i < nd; i++) {
    DeviceCtx& dc = r->dev[(size_t)i];
    dc.pinned = device_node_cpus(dc.device, &dc.numa, &dc.cpus);
    const int share = std::max(1, ht / nd + (i < ht % nd ? 1 : 0));
    dc.pool = new HostPool(share, dc.pinned ? &dc.cpus : nullptr);
  }
  return r;
}

void uphip_runner_destroy(UphipRunner* r) {
  if (!r) return;
  for (DeviceCtx& dc : r->dev) {
    delete dc.pool;
    dc.pool = nullptr;
  }
  for (DeviceCtx& dc : r->dev) {
    uphip_set_device(dc.device);
    for (Slot& sl : dc.slots) {
      if (sl.b) uphip_batch_destroy(sl.b);
      if (sl.hin) hipHostFree(sl.hin);
      if (sl.hout) hipHostFree(sl.hout);
      if (sl.din) hipFree(sl.din);
      if (sl.djpg) hipFree(sl.djpg);
      if (sl.dscr) hipFree(sl.dscr);
      if (sl.djpk) hipFree(sl.djpk);
      if (sl.djsc) hipFree(sl.djsc);
      if (sl.djst) hipFree(sl.djst);
      if (sl.djob) hipFree(sl.djob);
      if (sl.hjob) hipHostFree(sl.hjob);
      if (sl.hjpg) hipHostFree(sl.hjpg);
      if (sl.hj2j) hipHostFree(sl.hj2j);
      if (sl.dj2j) hipFree(sl.dj2j);
      if (sl.dj2c) hipFree(sl.dj2c);
      if (sl.dj2t) hipFree(sl.dj2t);
      if (sl.dj2e) hipFree(sl.dj2e);
      if (sl.hj2e) hipHostFree(sl.hj2e);
      for (JpegPage& jp : sl.jpg)
        if (jp.host) hipHostFree(jp.host);
    }
  }
  delete r;
}

int uphip_runner_layout(UphipRunner* r, int32_t* batches_per_device, int32_t* capacity,
                        int64_t* batch_bytes) {
  if (!r) return fail("runner_layout: null runner"), -1;
  if (batches_per_device) *batches_per_device = r->cfg.batches_per_device;
  if (capacity) *capacity = r->geo.capacity;
  if (batch_bytes) *batch_bytes = r->batch_bytes;
  return 0;
}

int uphip_runner_placement(UphipRunner* r, int32_t device_index, int32_t* numa_node,
                           int32_t* ncpus, int32_t* pool_threads) {
  if (!r || device_index < 0 || device_index >= (int)r->dev.size())
    return fail("runner_placement: bad device index"), -1;
  const DeviceCtx& dc = r->dev[(size_t)device_index];
  if (numa_node) *numa_node = dc.pinned ? dc.numa : -1;
  if (ncpus) *ncpus = dc.pinned ? CPU_COUNT(&dc.cpus) : 0;
  if (pool_threads) *pool_threads = dc.pool ? dc.pool->size() : 0;
  return 0;
}

int64_t uphip_runner_slot_chunk(UphipRunner* r, int32_t device_index, int32_t slot,
                                int32_t* count) {
  if (!r || device_index < 0 || device_index >= (int)r->dev.size() || slot < 0 ||
      slot >= (int)r->dev[(size_t)device_index].slots.size())
    return fail("runner_slot_chunk: bad arguments"), -1;
  const Slot& sl = r->dev[(size_t)device_index].slots[(size_t)slot];
  if (count) *count = sl.last_first >= 0 ? sl.last_count : 0;
  return sl.last_first;
}

UphipBatch* uphip_runner_batch(UphipRunner* r, int32_t device_index, int32_t slot) {
  if (!r || device_index < 0 || device_index >= (int)r->dev.size() || slot < 0 ||
      slot >= (int)r->dev[(size_t)device_index].slots.size())
    return nullptr;
  return r->dev[(size_t)device_index].slots[(size_t)slot].b;
}

int uphip_runner_run_device(UphipRunner* r, const UphipDevicePages* shards, int32_t passes) {
  if (!r || !shards || passes < 1) return fail("runner_run_device: bad arguments"), -1;
  const auto t0 = Clock::now();
  const int S = r->geo.capacity;
  std::vector<std::thread> th;
  for (size_t i = 0; i < r->dev.size(); i++) {
    th.emplace_back([r, i, S, shards, passes] {
      DeviceCtx& dc = r->dev[i];
      dc.done = dc.failed = 0;
      dc.error.clear();
      const auto a = Clock::now();
      dc.bind();
      uphip_set_device(dc.device);
      const UphipDevicePages& sh = shards[i];
      const int64_t nin = r->opts.input_count;
      const size_t ns = dc.slots.size();
      std::vector<int32_t> used(ns, 0);
      // Each chunk goes to a slot whose stream is idle (the first batches to
      // the slots in order, then to whichever finishes first), so a slow
      // chunk -- a sheet whose blackfilter replay runs long -- delays only its
      // own slot: a fixed chunk -> slot mapping would queue every later chunk
      // of that slot, pass after pass, behind it.
      size_t next_fresh = 0;
      auto idle_slot = [&]() -> size_t {
        if (next_fresh < ns) return next_fresh++;
        for (;;) {
          for (size_t s = 0; s < ns; s++)
            if (uphip_batch_query(dc.slots[s].b) != 0) return s;  // idle, or failed (run reports)
          std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
      };
      for (int32_t pass = 0; pass < passes; pass++)
      for (int64_t first = 0; first < sh.count; first += S) {
        const int32_t n = (int32_t)std::min<int64_t>(S, sh.count - first);
        const size_t k = idle_slot();
        Slot& sl = dc.slots[k];
        if (uphip_batch_run_device(sl.b, n, (const uint8_t*)sh.pages + first * nin * sh.page_stride,
                                   sh.pitch, sh.page_stride) != 0) {
          if (dc.error.empty()) dc.error = uphip_last_error() ? uphip_last_error() : "run failed";
          uphip_clear_error();
          dc.failed += n;
          continue;
        }
        used[k] = n;
        sl.last_first = first;
        sl.last_count = n;
        dc.done += n;
      }
      for (size_t s = 0; s < dc.slots.size(); s++) {
        if (!used[s]) continue;
        if (uphip_batch_wait(dc.slots[s].b) != 0) {
          if (dc.error.empty()) dc.error = uphip_last_error() ? uphip_last_error() : "wait failed";
          uphip_clear_error();
          dc.failed += 1;  // at least one sheet; the sticky status does not say how many
        }
      }
      dc.busy_s = secs(a, Clock::now());
    });
  }
  for (auto& t : th) t.join();
  memset(&r->stats, 0, sizeof(r->stats));
  int64_t failed = 0;
  std::string err;
  for (DeviceCtx& dc : r->dev) {
    r->stats.jobs_done += dc.done;
    r->stats.jobs_failed += dc.failed;
    failed += dc.failed;
    if (err.empty() && !dc.error.empty()) err = dc.error;
  }
  for (size_t i = 0; i < r->dev.size() && i < UPHIP_RUNNER_MAX_DEVICES; i++)
    r->stats.jobs_per_device[i] = r->dev[i].done;
  r->stats.wall_s = secs(t0, Clock::now());
  if (!err.empty()) fail("runner: %s", err.c_str());
  return (int)std::min<int64_t>(failed, 1 << 30);
}

int uphip_runner_run_host(UphipRunner* r, int64_t njobs, UphipSource* src, UphipSink* sink) {
  if (!r || !src || !sink || njobs < 0) return fail("runner_run_host: bad arguments"), -1;
  const int S = r->geo.capacity;
  const int nin = r->opts.input_count;
  if (!r->staged) {  // pinned staging per slot, laid out like the batch's input slots
    // each device's staging from a thread on its node (hipHostMalloc places
    // pinned memory on the node nearest the current device; the thread's
    // binding makes any first-touch local too)
    std::atomic<bool> ok{true};
    {
      std::vector<std::thread> th;
      for (DeviceCtx& dc : r->dev)
        th.emplace_back([&, pdc = &dc] {
          pdc->bind();
          uphip_set_device(pdc->device);
          for (Slot& sl : pdc->slots) {
            if (!UPH_HIP(hipHostMalloc((void**)&sl.hin, (size_t)(r->in_page_stride * S * nin),
                                       hipHostMallocDefault)) ||
                !UPH_HIP(hipHostMalloc((void**)&sl.hout, (size_t)(r->out_sheet_stride * S),
                                       hipHostMallocDefault)))
              ok = false;
          }
          if (!ok) uphip_clear_error();  // reported below from this thread
        });
      for (auto& t : th) t.join();
    }
    if (!ok) fail("runner: pinned staging allocation failed");
    if (!ok) {  // all or nothing: a later call allocates afresh
      for (DeviceCtx& dc : r->dev)
        for (Slot& sl : dc.slots) {
          if (sl.hin) hipHostFree(sl.hin);
          if (sl.hout) hipHostFree(sl.hout);
          sl.hin = sl.hout = nullptr;
        }
    }
    if (!ok) return -1;
    r->staged = true;
  }
  // Direct paths: a memory source whose pages all exist is copied H2D from
  // the caller's (registered) buffer into a dense device chunk that the batch
  // reads in place (uphip_batch_run_device takes any pitch); a memory sink
  // laid out like the batch's output rows receives the D2H copy itself.
  const int oc = r->opts.output_count < 1 ? 1 : r->opts.output_count;
  // The direct source needs pages the batch can read in place: rows at least
  // a row long and pages that do not overlap (page_stride 0, a repeated page,
  // or overlapping pages take the staged path, which copies page by page).
  const int64_t in_row = row_bytes(r->geo.page_width, r->geo.page_format);
  const int64_t in_extent = (int64_t)(r->geo.page_height - 1) * src->linesize + in_row;
  const bool dsrc = src->base && !src->load && src->npages >= njobs * nin && njobs > 0 &&
                    src->linesize >= in_row && src->page_stride >= in_extent &&
                    src->reg.ensure(src->base, (size_t)((src->npages - 1) * src->page_stride + in_extent));
  const int64_t out_extent =
      (int64_t)(r->out_h - 1) * r->out_linesize + row_bytes(r->out_w, r->out_fmt);
  const bool dsnk = sink->base && !sink->store && oc == 1 && sink->nsheets >= njobs && njobs > 0 &&
                    sink->linesize == r->out_linesize && sink->sheet_stride == r->out_sheet_stride &&
                    sink->reg.ensure(sink->base,
                                     (size_t)((sink->nsheets - 1) * sink->sheet_stride + out_extent));
  if (dsrc) {
    const size_t need = (size_t)(src->page_stride * S * nin);
    const int caller_dev = uphip_get_device();
    bool ok = true;
    for (DeviceCtx& dc : r->dev) {
      uphip_set_device(dc.device);
      for (Slot& sl : dc.slots) {
        if (sl.din && sl.din_bytes >= need) continue;
        if (sl.din) hipFree(sl.din);
        sl.din = nullptr;
        sl.din_bytes = 0;
        if (!UPH_HIP(hipMalloc((void**)&sl.din, need))) {
          sl.din = nullptr;
          ok = false;
        } else {
          sl.din_bytes = need;
        }
      }
    }
    uphip_set_device(caller_dev);
    if (!ok) return -1;
  }
  const auto t0 = Clock::now();
  std::atomic<int64_t> next{0};
  std::atomic<int64_t> load_ns{0}, store_ns{0};
  std::vector<std::thread> th;
  // A slot moves FREE -> LOADING (page tasks on the host pool) -> LOADED
  // (last task) -> RUNNING (H2D + pipeline queued on its stream) -> DRAINING
  // (status read, D2H queued) -> STORING (sheet tasks on the pool) -> FREE
  // (last task).  The device thread only moves slots along and never does
  // host copies itself, so decode, DMA, kernels and encode of different
  // slots overlap.
  enum : int { FREE = 0, LOADING, LOADED, RUNNING, DRAINING, STORING };
  for (size_t i = 0; i < r->dev.size(); i++) {
    th.emplace_back([&, i] {
      DeviceCtx& dc = r->dev[i];
      dc.done = dc.failed = 0;
      dc.error.clear();
      dc.bind();
      uphip_set_device(dc.device);
      auto note = [&dc](const char* what) {
        if (dc.error.empty()) dc.error = uphip_last_error() ? uphip_last_error() : what;
        uphip_clear_error();
      };
      const int K = (int)dc.slots.size();
      std::unique_ptr<std::atomic<int>[]> state(new std::atomic<int>[K]);
      std::unique_ptr<std::atomic<int>[]> pend(new std::atomic<int>[K]);
      std::vector<int> phase(K, FREE);  // the device thread's view
      for (int k = 0; k < K; k++) {
        state[k] = FREE;
        pend[k] = 0;
      }
      std::deque<int> inflight;  // RUNNING / DRAINING slots in submission order
      bool jobs_left = true;
      for (;;) {
        bool progress = false;
        for (int k = 0; k < K; k++) {
          Slot* sl = &dc.slots[(size_t)k];
          const int st = state[k].load();
          if (st == FREE && phase[k] == STORING) {  // stored: account the chunk
            for (int s = 0; s < sl->count; s++) {
              if (sl->failed[(size_t)s]) {
                dc.failed++;
                if ((sl->failed[(size_t)s] & 2) && dc.error.empty()) dc.error = "a sheet could not be stored";
                if ((sl->failed[(size_t)s] & 4) && dc.error.empty()) dc.error = "a page could not be loaded";
              } else {
                dc.done++;
              }
            }
            phase[k] = FREE;
            progress = true;
          }
          if (st == FREE && phase[k] == FREE && jobs_left) {
            const int64_t first = next.fetch_add(S);
            if (first >= njobs) {
              jobs_left = false;
              continue;
            }
            sl->first = first;
            sl->jdev = false;
            sl->count = (int32_t)std::min<int64_t>(S, njobs - first);
            sl->failed.assign((size_t)sl->count, 0);
            sl->last_first = first;
            sl->last_count = sl->count;
            if (dsrc) {  // one DMA copy from the caller's pages, then the run
              const size_t bytes = (size_t)((sl->count * nin - 1) * src->page_stride + in_extent);
              hipStream_t bst = (hipStream_t)uphip_batch_stream(sl->b);
              if (!UPH_HIP(hipMemcpyAsync(sl->din, src->base + first * nin * src->page_stride, bytes,
                                          hipMemcpyHostToDevice, bst)) ||
                  uphip_batch_run_device(sl->b, sl->count, sl->din, src->linesize,
                                         src->page_stride) != 0 ||
                  (sink->jpeg &&
                   uphip_batch_encode_jpeg_async(sl->b, sink->quality, sink->sampling) != 0)) {
                note("run failed");
                for (int s = 0; s < sl->count; s++) sl->failed[(size_t)s] |= 1;
                phase[k] = STORING;
                state[k] = FREE;
              } else {
                phase[k] = RUNNING;
                state[k] = RUNNING;
                inflight.push_back(k);
              }
              progress = true;
              continue;
            }
            if (sl->jpg.size() < (size_t)(sl->count * nin)) sl->jpg.resize((size_t)(sl->count * nin));
            for (JpegPage& jp : sl->jpg) jp.on = false;
            pend[k] = sl->count;
            state[k] = LOADING;
            phase[k] = LOADING;
            for (int s = 0; s < sl->count; s++) {
              dc.pool->submit([&, sl, k, s, first] {
                const auto a = Clock::now();
                for (int j = 0; j < nin; j++) {
                  uint8_t* dst = sl->hin + ((int64_t)s * nin + j) * r->in_page_stride;
                  if (!load_page(r, dc.device, src, first + s, j, dst, &sl->jpg[(size_t)(s * nin + j)])) {
                    sl->failed[(size_t)s] |= 4;
                    uphip_clear_error();
                    // the slot still runs: a blank (white) page, cheap and
                    // deterministic, instead of stale staging bytes
                    memset(dst, r->geo.page_format == UPHIP_FMT_MONOWHITE ? 0x00 : 0xFF,
                           (size_t)r->in_page_stride);
                  }
                }
                load_ns += (int64_t)(secs(a, Clock::now()) * 1e9);
                if (pend[k].fetch_sub(1) == 1) state[k] = LOADED;
              });
            }
            progress = true;
          }
          if (st == LOADED && phase[k] == LOADING) {
            if (!upload_staging(r, sl, sl->count * nin) || !jpeg_submit(sl, sl->count * nin) ||
                uphip_batch_run(sl->b, sl->count) != 0 ||
                (sink->jpeg &&
                 uphip_batch_encode_jpeg_async(sl->b, sink->quality, sink->sampling) != 0)) {
              note("run failed");
              for (int s = 0; s < sl->count; s++) sl->failed[(size_t)s] |= 1;
              phase[k] = STORING;  // accounted (all failed) on the next pass
              state[k] = FREE;
            } else {
              phase[k] = RUNNING;
              state[k] = RUNNING;
              inflight.push_back(k);
            }
            progress = true;
          }
        }
        // the oldest slots on the GPU: a finished run -> its D2H; a finished
        // D2H -> the sink, in submission order
        for (size_t q = 0; q < inflight.size();) {
          const int k = inflight[q];
          Slot* sl = &dc.slots[(size_t)k];
          if (uphip_batch_query(sl->b) != 1) break;
          if (phase[k] == RUNNING) {
            std::vector<char> pre = sl->failed;
            collect_failures(*sl);  // the stream is idle: a status read only
            for (size_t s = 0; s < pre.size(); s++) sl->failed[s] |= pre[s];
            if (sl->jdev) {  // pages whose entropy-coded data the device found corrupt
              std::vector<int32_t> jst((size_t)(sl->count * nin), 0);
              if (!UPH_HIP(hipMemcpy(jst.data(), sl->djst, 4 * jst.size(), hipMemcpyDeviceToHost)))
                jst.assign(jst.size(), 1);
              for (size_t q = 0; q < jst.size(); q++)
                if (jst[q]) {
                  sl->failed[q / (size_t)nin] |= 4;
                  if (dc.error.empty()) dc.error = "corrupt JPEG entropy-coded data (device decode)";
                }
            }
            // straight into a memory sink unless a sheet failed (its slot in
            // the sink stays untouched, as with the store tasks)
            bool clean = true;
            for (int s = 0; s < sl->count; s++) clean &= !sl->failed[(size_t)s];
            sl->direct_out = dsnk && clean;
            uint8_t* dst = sl->direct_out ? sink->base + sl->first * sink->sheet_stride : sl->hout;
            bool queued;
            if (sink->jpeg) {
              // only the encoded files come back: sizes (already on the
              // host), then one copy of the packed files
              const int npg = sl->count * oc;
              sl->jsize.assign((size_t)npg, -1);
              sl->joff.assign((size_t)npg, 0);
              const int64_t total = uphip_batch_jpeg_sizes(sl->b, sl->jsize.data(), npg);
              int64_t o = 0;
              for (int i = 0; i < npg; i++) {
                sl->joff[(size_t)i] = o;
                if (sl->jsize[(size_t)i] > 0) o += sl->jsize[(size_t)i];
              }
              queued = total >= 0;
              if (queued && sl->hjpg_cap < (size_t)total) {
                if (sl->hjpg) hipHostFree(sl->hjpg);
                sl->hjpg = nullptr;
                sl->hjpg_cap = 0;
                const size_t cap = (size_t)total + (size_t)total / 2 + 4096;
                queued = UPH_HIP(hipHostMalloc((void**)&sl->hjpg, cap, hipHostMallocDefault));
                if (queued) sl->hjpg_cap = cap;
              }
              queued = queued && uphip_batch_jpeg_download_async(sl->b, sl->hjpg, (int64_t)sl->hjpg_cap) == 0;
            } else if (sink->jp2) {
              // the chunk's pages coded on the device; the store tasks write
              queued = jp2_chunk_submit(r, sl, sl->count * oc);
            } else {
              queued = uphip_batch_download_async(sl->b, dst, r->out_linesize, r->out_sheet_stride) == 0;
            }
            if (!queued) {
              note("download failed");
              for (int s = 0; s < sl->count; s++) sl->failed[(size_t)s] |= 1;
              inflight.erase(inflight.begin() + (long)q);
              phase[k] = STORING;
              state[k] = FREE;
              progress = true;
              continue;
            }
            phase[k] = DRAINING;
            state[k] = DRAINING;
            progress = true;
            q++;
            continue;
          }
          // DRAINING and the copy is done
          inflight.erase(inflight.begin() + (long)q);
          int nstore = 0;
          for (int s = 0; s < sl->count; s++) nstore += !sl->failed[(size_t)s];
          phase[k] = STORING;
          if (sl->direct_out) {  // the copy went straight into the sink
            state[k] = FREE;
          } else if (nstore == 0) {
            state[k] = FREE;
          } else {
            pend[k] = nstore;
            state[k] = STORING;
            for (int s = 0; s < sl->count; s++) {
              if (sl->failed[(size_t)s]) continue;
              dc.pool->submit([&, sl, k, s] {
                const auto a = Clock::now();
                bool good = true;
                if (sink->jpeg)
                  store_jpeg_sheet(r, sink, dc.device, sl->b, sl->first + s, s, sl->hjpg, sl->jsize,
                                   sl->joff, &good);
                else if (sink->jp2)
                  store_jp2_chunk_sheet(r, sink, dc.device, sl, sl->first + s, s, &good);
                else
                  store_sheet(r, sink, sl->first + s, sl->hout + (int64_t)s * r->out_sheet_stride, &good);
                if (!good) {
                  sl->failed[(size_t)s] |= 2;
                  uphip_clear_error();
                }
                store_ns += (int64_t)(secs(a, Clock::now()) * 1e9);
                if (pend[k].fetch_sub(1) == 1) state[k] = FREE;
              });
            }
          }
          progress = true;
        }
        bool idle = !jobs_left;
        for (int k = 0; k < K && idle; k++) idle = state[k].load() == FREE && phase[k] == FREE;
        if (idle) break;
        if (!progress) std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    });
  }
  for (auto& t : th) t.join();
  memset(&r->stats, 0, sizeof(r->stats));
  int64_t failed = 0;
  std::string err;
  for (size_t i = 0; i < r->dev.size(); i++) {
    DeviceCtx& dc = r->dev[i];
    r->stats.jobs_done += dc.done;
    r->stats.jobs_failed += dc.failed;
    if (i < UPHIP_RUNNER_MAX_DEVICES) r->stats.jobs_per_device[i] = dc.done;
    failed += dc.failed;
    if (err.empty() && !dc.error.empty()) err = dc.error;
  }
  r->stats.load_s = load_ns.load() * 1e-9;
  r->stats.store_s = store_ns.load() * 1e-9;
  r->stats.wall_s = secs(t0, Clock::now());
  if (!err.empty()) fail("runner: %s", err.c_str());
  return (int)std::min<int64_t>(failed, 1 << 30);
}

int uphip_runner_get_stats(UphipRunner* r, UphipRunnerStats* out) {
  if (!r || !out) return -1;
  *out = r->stats;
  return 0;
}

int uphip_runner_output_info(UphipRunner* r, int32_t* width, int32_t* height, int32_t* format,
                             int64_t* linesize) {
  if (!r) return -1;
  if (width) *width = r->out_w;
  if (height) *height = r->out_h;
  if (format) *format = r->out_fmt;
  if (linesize) *linesize = r->out_linesize;
  return 0;
}

}  // extern "C"
