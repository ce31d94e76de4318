// runtime.hip — device discovery, TLS device/stream, stream pool, errors,
// argument staging ring, scratch buffers, frame allocation.
//
// Peer of imageprocess/cuda_runtime.c (dlopen'ed driver API, TLS stream at
// :70), cuda_stream_pool.c and cuda_mempool.c in the reference.  Differences:
// the current DEVICE is thread-local too (multi-GPU per process), and frames
// are allocated with a 256-byte pitch so every row is cache-line aligned.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "runtime.h"

namespace uph {

namespace {

std::once_flag g_init_once;
UphipInitStatus g_init_status = UPHIP_INIT_ERROR;
int g_device_count = 0;
bool g_fatal = false;

thread_local int t_device = 0;
thread_local bool t_device_set = false;
thread_local hipStream_t t_stream = nullptr;  // user-provided (set_current_stream)
thread_local std::string t_error;
thread_local bool t_has_error = false;

struct PerThreadDevice {
  hipStream_t stream = nullptr;
  // argument ring
  static constexpr int kSlots = 16;
  static constexpr size_t kSlotBytes = 64 * 1024;
  void* host = nullptr;
  void* dev = nullptr;
  hipEvent_t ev[kSlots] = {};
  bool ev_live[kSlots] = {};
  int next = 0;
  int pending[kSlots] = {};
  int npending = 0;
};

// Op-level scratch belongs to a STREAM, not to a thread: a worker that
// switches streams per job (lib/batch_worker.c:197-202) must not hand the
// next job's kernels a buffer the previous job's kernels, still queued on
// another stream, are reading.  Everything on one stream is ordered, so
// per-stream buffers need no further fencing.  As with the reference's TLS
// stream, one stream is current on one thread at a time (two threads issuing
// ops on one stream would share its scratch); resizes hold the entry's lock.
// uphip_stream_forget frees a caller-owned stream's entry before the caller
// destroys the stream (a recycled handle then starts empty).
struct StreamScratch {
  std::mutex mu;
  void* scr[8] = {};
  size_t scr_bytes[8] = {};
};
std::mutex g_scr_mu;
std::map<std::pair<int, hipStream_t>, StreamScratch*> g_scr;

thread_local PerThreadDevice* t_dev[64] = {};

// global stream pool per device
std::mutex g_pool_mu;
std::vector<std::vector<hipStream_t>> g_pool_free;

PerThreadDevice& ptd() {
  int d = current_device();
  if (!t_dev[d]) t_dev[d] = new PerThreadDevice();
  return *t_dev[d];
}

}  // namespace

bool fail(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (!t_has_error) {  // keep the first error until cleared
    t_error = buf;
    t_has_error = true;
  }
  if (g_fatal) {
    fprintf(stderr, "unpaper-hip: %s\n", buf);
    exit(1);
  }
  return false;
}

bool check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  return fail("%s failed: %s", what, hipGetErrorString(e));
}

static void do_init() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    g_init_status = (e == hipErrorNoDevice) ? UPHIP_INIT_NO_DEVICE : UPHIP_INIT_NO_RUNTIME;
    g_device_count = 0;
    return;
  }
  g_device_count = n;
  g_init_status = n > 0 ? UPHIP_INIT_OK : UPHIP_INIT_NO_DEVICE;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool_free.assign(n, {});
}

bool runtime_ready() {
  std::call_once(g_init_once, do_init);
  return g_init_status == UPHIP_INIT_OK;
}

int current_device() {
  if (!t_device_set) {
    t_device = 0;
    t_device_set = true;
  }
  return t_device;
}

hipStream_t current_stream() {
  if (t_stream) return t_stream;
  PerThreadDevice& p = ptd();
  if (!p.stream) {
    hipSetDevice(current_device());
    UPH_HIP(hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
  }
  return p.stream;
}

ArgBlock arg_alloc(size_t bytes) {
  PerThreadDevice& p = ptd();
  if (bytes > PerThreadDevice::kSlotBytes) {
    fail("argument block too large (%zu bytes)", bytes);
    return ArgBlock{nullptr, nullptr};
  }
  hipSetDevice(current_device());
  if (!p.host) {
    if (!UPH_HIP(hipHostMalloc(&p.host, PerThreadDevice::kSlots * PerThreadDevice::kSlotBytes,
                               hipHostMallocDefault)))
      return ArgBlock{nullptr, nullptr};
    if (!UPH_HIP(hipMalloc(&p.dev, PerThreadDevice::kSlots * PerThreadDevice::kSlotBytes)))
      return ArgBlock{nullptr, nullptr};
    for (int i = 0; i < PerThreadDevice::kSlots; i++)
      UPH_HIP(hipEventCreateWithFlags(&p.ev[i], hipEventDisableTiming));
  }
  const int i = p.next;
  p.next = (p.next + 1) % PerThreadDevice::kSlots;
  if (p.npending >= PerThreadDevice::kSlots - 1) {
    fail("too many argument blocks without a fence");
    return ArgBlock{nullptr, nullptr};
  }
  if (p.ev_live[i]) {
    UPH_HIP(hipEventSynchronize(p.ev[i]));  // slot reuse: its readers are done
    p.ev_live[i] = false;
  }
  const size_t off = (size_t)i * PerThreadDevice::kSlotBytes;
  return ArgBlock{(char*)p.host + off, (char*)p.dev + off};
}

bool arg_commit(const ArgBlock& b, size_t bytes, hipStream_t st) {
  PerThreadDevice& p = ptd();
  const size_t off = (char*)b.host - (char*)p.host;
  const int i = (int)(off / PerThreadDevice::kSlotBytes);
  if (!UPH_HIP(hipMemcpyAsync(b.dev, b.host, bytes, hipMemcpyHostToDevice, st))) return false;
  p.pending[p.npending++ % PerThreadDevice::kSlots] = i;
  return true;
}

void arg_fence(hipStream_t st) {
  // recorded after the kernels that read the slots: reuse waits for them
  PerThreadDevice& p = ptd();
  for (int k = 0; k < p.npending && k < PerThreadDevice::kSlots; k++) {
    const int i = p.pending[k];
    UPH_HIP(hipEventRecord(p.ev[i], st));
    p.ev_live[i] = true;
  }
  p.npending = 0;
}

void* scratch(int slot, size_t bytes) {
  if (slot < 0 || slot >= 8) return nullptr;
  const int dev = current_device();
  hipStream_t st = current_stream();
  StreamScratch* ps;
  {
    std::lock_guard<std::mutex> lk(g_scr_mu);
    StreamScratch*& e = g_scr[{dev, st}];
    if (!e) e = new StreamScratch();
    ps = e;
  }
  StreamScratch& p = *ps;
  std::lock_guard<std::mutex> lk(p.mu);
  if (p.scr_bytes[slot] < bytes) {
    hipSetDevice(dev);
    if (p.scr[slot]) {
      hipStreamSynchronize(st);  // the stream's earlier kernels are the only readers
      hipFree(p.scr[slot]);
    }
    size_t n = bytes < 4096 ? 4096 : bytes;
    if (!UPH_HIP(hipMalloc(&p.scr[slot], n))) {
      p.scr[slot] = nullptr;
      p.scr_bytes[slot] = 0;
      return nullptr;
    }
    p.scr_bytes[slot] = n;
  }
  return p.scr[slot];
}

UphipFrame* frame_alloc(int32_t w, int32_t h, int32_t fmt) {
  if (!runtime_ready()) {
    fail("HIP runtime not available: %s", uphip_init_status_string(uphip_try_init()));
    return nullptr;
  }
  if (w <= 0 || h <= 0 || fmt < UPHIP_FMT_GRAY8 || fmt > UPHIP_FMT_MONOBLACK) {
    fail("invalid frame geometry %dx%d fmt %d", w, h, fmt);
    return nullptr;
  }
  UphipFrame* f = new UphipFrame();
  f->width = w;
  f->height = h;
  f->format = fmt;
  f->device = current_device();
  f->pitch = round_pitch(row_bytes(w, fmt));
  hipSetDevice(f->device);
  if (!UPH_HIP(hipMalloc(&f->data, (size_t)f->pitch * h))) {
    delete f;
    return nullptr;
  }
  // deterministic padding / fresh content (av_frame_get_buffer zeroes too)
  UPH_HIP(hipMemsetAsync(f->data, 0, (size_t)f->pitch * h, current_stream()));
  return f;
}

void frame_free(UphipFrame* f) {
  if (!f) return;
  hipSetDevice(f->device);
  hipStreamSynchronize(current_stream());
  hipFree(f->data);
  delete f;
}

Planes frame_planes(const UphipFrame* f) {
  Planes P;
  P.base[0] = f->data;
  P.base[1] = f->data;
  P.pitch = f->pitch;
  P.stride = 0;
  P.W = f->width;
  P.H = f->height;
  P.fmt = f->format;
  P.count = 1;
  return P;
}

}  // namespace uph

using namespace uph;

extern "C" {

UphipInitStatus uphip_try_init(void) {
  std::call_once(g_init_once, do_init);
  return g_init_status;
}

const char* uphip_init_status_string(UphipInitStatus st) {
  switch (st) {
    case UPHIP_INIT_OK: return "ok";
    case UPHIP_INIT_NO_RUNTIME: return "HIP runtime unavailable";
    case UPHIP_INIT_NO_DEVICE: return "no HIP device";
    default: return "HIP initialisation error";
  }
}

int uphip_device_count(void) {
  uphip_try_init();
  return g_device_count;
}

int uphip_set_device(int device) {
  if (!runtime_ready()) return fail("no HIP device"), -1;
  if (device < 0 || device >= g_device_count || device >= 64)
    return fail("device %d out of range (%d devices)", device, g_device_count), -1;
  t_device = device;
  t_device_set = true;
  t_stream = nullptr;
  return UPH_HIP(hipSetDevice(device)) ? 0 : -1;
}

int uphip_get_device(void) { return current_device(); }

void* uphip_stream_acquire(void) {
  if (!runtime_ready()) return nullptr;
  int d = current_device();
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool_free[d].empty()) {
      hipStream_t s = g_pool_free[d].back();
      g_pool_free[d].pop_back();
      return (void*)s;
    }
  }
  hipSetDevice(d);
  hipStream_t s = nullptr;
  if (!UPH_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking))) return nullptr;
  return (void*)s;
}

void uphip_stream_release(void* stream) {
  if (!stream) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool_free[current_device()].push_back((hipStream_t)stream);
}

void uphip_stream_forget(void* stream) {
  if (!stream) return;
  const int dev = current_device();
  StreamScratch* e = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_scr_mu);
    auto it = g_scr.find({dev, (hipStream_t)stream});
    if (it == g_scr.end()) return;
    e = it->second;
    g_scr.erase(it);
  }
  hipSetDevice(dev);
  hipStreamSynchronize((hipStream_t)stream);  // its kernels were the only readers
  for (void* q : e->scr)
    if (q) hipFree(q);
  delete e;
  if (t_stream == (hipStream_t)stream) t_stream = nullptr;
}

void uphip_set_current_stream(void* stream) { t_stream = (hipStream_t)stream; }
void* uphip_get_current_stream(void) { return (void*)current_stream(); }

int uphip_synchronize(void) {
  if (!runtime_ready()) return -1;
  return UPH_HIP(hipStreamSynchronize(current_stream())) ? 0 : -1;
}

const char* uphip_last_error(void) { return t_has_error ? t_error.c_str() : nullptr; }
void uphip_clear_error(void) {
  t_has_error = false;
  t_error.clear();
}
void uphip_set_fatal_errors(bool fatal) { g_fatal = fatal; }
const char* uphip_version(void) {
#ifdef UPHIP_DIAG
  return "unpaper-hip 0.2 (gfx950, diag)";  // tuning build: UPHIP_DIAG_* honoured
#else
  return "unpaper-hip 0.2 (gfx950)";
#endif
}

size_t uphip_abi_sizeof(const char* name) {
#define S(T) \
  if (!strcmp(name, #T)) return sizeof(T);
  S(UphipPoint) S(UphipDelta) S(UphipDirection) S(UphipEdges) S(UphipPixel)
  S(UphipRectangle) S(UphipRectangleSize) S(UphipBorder) S(UphipWipes)
  S(UphipBlackfilterParameters) S(UphipBlurfilterParameters) S(UphipGrayfilterParameters)
  S(UphipMaskDetectionParameters) S(UphipMaskAlignmentParameters)
  S(UphipBorderScanParameters) S(UphipDeskewParameters) S(UphipOptions)
  S(UphipSheetReport) S(UphipBatchGeometry) S(UphipImage) S(UphipInterpolation) S(UphipLayout)
  S(UphipRunnerConfig) S(UphipDevicePages) S(UphipRunnerStats) S(UphipPnmInfo)
#undef S
  return 0;
}

size_t uphip_abi_offsetof(const char* type, const char* field) {
  // every field of the value types the reference's backend.h signatures use
  // (tests/golden/abi_layout.json holds the reference headers' offsets)
  if (!type || !field) return (size_t)-1;
#define O(T, F) \
  if (!strcmp(type, #T) && !strcmp(field, #F)) return __builtin_offsetof(T, F);
  O(UphipPoint, x)
  O(UphipPoint, y)
  O(UphipDelta, horizontal)
  O(UphipDelta, vertical)
  O(UphipDirection, horizontal)
  O(UphipDirection, vertical)
  O(UphipEdges, left)
  O(UphipEdges, top)
  O(UphipEdges, right)
  O(UphipEdges, bottom)
  O(UphipPixel, r)
  O(UphipPixel, g)
  O(UphipPixel, b)
  O(UphipRectangle, vertex[0].x)
  O(UphipRectangle, vertex[0].y)
  O(UphipRectangle, vertex[1].x)
  O(UphipRectangle, vertex[1].y)
  O(UphipRectangleSize, width)
  O(UphipRectangleSize, height)
  O(UphipImage, frame)
  O(UphipImage, background)
  O(UphipImage, abs_black_threshold)
  O(UphipBorder, left)
  O(UphipBorder, top)
  O(UphipBorder, right)
  O(UphipBorder, bottom)
  O(UphipWipes, count)
  O(UphipWipes, areas)
  O(UphipWipes, areas[99])
  O(UphipBlurfilterParameters, scan_size)
  O(UphipBlurfilterParameters, scan_step)
  O(UphipBlurfilterParameters, intensity)
  O(UphipGrayfilterParameters, scan_size)
  O(UphipGrayfilterParameters, scan_step)
  O(UphipGrayfilterParameters, abs_threshold)
  O(UphipBlackfilterParameters, scan_size)
  O(UphipBlackfilterParameters, scan_step)
  O(UphipBlackfilterParameters, scan_depth.horizontal)
  O(UphipBlackfilterParameters, scan_depth.vertical)
  O(UphipBlackfilterParameters, scan_direction)
  O(UphipBlackfilterParameters, abs_threshold)
  O(UphipBlackfilterParameters, intensity)
  O(UphipBlackfilterParameters, exclusions_count)
  O(UphipBlackfilterParameters, exclusions)
  O(UphipMaskDetectionParameters, scan_size)
  O(UphipMaskDetectionParameters, scan_step)
  O(UphipMaskDetectionParameters, scan_depth.horizontal)
  O(UphipMaskDetectionParameters, scan_depth.vertical)
  O(UphipMaskDetectionParameters, scan_direction)
  O(UphipMaskDetectionParameters, scan_threshold.horizontal)
  O(UphipMaskDetectionParameters, scan_threshold.vertical)
  O(UphipMaskDetectionParameters, minimum_width)
  O(UphipMaskDetectionParameters, maximum_width)
  O(UphipMaskDetectionParameters, minimum_height)
  O(UphipMaskDetectionParameters, maximum_height)
  O(UphipMaskAlignmentParameters, alignment)
  O(UphipMaskAlignmentParameters, margin)
  O(UphipBorderScanParameters, scan_size)
  O(UphipBorderScanParameters, scan_step)
  O(UphipBorderScanParameters, scan_threshold.horizontal)
  O(UphipBorderScanParameters, scan_threshold.vertical)
  O(UphipBorderScanParameters, scan_direction)
  O(UphipDeskewParameters, deskewScanRangeRad)
  O(UphipDeskewParameters, deskewScanStepRad)
  O(UphipDeskewParameters, deskewScanDeviationRad)
  O(UphipDeskewParameters, deskewScanSize)
  O(UphipDeskewParameters, deskewScanDepth)
  O(UphipDeskewParameters, scan_edges)
#undef O
  return (size_t)-1;
}

}  // extern "C"
