// runtime.h — host runtime of the HIP backend: devices, thread-local current
// device/stream (cuda_runtime.c:70 peer), error reporting, argument staging.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "common.h"

struct UphipFrame {
  uint8_t* data;     // device pointer, rows `pitch` bytes apart (256-aligned)
  int64_t pitch;
  int32_t width, height;
  int32_t format;    // UphipPixelFormat
  int32_t device;
};

namespace uph {

// Record an error (and exit when fatal errors are on).  Returns false.
bool fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
bool check_hip(hipError_t e, const char* what);
#define UPH_HIP(call) ::uph::check_hip((call), #call)

int current_device();
hipStream_t current_stream();   // per-thread stream of the current device
bool runtime_ready();           // uphip_try_init() succeeded

// Argument staging: small per-launch argument blocks copied host->device on
// the current stream.  The returned device pointer stays valid until the
// ring wraps (each slot is fenced by an event).
struct ArgBlock {
  void* host;
  void* dev;
};
ArgBlock arg_alloc(size_t bytes);
bool arg_commit(const ArgBlock& b, size_t bytes, hipStream_t st);
// Call after launching the kernels that read the committed blocks.
void arg_fence(hipStream_t st);

template <class T>
T* stage_args(const T* host_items, size_t n, hipStream_t st) {
  ArgBlock b = arg_alloc(sizeof(T) * n);
  if (!b.dev) return nullptr;
  memcpy(b.host, host_items, sizeof(T) * n);
  if (!arg_commit(b, sizeof(T) * n, st)) return nullptr;
  return static_cast<T*>(b.dev);
}

// Device scratch of the current stream (per device), grown on demand;
// stream-ordered, so a thread may switch streams between ops.
void* scratch(int slot, size_t bytes);

// Frame helpers
UphipFrame* frame_alloc(int32_t w, int32_t h, int32_t fmt);
void frame_free(UphipFrame* f);
Planes frame_planes(const UphipFrame* f);

}  // namespace uph
