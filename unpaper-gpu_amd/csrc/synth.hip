// synth.hip — synthetic page generation (device + host) and raw device
// buffers for benchmarks and tests.  Not part of the cleanup path.
#include "runtime.h"
#include "synth.h"

namespace uph {

__global__ void __launch_bounds__(256) k_synth(uint8_t* dst, int64_t pitch, int64_t stride,
                                               int32_t W, int32_t H, uint32_t first) {
  const int p = blockIdx.z;
  uint8_t* page = dst + (int64_t)p * stride;
  const int32_t y = blockIdx.y;
  for (int32_t x = blockIdx.x * 256 + threadIdx.x; x < W; x += gridDim.x * 256)
    page[(int64_t)y * pitch + x] = synth_pixel(first + p, W, H, x, y);
}

__global__ void __launch_bounds__(256) k_synth_rgb(uint8_t* dst, int64_t pitch, int64_t stride,
                                                   int32_t W, int32_t H, uint32_t first) {
  const int p = blockIdx.z;
  uint8_t* page = dst + (int64_t)p * stride;
  const int32_t y = blockIdx.y;
  for (int32_t i = blockIdx.x * 256 + threadIdx.x; i < 3 * W; i += gridDim.x * 256)
    page[(int64_t)y * pitch + i] = synth_rgb_channel(first + p, W, H, i / 3, y, i % 3);
}

}  // namespace uph

using namespace uph;

extern "C" {

int uphip_synth_pages(void* dev, int64_t pitch, int64_t page_stride, int32_t W, int32_t H,
                      uint32_t first_page, int32_t count) {
  if (!runtime_ready()) return fail("synth: no HIP device"), -1;
  if (!dev || pitch < W || W <= 0 || H <= 0 || count <= 0) return fail("synth: bad args"), -1;
  hipStream_t st = current_stream();
  dim3 grid((W + 255) / 256, H, count);
  hipLaunchKernelGGL(k_synth, grid, dim3(256), 0, st, (uint8_t*)dev, pitch, page_stride, W, H,
                     first_page);
  return UPH_HIP(hipStreamSynchronize(st)) ? 0 : -1;
}

int uphip_synth_sheets_rgb(void* dev, int64_t pitch, int64_t sheet_stride, int32_t W, int32_t H,
                           uint32_t first_sheet, int32_t count) {
  if (!runtime_ready()) return fail("synth: no HIP device"), -1;
  if (!dev || pitch < 3 * (int64_t)W || W <= 1 || H <= 0 || count <= 0)
    return fail("synth: bad args"), -1;
  hipStream_t st = current_stream();
  dim3 grid((3 * W + 255) / 256, H, count);
  hipLaunchKernelGGL(k_synth_rgb, grid, dim3(256), 0, st, (uint8_t*)dev, pitch, sheet_stride, W,
                     H, first_sheet);
  return UPH_HIP(hipStreamSynchronize(st)) ? 0 : -1;
}

void uphip_synth_sheet_rgb_host(uint8_t* host, int64_t linesize, int32_t W, int32_t H,
                                uint32_t sheet) {
  for (int32_t y = 0; y < H; y++)
    for (int32_t x = 0; x < W; x++)
      for (int c = 0; c < 3; c++)
        host[(int64_t)y * linesize + 3 * x + c] = synth_rgb_channel(sheet, W, H, x, y, c);
}

void uphip_synth_page_host(uint8_t* host, int64_t linesize, int32_t W, int32_t H, uint32_t page) {
  for (int32_t y = 0; y < H; y++)
    for (int32_t x = 0; x < W; x++) host[(int64_t)y * linesize + x] = synth_pixel(page, W, H, x, y);
}

void* uphip_device_alloc(size_t bytes) {
  if (!runtime_ready()) return fail("device_alloc: no HIP device"), nullptr;
  void* p = nullptr;
  hipSetDevice(current_device());
  if (!UPH_HIP(hipMalloc(&p, bytes ? bytes : 1))) return nullptr;
  return p;
}

void uphip_device_free(void* p) {
  if (p) hipFree(p);
}

void* uphip_host_alloc(size_t bytes) {
  if (!runtime_ready()) return fail("host_alloc: no HIP device"), nullptr;
  void* p = nullptr;
  if (!UPH_HIP(hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault))) return nullptr;
  return p;
}

void uphip_host_free(void* p) {
  if (p) hipHostFree(p);
}

int uphip_memcpy_htod(void* dst, const void* src, size_t bytes) {
  return UPH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)) ? 0 : -1;
}

int uphip_memcpy_dtoh(void* dst, const void* src, size_t bytes) {
  return UPH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)) ? 0 : -1;
}

}  // extern "C"
