// synth.hip — synthetic page generation (device + host) and raw device
// buffers for benchmarks and tests.  Not part of the cleanup path.
#include <cmath>
#include <cstring>
#include <vector>

#include "libm_glibc.h"
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

// uphip_check_libm: the device's glibc sinf/cosf/powf(x, 2) (libm_glibc.h)
// over every `stride`-th float bit pattern from `first`, both signs
__global__ void __launch_bounds__(256) k_libm_eval(uint32_t first, uint32_t stride, int64_t n,
                                                   const uint32_t* pow2, int npow2, float* out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t u = first + (uint32_t)((i >> 1) * stride) | (uint32_t)(i & 1) << 31;
  float x;
  __builtin_memcpy(&x, &u, 4);
  out[3 * i] = glibc::sinf(x);
  out[3 * i + 1] = glibc::cosf(x);
  out[3 * i + 2] = glibc::pow2(x, pow2, npow2);
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

int uphip_check_libm(uint32_t stride, uint64_t counts[4]) {
  if (!runtime_ready()) return fail("check_libm: no HIP device"), -1;
  if (!counts || stride == 0) return fail("check_libm: bad args"), -1;
  int npow2 = 0;
  const uint32_t* t = glibc_pow2_table(&npow2);
  if (!t) return fail("check_libm: powf(x, 2) not reproducible"), -1;
  static float (*volatile h_sinf)(float) = ::sinf;
  static float (*volatile h_cosf)(float) = ::cosf;
  static float (*volatile h_powf)(float, float) = ::powf;
  hipStream_t st = current_stream();
  uint32_t* dtab = (uint32_t*)uphip_device_alloc(sizeof(uint32_t) * (npow2 + 1));
  const int64_t chunk = 1 << 24;
  float* dout = (float*)uphip_device_alloc(sizeof(float) * 3 * chunk);
  std::vector<float> out((size_t)3 * chunk);
  bool ok = dtab && dout && UPH_HIP(hipMemcpy(dtab, t, sizeof(uint32_t) * npow2,
                                              hipMemcpyHostToDevice));
  memset(counts, 0, 4 * sizeof(uint64_t));
  // sin/cos over |x| < 120 (0x42F00000); powf(x, 2) over 2^-60 <= |x| < 2^61
  const uint32_t ranges[2][2] = {{0u, 0x42F00000u}, {(127u - 60) << 23, (127u + 61) << 23}};
  for (int r = 0; r < 2 && ok; r++) {
    const int64_t total = 2 * (((int64_t)ranges[r][1] - ranges[r][0] + stride - 1) / stride);
    for (int64_t base = 0; base < total && ok; base += chunk) {
      const int64_t n = total - base < chunk ? total - base : chunk;
      const uint32_t first = ranges[r][0] + (uint32_t)((base >> 1) * stride);
      hipLaunchKernelGGL(k_libm_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, first,
                         stride, n, dtab, npow2, dout);
      ok = UPH_HIP(hipMemcpyAsync(out.data(), dout, sizeof(float) * 3 * n, hipMemcpyDeviceToHost,
                                  st)) &&
           UPH_HIP(hipStreamSynchronize(st));
      for (int64_t i = 0; i < n && ok; i++) {
        uint32_t u = first + (uint32_t)((i >> 1) * stride) | (uint32_t)(i & 1) << 31;
        float x, e[3];
        memcpy(&x, &u, 4);
        if (r == 0) {
          e[0] = h_sinf(x);
          e[1] = h_cosf(x);
          counts[0] += memcmp(&e[0], &out[3 * i], 4) != 0;
          counts[1] += memcmp(&e[1], &out[3 * i + 1], 4) != 0;
        } else {
          e[2] = h_powf(x, 2.0f);
          counts[2] += memcmp(&e[2], &out[3 * i + 2], 4) != 0;
        }
        counts[3]++;
      }
    }
  }
  uphip_device_free(dout);
  uphip_device_free(dtab);
  return ok ? 0 : -1;
}

int uphip_memcpy_htod(void* dst, const void* src, size_t bytes) {
  return UPH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)) ? 0 : -1;
}

int uphip_memcpy_dtoh(void* dst, const void* src, size_t bytes) {
  return UPH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)) ? 0 : -1;
}

}  // extern "C"
