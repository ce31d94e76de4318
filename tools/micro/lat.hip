// latency probes for the blackfilter replay's cost model (tuning only)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k_lat(uint64_t* buf, uint64_t* out, int n, int mode) {
  const int lane = threadIdx.x;
  uint64_t acc = 0;
  uint64_t t0 = 0, t1 = 0;
  // warm: touch the lines
  uint64_t idx = lane;
  for (int i = 0; i < 64; i++) acc += __hip_atomic_load(buf + ((i * 64 + lane) & 8191), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_s_waitcnt(0);
  t0 = wall_clock64();
  uint64_t c0 = clock64();
  for (int i = 0; i < n; i++) {
    if (mode == 0) {  // dependent load chain, same 64 lines
      uint64_t v = __hip_atomic_load(buf + ((idx + acc) & 4095), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += v & 1;
      idx += 64;
    } else if (mode == 1) {  // dependent: ballot of a load, next address from ballot
      uint64_t v = __hip_atomic_load(buf + ((idx + acc) & 4095), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint64_t b = __ballot(v & 1);
      acc += b & 1;
      idx += 64;
    } else if (mode == 2) {  // atomic or, then dependent load of the same word
      __hip_atomic_fetch_or(buf + ((idx + acc) & 4095), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint64_t v = __hip_atomic_load(buf + ((idx + acc) & 4095), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += v & 1;
      idx += 64;
    } else if (mode == 3) {  // timer cost
      acc += wall_clock64() & 1;
    } else if (mode == 4) {  // plain (L1) dependent loads
      uint64_t v = buf[(idx + acc) & 4095];
      acc += v & 1;
      idx += 64;
    } else if (mode == 5) {  // LDS dependent chain
      __shared__ uint64_t sh[4096];
      uint64_t v = sh[(idx + acc) & 4095];
      acc += v & 1;
      idx += 64;
    } else if (mode == 6) {  // 64 distinct lines per load (column access), dependent
      uint64_t v = __hip_atomic_load(buf + (((idx + acc) * 16 + lane * 16) & 262143), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += __ballot(v & 1) & 1;
      idx += 1;
    } else if (mode == 8 || mode == 9 || mode == 10) {  // 64-lane atomic or, then dependent load
      const int sh = mode == 8 ? 3 : mode == 9 ? 6 : 0;
      const uint64_t a = ((idx + acc) & 2047) + (uint64_t)((lane >> sh) << (mode == 10 ? 4 : 0));
      __hip_atomic_fetch_or(buf + a, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint64_t v = __hip_atomic_load(buf + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += v & 1;
      idx += 64;
    } else if (mode == 11) {  // 4 such atomics (8 lanes a word) back to back, then a load
      for (int q = 0; q < 4; q++)
        __hip_atomic_fetch_or(buf + ((idx + acc + 256 * q) & 2047) + (lane >> 3), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      uint64_t v = __hip_atomic_load(buf + ((idx + acc) & 2047), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += v & 1;
      idx += 64;
    } else if (mode == 12) {  // plain store (8 lanes a word, same value), then a load
      buf[((idx + acc) & 2047) + (lane >> 3)] = 0;
      uint64_t v = __hip_atomic_load(buf + ((idx + acc) & 2047), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      acc += v & 1;
      idx += 64;
    } else if (mode == 7) {  // 64 dependent SALU-ish ops: ballot + ffs chain
      uint64_t b = __ballot(((acc + lane) & 3) == 0);
      acc += __ffsll((long long)b);
    }
  }
  t1 = wall_clock64();
  uint64_t c1 = clock64();
  if (lane == 0) { out[0] = t1 - t0; out[1] = c1 - c0; out[2] = acc; }
}
int main() {
  uint64_t *buf, *out;
  hipMalloc(&buf, 8 << 20);
  hipMemset(buf, 0, 8 << 20);
  hipMalloc(&out, 64);
  const char* names[] = {"dep load sc0 (L2/L1)", "dep load+ballot", "atomic+load same word", "wall_clock64",
                         "dep load plain", "dep LDS load", "64-line load+ballot", "ballot+ffs chain",
                         "atomic 8 lanes/word", "atomic 64 lanes/word", "atomic 1 lane/word", "4 atomics 8/word", "store 8 lanes/word"};
  for (int mode = 0; mode < 13; mode++) {
    const int n = 1000;
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, buf, out, n, mode);
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, buf, out, n, mode);
    uint64_t h[3];
    hipMemcpy(h, out, 24, hipMemcpyDeviceToHost);
    printf("%-24s %8.1f ns/iter  %8.1f clk/iter\n", names[mode], h[0] * 10.0 / n, (double)h[1] / n);
  }
  return 0;
}
