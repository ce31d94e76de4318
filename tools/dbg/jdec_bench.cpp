// jdec_bench.cpp — development probe: times the device Huffman decode
// (jdec_launch_batch) alone on a batch of JPEG files, without the runner's
// other kernels competing for the CUs.  Usage: jdec_bench N REPS file...
// (N pages, files reused round robin).  Build: tools/dbg/jdec_bench.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "jpeg.h"

using namespace uph;

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      exit(1);                                                       \
    }                                                                \
  } while (0)

static std::vector<uint8_t> slurp(const char* p) {
  FILE* f = fopen(p, "rb");
  if (!f) exit(2);
  std::vector<uint8_t> v;
  uint8_t b[65536];
  size_t r;
  while ((r = fread(b, 1, sizeof b, f)) > 0) v.insert(v.end(), b, b + r);
  fclose(f);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int n = atoi(argv[1]), reps = atoi(argv[2]), nf = argc - 3;
  std::vector<JdecStreamHost> S(nf);
  for (int i = 0; i < nf; i++) {
    auto f = slurp(argv[3 + i]);
    if (jpeg_stream_prepare(f.data(), f.size(), argv[3 + i], &S[i]) != 1) return 3;
  }
  std::vector<JdecJob> jobs(n);
  int64_t mx = 0, mm = 0, bits = 0;
  int32_t* dst;
  CK(hipMalloc(&dst, 4 * n));
  CK(hipMemset(dst, 0, 4 * n));
  for (int i = 0; i < n; i++) {
    const JdecStreamHost& s = S[i % nf];
    std::vector<uint8_t> h((size_t)s.hd.total_bytes + 16);
    jpeg_stream_pack(s, h.data());
    uint8_t *ds, *dp, *dsc;
    CK(hipMalloc(&ds, h.size()));
    CK(hipMemcpy(ds, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMalloc(&dp, s.hd.h.total_bytes));
    CK(hipMalloc(&dsc, jdec_scratch_bytes(s.hd)));
    jobs[i] = JdecJob{ds, dp, dsc, dst + i};
    mx = std::max<int64_t>(mx, s.hd.nsub);
    mm = std::max<int64_t>(mm, s.hd.nmac);
    bits += s.hd.nbits;
  }
  JdecJob* dj;
  CK(hipMalloc(&dj, sizeof(JdecJob) * n));
  CK(hipMemcpy(dj, jobs.data(), sizeof(JdecJob) * n, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  if (!jdec_launch_batch(dj, n, mx, mm, st)) return 4;
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; r++)
    if (!jdec_launch_batch(dj, n, mx, mm, st)) return 4;
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<int32_t> stv(n);
  CK(hipMemcpy(stv.data(), dst, 4 * n, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int v : stv) bad += v != 0;
  printf("{\"pages\": %d, \"ms_per_batch\": %.3f, \"pages_per_s\": %.1f, \"Mbit_per_page\": %.2f, "
         "\"nsub\": %lld, \"nmac\": %lld, \"bad\": %d}\n",
         n, ms / reps, n * reps / (ms / 1e3), bits / 1e6 / n, (long long)mx, (long long)mm, bad);
  return bad ? 5 : 0;
}
