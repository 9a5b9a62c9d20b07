// Dev: host-side transfer rates on the GPU box, for the design of art_propagate_host's chunked
// pipeline (art_capi.cpp). Measures, for a 1.5 GB buffer (the D2H volume of a 1e7-ray call):
//   * multi-threaded memcpy between pageable memory and hipHostMalloc'd pinned memory,
//     1/2/4/8/16 threads (the gather/scatter of the pipeline);
//   * hipHostRegister / hipHostUnregister of pageable memory (the alternative: DMA straight
//     into the caller's arrays);
//   * DMA rates H2D / D2H for pinned, registered and pageable host memory.
// Build: hipcc -O2 -std=c++17 tools/host_copy_bench.cpp -o tools/build/host_copy_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par_copy(char* dst, const char* src, size_t bytes, int nt) {
  std::vector<std::thread> th;
  const size_t per = (bytes + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const size_t a = t * per, b = std::min(bytes, a + per);
    if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main() {
  const size_t B = size_t(1520) << 20;
  char* pg = (char*)std::malloc(B);
  char* pg2 = (char*)std::malloc(B);
  std::memset(pg, 1, B);
  std::memset(pg2, 2, B);
  char* pin = nullptr;
  CK(hipHostMalloc((void**)&pin, B, hipHostMallocDefault));
  std::memset(pin, 3, B);
  void* dev = nullptr;
  CK(hipMalloc(&dev, B));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  std::printf("{\"bytes\": %zu", B);
  for (int nt : {1, 2, 4, 8, 16}) {
    double t0 = now();
    par_copy(pin, pg, B, nt);
    double t1 = now();
    par_copy(pg2, pin, B, nt);
    double t2 = now();
    std::printf(", \"memcpy_to_pinned_%dt_GBs\": %.2f, \"memcpy_from_pinned_%dt_GBs\": %.2f", nt, B / (t1 - t0) / 1e9, nt,
                B / (t2 - t1) / 1e9);
  }
  // DMA from pinned
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    CK(hipMemcpyAsync(dev, pin, B, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double t1 = now();
    CK(hipMemcpyAsync(pin, dev, B, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    double t2 = now();
    if (rep) std::printf(", \"dma_pinned_h2d_GBs\": %.2f, \"dma_pinned_d2h_GBs\": %.2f", B / (t1 - t0) / 1e9, B / (t2 - t1) / 1e9);
  }
  // both directions at once (two streams)
  {
    hipStream_t s2;
    CK(hipStreamCreate(&s2));
    char* pin2 = nullptr;
    CK(hipHostMalloc((void**)&pin2, B / 2, hipHostMallocDefault));
    void* dev2 = nullptr;
    CK(hipMalloc(&dev2, B / 2));
    double t0 = now();
    CK(hipMemcpyAsync(dev, pin, B / 2, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(pin2, dev2, B / 2, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(s2));
    double t1 = now();
    std::printf(", \"dma_pinned_duplex_GBs\": %.2f", B / (t1 - t0) / 1e9);
    CK(hipHostFree(pin2));
    CK(hipFree(dev2));
    CK(hipStreamDestroy(s2));
  }
  // pageable DMA
  {
    double t0 = now();
    CK(hipMemcpyAsync(dev, pg, B, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double t1 = now();
    CK(hipMemcpyAsync(pg2, dev, B, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    double t2 = now();
    std::printf(", \"dma_pageable_h2d_GBs\": %.2f, \"dma_pageable_d2h_GBs\": %.2f", B / (t1 - t0) / 1e9, B / (t2 - t1) / 1e9);
  }
  // register pageable memory in place, DMA, unregister
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    CK(hipHostRegister(pg2, B, hipHostRegisterDefault));
    double t1 = now();
    CK(hipMemcpyAsync(pg2, dev, B, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    double t2 = now();
    CK(hipHostUnregister(pg2));
    double t3 = now();
    std::printf(", \"register_ms_%d\": %.1f, \"dma_registered_d2h_GBs_%d\": %.2f, \"unregister_ms_%d\": %.1f", rep,
                (t1 - t0) * 1e3, rep, B / (t2 - t1) / 1e9, rep, (t3 - t2) * 1e3);
  }
  std::printf("}\n");
  CK(hipFree(dev));
  CK(hipHostFree(pin));
  std::free(pg);
  std::free(pg2);
  return 0;
}
