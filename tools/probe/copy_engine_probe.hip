// Dev probe: do hipMemcpyAsync H2D / D2H copies progress while a kernel holds every CU slot?
// A blit-kernel copy waits for the hog to end; an SDMA copy finishes during it. The hog spins a
// bounded time (s_memrealtime, 100 MHz) and every wave exits, so the grid always drains.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__global__ void tiny(double* sink) {
  if (threadIdx.x == 0) sink[1] = 1.0;
}

__global__ __launch_bounds__(256) void hog(unsigned long long ticks, double* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  double a = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    for (int i = 0; i < 64; ++i) a = __builtin_fma(a, 0.999999, 1e-9);
  }
  if (a == -1.0) sink[0] = a;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bytes = 64ull << 20;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  double* sink;
  CK(hipMalloc(&sink, 64));
  void *dev, *pin_coh, *pin_nc, *reg;
  CK(hipMalloc(&dev, bytes));
  CK(hipHostMalloc(&pin_coh, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&pin_nc, bytes, hipHostMallocNonCoherent));
  reg = std::aligned_alloc(4096, bytes);
  std::memset(reg, 1, bytes);
  CK(hipHostRegister(reg, bytes, hipHostRegisterDefault));
  hipStream_t sk, sc;
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  struct Case { const char* name; void* host; bool h2d; };
  const Case cases[] = {{"h2d_hostmalloc", pin_coh, true},   {"d2h_hostmalloc", pin_coh, false},
                        {"h2d_noncoherent", pin_nc, true},   {"d2h_noncoherent", pin_nc, false},
                        {"h2d_registered", reg, true},       {"d2h_registered", reg, false},
                        {"control_kernel", nullptr, true}};
  // warm up every path once
  for (const Case& c : cases)
    if (c.host) CK(hipMemcpyAsync(c.h2d ? dev : c.host, c.h2d ? c.host : dev, bytes, c.h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, sc));
  CK(hipStreamSynchronize(sc));
  // the hog: 8 blocks of 256 per CU (every wave slot of a small kernel), 300 ms
  const unsigned long long ticks = 30'000'000ull;
  for (const Case& c : cases) {
    hipEvent_t k1, c0, c1;
    CK(hipEventCreate(&k1));
    CK(hipEventCreate(&c0));
    CK(hipEventCreate(&c1));
    const double t0 = now_ms();
    hipLaunchKernelGGL(hog, dim3(ncu * 8), dim3(256), 0, sk, ticks, sink);
    CK(hipGetLastError());
    CK(hipEventRecord(k1, sk));
    std::this_thread::sleep_for(std::chrono::milliseconds(20));  // the hog is resident
    CK(hipEventRecord(c0, sc));
    if (c.host) {
      CK(hipMemcpyAsync(c.h2d ? dev : c.host, c.h2d ? c.host : dev, bytes, c.h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, sc));
    } else {  // control: does a tiny kernel find a free slot under the hog?
      hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, sc, sink);
      CK(hipGetLastError());
    }
    CK(hipEventRecord(c1, sc));
    double tc = -1, tk = -1;
    while (tc < 0 || tk < 0) {
      if (tc < 0 && hipEventQuery(c1) == hipSuccess) tc = now_ms() - t0;
      if (tk < 0 && hipEventQuery(k1) == hipSuccess) tk = now_ms() - t0;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, c0, c1));
    std::printf("{\"case\": \"%s\", \"copy_done_ms\": %.2f, \"hog_done_ms\": %.2f, \"copy_ms\": %.3f, \"GB_s\": %.1f, \"overlapped\": %s}\n",
                c.name, tc, tk, ms, bytes / (ms * 1e6), tc < tk ? "true" : "false");
    std::fflush(stdout);
  }
  return 0;
}
