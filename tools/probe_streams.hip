// Dev probe (never part of the product): two facts the streamed host pipeline depends on.
//  1. hipStreamWaitValue64 on hipMallocSignalMemory: does a stream waiting on a counter start
//     its next kernel while the kernel that bumps the counter (system-scope atomic) is still
//     running? Prints the s_memrealtime stamps of the bump, of the waiting stream's marker kernel
//     and of the bumping kernel's end.
//  2. Device->pinned-host copies (hipMemcpyAsync) next to a kernel that holds every CU slot
//     (256 VGPRs, 80 KB LDS per block, 2 blocks per CU) or all but a few: copy time alone, under
//     the full hog and under the reduced hog.
// Every wait is satisfied unconditionally (the bump always happens), every kernel has a bounded
// run time. Build: hipcc --offload-arch=gfx950 -O2 tools/probe_streams.hip -o tools/build/probe_streams
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__device__ inline unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// sleeps ~t1 ticks, bumps the counter (block 0, lane 0), sleeps ~t2 more
__global__ void bumper(unsigned long long* sig, unsigned long long* stamp, unsigned long long t1,
                       unsigned long long t2) {
  const unsigned long long t0 = rt();
  while (rt() - t0 < t1) __builtin_amdgcn_s_sleep(10);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    stamp[0] = rt();
    __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  while (rt() - t0 < t1 + t2) __builtin_amdgcn_s_sleep(10);
  if (blockIdx.x == 0 && threadIdx.x == 0) stamp[1] = rt();
}

__global__ void marker(unsigned long long* stamp) {
  if (threadIdx.x == 0) stamp[2] = rt();
}

// a CU hog: 80 KB of LDS per block and the whole VGPR budget of 2 waves/SIMD, for ~t ticks
__global__ __launch_bounds__(256, 2) void hog(double* sink, unsigned long long t) {
  __shared__ double lds[10240];
  const unsigned long long t0 = rt();
  double acc = threadIdx.x;
  asm volatile("v_mov_b32 v255, 0" ::: "v255");  // the integrator's register budget: 256 VGPRs
  for (int i = threadIdx.x; i < 10240; i += 256) lds[i] = i;
  __syncthreads();
  while (rt() - t0 < t) {
    acc += lds[(threadIdx.x * 7) % 10240] * 1e-9;
    __builtin_amdgcn_s_sleep(2);
  }
  if (acc == -1.0) sink[0] = acc;
}

int main() {
  int dev = 0, can = -1, ncu = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::printf("{\"can_use_stream_wait_value\": %d, \"cus\": %d}\n", can, ncu);
  hipStream_t sa, sb, sc;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  // ---- 1. wait value ----
  if (can) {
    unsigned long long *sig = nullptr, *stamp = nullptr;
    CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
    CK(hipMalloc(&stamp, 64));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(sig, 0, 8));
      CK(hipMemset(stamp, 0, 64));
      CK(hipDeviceSynchronize());
      CK(hipStreamWaitValue64(sb, sig, 1, hipStreamWaitValueGte));
      marker<<<1, 64, 0, sb>>>(stamp);
      bumper<<<4, 64, 0, sa>>>(sig, stamp, 2000000ull /* 20 ms */, 3000000ull /* 30 ms */);
      CK(hipGetLastError());
      CK(hipStreamSynchronize(sa));
      CK(hipStreamSynchronize(sb));
      unsigned long long h[3];
      CK(hipMemcpy(h, stamp, sizeof h, hipMemcpyDeviceToHost));
      std::printf("{\"probe\": \"wait_value\", \"rep\": %d, \"bump_to_marker_ms\": %.3f, \"bump_to_end_ms\": %.3f}\n", rep,
                  (double)(long long)(h[2] - h[0]) * 1e-5, (double)(long long)(h[1] - h[0]) * 1e-5);
    }
    CK(hipFree(sig));
    CK(hipFree(stamp));
  }
  // ---- 2. D2H copies next to a CU hog ----
  const size_t bytes = size_t(256) << 20;
  void *d = nullptr, *h = nullptr;
  double* sink = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(d, 1, bytes));
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto copy_ms = [&]() {
    CK(hipEventRecord(e0, sc));
    CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, sc));
    CK(hipEventRecord(e1, sc));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  copy_ms();
  std::printf("{\"probe\": \"d2h_alone\", \"MB\": 256, \"ms\": %.3f}\n", copy_ms());
  for (int spare : {0, 8, 32}) {  // CUs' worth of hog blocks left out
    const int blocks = 2 * (ncu - spare);
    hog<<<blocks, 256, 0, sa>>>(sink, 8000000ull /* 80 ms */);
    CK(hipGetLastError());
    auto t0 = std::chrono::steady_clock::now();
    // let the hog occupy the device first
    while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() < 5.0) {}
    const float ms = copy_ms();
    CK(hipStreamSynchronize(sa));
    std::printf("{\"probe\": \"d2h_under_hog\", \"spare_cus\": %d, \"MB\": 256, \"ms\": %.3f}\n", spare, ms);
  }
  CK(hipDeviceSynchronize());
  std::printf("{\"probe\": \"done\"}\n");
  return 0;
}
