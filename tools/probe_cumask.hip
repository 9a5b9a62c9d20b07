// Dev probe (never part of the product): what hipExtStreamCreateWithCUMask does on this device.
// A kernel on a stream masked to "all CUs but the last R" and one masked to "the last R" record
// the hardware ids (XCC, SE, CU) their blocks ran on; then a CU hog (256 VGPRs, 80 KB LDS) on
// the big stream and a small kernel on the reserved stream show whether the two run together.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe_cumask.hip -o tools/build/probe_cumask
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <tuple>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);        \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

__device__ inline unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__global__ void where(unsigned* ids) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11)); // HW_REG_XCC_ID
    ids[2 * blockIdx.x] = hw;
    ids[2 * blockIdx.x + 1] = xcc;
  }
  const unsigned long long t0 = rt();
  while (rt() - t0 < 2000) __builtin_amdgcn_s_sleep(4);  // 20 us: spread over the CUs
}

__global__ __launch_bounds__(256, 2) void hog(double* sink, unsigned long long t, unsigned long long* t_end) {
  __shared__ double lds[10240];
  const unsigned long long t0 = rt();
  double acc = threadIdx.x;
  asm volatile("v_mov_b32 v255, 0" ::: "v255");
  for (int i = threadIdx.x; i < 10240; i += 256) lds[i] = i;
  __syncthreads();
  while (rt() - t0 < t) {
    acc += lds[(threadIdx.x * 7) % 10240] * 1e-9;
    __builtin_amdgcn_s_sleep(2);
  }
  if (acc == -1.0) sink[0] = acc;
  if (blockIdx.x == 0 && threadIdx.x == 0) t_end[0] = rt();
}

__global__ void small(unsigned long long* t_small) {
  if (blockIdx.x == 0 && threadIdx.x == 0) t_small[0] = rt();
}

static void report(const char* name, hipStream_t s, int blocks) {
  unsigned* d = nullptr;
  CK(hipMalloc(&d, sizeof(unsigned) * 2 * blocks));
  CK(hipMemset(d, 0xff, sizeof(unsigned) * 2 * blocks));
  where<<<blocks, 64, 0, s>>>(d);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(s));
  std::vector<unsigned> h(2 * blocks);
  CK(hipMemcpy(h.data(), d, sizeof(unsigned) * 2 * blocks, hipMemcpyDeviceToHost));
  std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> cus;
  std::set<unsigned> xccs;
  for (int b = 0; b < blocks; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    cus.insert({xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 0xf});
    xccs.insert(xcc);
  }
  std::printf("{\"probe\": \"%s\", \"blocks\": %d, \"distinct_cus\": %zu, \"xccs\": [", name, blocks, cus.size());
  bool first = true;
  for (unsigned x : xccs) { std::printf("%s%u", first ? "" : ", ", x); first = false; }
  std::printf("], \"cus_per_xcc\": [");
  first = true;
  for (unsigned x : xccs) {
    int k = 0;
    for (auto& t : cus) k += std::get<0>(t) == x;
    std::printf("%s%d", first ? "" : ", ", k);
    first = false;
  }
  std::printf("]}\n");
  CK(hipFree(d));
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? std::atoi(argv[1]) : 8;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int words = (ncu + 31) / 32;
  std::vector<uint32_t> mc(words, 0), mh(words, 0);
  for (int i = 0; i < ncu; ++i) (i >= ncu - R ? mh : mc)[i / 32] |= 1u << (i % 32);
  hipStream_t sc, sh, sp;
  CK(hipExtStreamCreateWithCUMask(&sc, words, mc.data()));
  CK(hipExtStreamCreateWithCUMask(&sh, words, mh.data()));
  CK(hipStreamCreateWithFlags(&sp, hipStreamNonBlocking));
  std::vector<uint32_t> g(words, 0);
  CK(hipExtStreamGetCUMask(sh, words, g.data()));
  std::printf("{\"ncu\": %d, \"reserve\": %d, \"helper_mask_words\": [", ncu, R);
  for (int i = 0; i < words; ++i) std::printf("%s\"%08x\"", i ? ", " : "", g[i]);
  std::printf("]}\n");
  report("plain", sp, 4096);
  report("compute_mask", sc, 4096);
  report("helper_mask", sh, 1024);
  // concurrency: the hog (on the compute mask, 2 blocks per masked CU) for 50 ms; the small
  // kernel on the helper mask 5 ms later
  double* sink = nullptr;
  unsigned long long* t = nullptr;
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&t, 64));
  CK(hipMemset(t, 0, 64));
  unsigned long long h0 = 0;
  hog<<<2 * (ncu - R), 256, 0, sc>>>(sink, 5000000ull, t);
  CK(hipGetLastError());
  // host-side 5 ms delay, then the small kernel
  const auto c0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count() < 5.0) {}
  small<<<1, 64, 0, sh>>>(t + 1);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(sh));
  const auto c1 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(sc));
  unsigned long long ht[2];
  CK(hipMemcpy(ht, t, sizeof ht, hipMemcpyDeviceToHost));
  std::printf("{\"probe\": \"concurrency\", \"small_done_host_ms\": %.2f, \"small_before_hog_end_ms\": %.2f}\n",
              std::chrono::duration<double, std::milli>(c1 - c0).count(), (double)(long long)(ht[0] - ht[1]) * 1e-5);
  (void)h0;
  std::printf("{\"probe\": \"done\"}\n");
  return 0;
}
