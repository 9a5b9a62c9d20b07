// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access width the engine uses:
// 8 bytes per lane (one f64 per lane, SoA), coalesced. Each kernel reads N doubles and
// writes N doubles; the printed byte counts are the ground truth that tools/pmc_summary.py
// divides the counters by. Also runs the 16-B/lane variant the microarch guide calibrates.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void copy8(const double* __restrict__ a, double* __restrict__ b, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    b[i] = 2.0 * a[i];
}

__global__ void copy16(const double2* __restrict__ a, double2* __restrict__ b, long n2) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
    double2 v = a[i];
    v.x *= 2.0; v.y *= 2.0;
    b[i] = v;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const long n = 1L << 27;  // 1 GiB per array: well past the 256 MiB Infinity Cache
  double *a, *b;
  CK(hipMalloc(&a, n * sizeof(double)));
  CK(hipMalloc(&b, n * sizeof(double)));
  CK(hipMemset(a, 0, n * sizeof(double)));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(copy8, dim3(8192), dim3(256), 0, 0, a, b, n);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, 0, (const double2*)a, (double2*)b, n / 2);
  CK(hipDeviceSynchronize());
  printf("{\"copy8_read_bytes\": %ld, \"copy8_write_bytes\": %ld, \"copy16_read_bytes\": %ld, \"copy16_write_bytes\": %ld}\n",
         n * 8, n * 8, n * 8, n * 8);
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
