// Microbenchmark (calibration, not product): achievable HBM rate on MI355X
// for R read streams + W write streams of 16-B elements, each stream `n`
// elements (default 0.93M = one compact field at 2048²), launched as one
// thread per element, 256 threads per block.  Prints GB/s per (R, W).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int R, int W>
__global__ void __launch_bounds__(256) k_mix(const double2* __restrict__ in, double2* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double2 a = make_double2(0.0, 0.0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double2 t = in[r * n + i];
    a.x += t.x;
    a.y += t.y;
  }
#pragma unroll
  for (int w = 0; w < W; ++w) out[w * n + i] = make_double2(a.x + w, a.y);
}

template <int R, int W>
void run(long long n, double2* in, double2* out) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int nb = (int)((n + 255) / 256);
  for (int it = 0; it < 5; ++it) hipLaunchKernelGGL((k_mix<R, W>), dim3(nb), dim3(256), 0, 0, in, out, n);
  const int reps = 50;
  CK(hipEventRecord(e0));
  for (int it = 0; it < reps; ++it) hipLaunchKernelGGL((k_mix<R, W>), dim3(nb), dim3(256), 0, 0, in, out, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  const double bytes = (double)(R + W) * n * 16;
  printf("R=%d W=%d  %.1f MB  %.2f us  %.0f GB/s\n", R, W, bytes / 1e6, us, bytes / us / 1e3);
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 682LL * 1368 * 3;
  double2 *in, *out;
  CK(hipMalloc(&in, 15 * n * sizeof(double2)));
  CK(hipMalloc(&out, 8 * n * sizeof(double2)));
  CK(hipMemset(in, 0, 15 * n * sizeof(double2)));
  run<1, 1>(n, in, out);
  run<2, 0>(n, in, out);
  run<0, 2>(n, in, out);
  run<5, 2>(n, in, out);
  run<9, 4>(n, in, out);
  run<3, 2>(n, in, out);
  run<12, 6>(n, in, out);
  // write-heavy mixes (the 8192-point column inverse: 2 compact reads, 6 mixed writes)
  run<0, 6>(n, in, out);
  run<1, 3>(n, in, out);
  run<2, 6>(n, in, out);
  run<1, 6>(n, in, out);
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
