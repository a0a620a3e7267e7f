// Microbenchmark (calibration, not product): does a buffer the previous
// kernel wrote come back from the 256 MiB Infinity Cache (MALL) faster than
// from HBM, and does other traffic in between evict it — temporal vs
// non-temporal?  The question behind the fused step's cache policy
// (sw_kernels.hip: state/history non-temporal, mixed fields temporal).
// A = one set of mixed fields at 2048² (the row pass's forward outputs,
// 115 MB); the traffic in between is the column step's state/history
// streams (≈ 224 MB).  Prints the read rate of A per scenario.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_write(double2* __restrict__ p, long long n, double v) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = make_double2(v, (double)i);
}
__global__ void __launch_bounds__(256) k_read(const double2* __restrict__ p, long long n, double* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  double s = 0.0;
  if (i < n) {
    const double2 t = p[i];
    s = t.x + t.y;
  }
  if (s == -1.0) out[blockIdx.x] = s;  // (never: keeps the load)
}
template <bool NT>
__global__ void __launch_bounds__(256) k_rw(const double2* __restrict__ in, double2* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if constexpr (NT) {
    const double x = __builtin_nontemporal_load(&in[i].x), y = __builtin_nontemporal_load(&in[i].y);
    __builtin_nontemporal_store(x + 1.0, &out[i].x);
    __builtin_nontemporal_store(y, &out[i].y);
  } else {
    const double2 t = in[i];
    out[i] = make_double2(t.x + 1.0, t.y);
  }
}

int main() {
  const long long nA = 115LL * 1000 * 1000 / 16, nB = 600LL * 1000 * 1000 / 16, nC = 112LL * 1000 * 1000 / 16;
  double2 *A, *B, *C, *D;
  double* out;
  CK(hipMalloc(&A, nA * 16));
  CK(hipMalloc(&B, nB * 16));
  CK(hipMalloc(&C, nC * 16));
  CK(hipMalloc(&D, nC * 16));
  CK(hipMalloc(&out, (nA / 256 + 1) * 8));
  CK(hipMemset(B, 0, nB * 16));
  CK(hipMemset(C, 0, nC * 16));
  auto nb = [](long long n) { return dim3((unsigned)((n + 255) / 256)); };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"written just before (hot)", "then 600 MB written elsewhere (evicted)",
                         "then 224 MB non-temporal read+write", "then 224 MB temporal read+write",
                         "read twice (second read)"};
  for (int sc = 0; sc < 5; ++sc) {
    std::vector<float> t;
    for (int rep = 0; rep < 7; ++rep) {
      hipLaunchKernelGGL(k_write, nb(nA), dim3(256), 0, 0, A, nA, (double)rep);
      if (sc == 1) hipLaunchKernelGGL(k_write, nb(nB), dim3(256), 0, 0, B, nB, 1.0);
      if (sc == 2) hipLaunchKernelGGL((k_rw<true>), nb(nC), dim3(256), 0, 0, C, D, nC);
      if (sc == 3) hipLaunchKernelGGL((k_rw<false>), nb(nC), dim3(256), 0, 0, C, D, nC);
      if (sc == 4) hipLaunchKernelGGL(k_read, nb(nA), dim3(256), 0, 0, A, nA, out);
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_read, nb(nA), dim3(256), 0, 0, A, nA, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2] * 1e3;
    printf("read A (%.0f MB) %-42s %8.2f us  %6.0f GB/s\n", nA * 16 / 1e6, names[sc], us, nA * 16 / us / 1e3);
  }
  return 0;
}
