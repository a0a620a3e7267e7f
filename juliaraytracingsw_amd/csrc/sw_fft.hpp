// Device-side fp64 FFT primitive for gfx950: one power-of-two transform of
// length N per "line", NT = N/8 threads per line, 8 complex points per thread,
// Stockham autosort stages (one leading radix-2/4 stage when log2 N is not a
// multiple of 3, then radix-8 stages) exchanged through LDS.
//
// Register convention: on entry thread t of a line holds v[s] = x[t + s*NT];
// on exit it holds v[s] = X[t + s*NT] (natural order).  The last radix-8
// stage already leaves its outputs at t + r*NT, so no final LDS round trip
// is made; callers that write LDS after fft_line must lds_barrier() first.
// DIR = -1: forward exp(-2πi jk/N); DIR = +1: inverse, unnormalised.
// Twiddles: one table load W_N^e per radix-8 butterfly, the other six powers
// by complex multiplication (≤ 3 roundings deep).  These transforms replace
// FF's rfftplan (CUFFT/FFTW) calls, SURVEY A2.
#pragma once
#include <hip/hip_runtime.h>

namespace sw {

// padded LDS index: one pad element every 8 complex (breaks the 128-B
// power-of-two strides of the early Stockham stores)
__device__ __forceinline__ int LP(int i) { return i + (i >> 3); }
__host__ __device__ constexpr int lds_line_elems(int N) { return N + N / 8; }

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
// multiply by i·s  (s real)
__device__ __forceinline__ double2 cmul_i(double2 a, double s) { return make_double2(-a.y * s, a.x * s); }

template <int DIR>
__device__ __forceinline__ void dft2(double2& a, double2& b) {
  double2 t = a;
  a = cadd(t, b);
  b = csub(t, b);
}

template <int DIR>
__device__ __forceinline__ void dft4(double2& x0, double2& x1, double2& x2, double2& x3) {
  double2 s0 = cadd(x0, x2), s1 = csub(x0, x2), s2 = cadd(x1, x3), d = csub(x1, x3);
  // d * W4, W4 = exp(DIR i π/2) = DIR·i
  double2 s3 = (DIR < 0) ? make_double2(d.y, -d.x) : make_double2(-d.y, d.x);
  x0 = cadd(s0, s2);
  x2 = csub(s0, s2);
  x1 = cadd(s1, s3);
  x3 = csub(s1, s3);
}

// in-place DFT-8 (natural order in, natural order out)
template <int DIR>
__device__ __forceinline__ void dft8(double2& v0, double2& v1, double2& v2, double2& v3,
                                     double2& v4, double2& v5, double2& v6, double2& v7) {
  const double c = 0.70710678118654752440084436210485;
  double2 a0 = cadd(v0, v4), a1 = cadd(v1, v5), a2 = cadd(v2, v6), a3 = cadd(v3, v7);
  double2 b0 = csub(v0, v4), b1 = csub(v1, v5), b2 = csub(v2, v6), b3 = csub(v3, v7);
  // b_r *= W8^r, W8 = c(1 + DIR i)
  b1 = make_double2(c * (b1.x - DIR * b1.y), c * (b1.y + DIR * b1.x));
  b2 = (DIR < 0) ? make_double2(b2.y, -b2.x) : make_double2(-b2.y, b2.x);
  b3 = make_double2(c * (-b3.x - DIR * b3.y), c * (-b3.y + DIR * b3.x));
  dft4<DIR>(a0, a1, a2, a3);
  dft4<DIR>(b0, b1, b2, b3);
  v0 = a0; v2 = a1; v4 = a2; v6 = a3;
  v1 = b0; v3 = b1; v5 = b2; v7 = b3;
}

__device__ __forceinline__ double2 twiddle(const double2* __restrict__ tw, int m, int dir) {
  double2 w = tw[m];
  return dir < 0 ? w : cconj(w);
}

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for
// every outstanding global load/store (vmcnt(0)), which would stall each FFT
// stage behind the previous pass's HBM stores; the LDS exchange needs only
// lgkmcnt(0) before the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void load_line(double2 (&v)[8], int t, int NT, const double2* __restrict__ line) {
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = line[LP(t + s * NT)];
}

// Leading radix-2 (lR = 1) or radix-4 (lR = 2) stage, Ns = 1 (no twiddles).
template <int DIR, int lR>
__device__ __forceinline__ void first_stage_small(double2 (&v)[8], int t, int NT,
                                                  double2* __restrict__ line) {
  constexpr int R = 1 << lR;
  constexpr int B = 8 / R;  // butterflies per thread
#pragma unroll
  for (int h = 0; h < B; ++h) {
    if constexpr (R == 4) {
      dft4<DIR>(v[h], v[h + B], v[h + 2 * B], v[h + 3 * B]);
    } else {
      dft2<DIR>(v[h], v[h + B]);
    }
  }
  lds_barrier();  // every thread has consumed the previous LDS contents
#pragma unroll
  for (int h = 0; h < B; ++h) {
    const int j = t + h * NT;  // Ns = 1: idxD = j*R
#pragma unroll
    for (int r = 0; r < R; ++r) line[LP(j * R + r)] = v[h + r * B];
  }
  lds_barrier();
}

// Radix-8 Stockham stage with sub-length Ns = 2^lNs (one butterfly per thread).
// last == true: outputs stay in registers (they land at t + r*NT).
template <int DIR>
__device__ __forceinline__ void radix8_stage(double2 (&v)[8], int t, int log2N, int lNs,
                                             const double2* __restrict__ tw,
                                             double2* __restrict__ line, bool last) {
  const int k = t & ((1 << lNs) - 1);
  if (lNs > 0) {
    const double2 w1 = twiddle(tw, k << (log2N - lNs - 3), DIR);
    const double2 w2 = cmul(w1, w1), w3 = cmul(w2, w1), w4 = cmul(w2, w2);
    const double2 w5 = cmul(w4, w1), w6 = cmul(w3, w3), w7 = cmul(w4, w3);
    v[1] = cmul(v[1], w1);
    v[2] = cmul(v[2], w2);
    v[3] = cmul(v[3], w3);
    v[4] = cmul(v[4], w4);
    v[5] = cmul(v[5], w5);
    v[6] = cmul(v[6], w6);
    v[7] = cmul(v[7], w7);
  }
  dft8<DIR>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
  if (last) return;
  lds_barrier();  // in-place LDS: everyone has loaded this stage's inputs
  const int idxD = ((t >> lNs) << (lNs + 3)) + k;
#pragma unroll
  for (int r = 0; r < 8; ++r) line[LP(idxD + (r << lNs))] = v[r];
  lds_barrier();
}

// Full transform.  v holds x[t + s*NT] on entry and X[t + s*NT] on exit.
// All threads of the block must call this (it contains barriers).
template <int DIR>
__device__ __forceinline__ void fft_line(double2 (&v)[8], int t, int NT, int log2N,
                                         const double2* __restrict__ tw, double2* __restrict__ line) {
  int lNs = 0;
  const int rem = log2N % 3;
  if (rem == 1) {
    first_stage_small<DIR, 1>(v, t, NT, line);
    lNs = 1;
    load_line(v, t, NT, line);
  } else if (rem == 2) {
    first_stage_small<DIR, 2>(v, t, NT, line);
    lNs = 2;
    load_line(v, t, NT, line);
  }
  while (true) {
    const bool last = lNs + 3 >= log2N;
    radix8_stage<DIR>(v, t, log2N, lNs, tw, line, last);
    if (last) break;
    lNs += 3;
    load_line(v, t, NT, line);
  }
}

}  // namespace sw
