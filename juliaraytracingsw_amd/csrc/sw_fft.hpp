// Device-side fp64 FFT primitive for gfx950: one power-of-two transform of
// length N per "line", NT = N/8 threads per line, 8 complex points per thread,
// Stockham autosort radix-8 stages (plus one radix-4/2 stage) exchanged
// through LDS.  Twiddles come from a per-length global table W_N^m, which is
// L1/L2 resident.
//
// Register convention: on entry thread t of a line holds v[s] = x[t + s*NT]
// (s = 0..7); on exit the transform sits in the line's LDS buffer in natural
// order (index via LP()).  DIR = -1: forward exp(-2πi jk/N); DIR = +1: inverse,
// unnormalised.  These transforms replace FF's rfftplan (CUFFT/FFTW) calls,
// SURVEY A2.
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

// in-place DFT-8 on v[0..7] (natural order in, natural order out)
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

// One Stockham stage of radix R = 2^lR (8, 4 or 2) with current sub-length
// Ns = 2^lNs.  v[] holds x[t + s*NT]; results are stored to LDS.
template <int DIR, int lR>
__device__ __forceinline__ void stockham_stage(double2 (&v)[8], int t, int NT, int log2N, int lNs,
                                               const double2* __restrict__ tw,
                                               double2* __restrict__ line) {
  constexpr int R = 1 << lR;
  constexpr int B = 8 / R;  // butterflies per thread
  const int Nsm1 = (1 << lNs) - 1;
  const int lts = log2N - lNs - lR;  // log2 of N/(Ns*R)
#pragma unroll
  for (int h = 0; h < B; ++h) {
    const int j = t + h * NT;
    const int k = j & Nsm1;
    double2 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = v[h + r * B];
    if (lNs > 0) {
#pragma unroll
      for (int r = 1; r < R; ++r) x[r] = cmul(x[r], twiddle(tw, (r * k) << lts, DIR));
    }
    if constexpr (R == 8) {
      dft8<DIR>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
    } else if constexpr (R == 4) {
      dft4<DIR>(x[0], x[1], x[2], x[3]);
    } else {
      dft2<DIR>(x[0], x[1]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) v[h + r * B] = x[r];
  }
  __syncthreads();  // every thread has consumed its inputs (in-place LDS)
#pragma unroll
  for (int h = 0; h < B; ++h) {
    const int j = t + h * NT;
    const int k = j & Nsm1;
    const int idxD = ((j >> lNs) << (lNs + lR)) + k;
#pragma unroll
    for (int r = 0; r < R; ++r) line[LP(idxD + (r << lNs))] = v[h + r * B];
  }
  __syncthreads();
}

__device__ __forceinline__ void load_line(double2 (&v)[8], int t, int NT, const double2* __restrict__ line) {
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = line[LP(t + s * NT)];
}

// Full transform.  v holds x[t + s*NT] on entry; result in `line` (natural order).
// All threads of the block must call this (it contains barriers).
template <int DIR>
__device__ __forceinline__ void fft_line(double2 (&v)[8], int t, int NT, int log2N,
                                         const double2* __restrict__ tw, double2* __restrict__ line) {
  int lNs = 0;
  const int rem = log2N % 3;
  if (rem == 1) {
    stockham_stage<DIR, 1>(v, t, NT, log2N, lNs, tw, line);
    lNs += 1;
    load_line(v, t, NT, line);
  } else if (rem == 2) {
    stockham_stage<DIR, 2>(v, t, NT, log2N, lNs, tw, line);
    lNs += 2;
    load_line(v, t, NT, line);
  }
  while (true) {
    stockham_stage<DIR, 3>(v, t, NT, log2N, lNs, tw, line);
    lNs += 3;
    if (lNs >= log2N) break;
    load_line(v, t, NT, line);
  }
}

}  // namespace sw
