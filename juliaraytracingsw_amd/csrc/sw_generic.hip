// libsw generic engine (sw_generic.hpp): MultiLayerQG + FilteredRK4 on grids
// of 2^a·3^b·5^c points per side (simulation/MattParameters.jl:8, nx = 384).
#include "sw.h"
#include "sw_generic.hpp"
#include "sw_fft.hpp"

#include <cmath>
#include <cstdlib>
#include <string>

namespace sw {
namespace gen {

__device__ __forceinline__ double2 zero2() { return make_double2(0.0, 0.0); }

int radices(int n, int rad[24]) {
  if (n < 16 || n > 4096 || (n & 1)) return 0;
  int k = 0;
  while (n % 4 == 0 && k < 24) rad[k++] = 4, n /= 4;
  while (n % 2 == 0 && k < 24) rad[k++] = 2, n /= 2;
  while (n % 3 == 0 && k < 24) rad[k++] = 3, n /= 3;
  while (n % 5 == 0 && k < 24) rad[k++] = 5, n /= 5;
  return n == 1 ? k : 0;
}

// the radix sequence of a line, passed by value to the kernels
struct Rad {
  int n, nr;
  int r[24];
};

// exp(-2πi j/n), j < n: the forward twiddle table of one line length
// (exact argument reduction: sincospi of 2j/n); the inverse uses conj
__global__ void k_twiddles(double2* __restrict__ tw, int n) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double sn, cs;
  sincospi(2.0 * (double)j / (double)n, &sn, &cs);
  tw[j] = make_double2(cs, -sn);
}

__device__ __forceinline__ double2 cadd2(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub2(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul2(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// i·DIR·a
template <int DIR>
__device__ __forceinline__ double2 rot(double2 a) { return DIR > 0 ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x); }

// the r-point DFT of v in place, sign DIR: exact ±1/±i for r = 2, 4; the
// radix-3/5 constants cos/sin(2π/3), cos/sin(2π/5), cos/sin(4π/5)
template <int DIR>
__device__ __forceinline__ void dft_small(int r, double2 (&v)[5]) {
  if (r == 4) {
    const double2 a = cadd2(v[0], v[2]), b = csub2(v[0], v[2]), c = cadd2(v[1], v[3]), d = rot<DIR>(csub2(v[1], v[3]));
    v[0] = cadd2(a, c);
    v[2] = csub2(a, c);
    v[1] = cadd2(b, d);
    v[3] = csub2(b, d);
  } else if (r == 2) {
    const double2 a = v[0];
    v[0] = cadd2(a, v[1]);
    v[1] = csub2(a, v[1]);
  } else if (r == 3) {
    constexpr double S3 = 0.86602540378443864676;  // sin(2π/3)
    const double2 s = cadd2(v[1], v[2]), d = csub2(v[1], v[2]);
    const double2 t = make_double2(v[0].x - 0.5 * s.x, v[0].y - 0.5 * s.y);
    const double2 e = rot<DIR>(make_double2(S3 * d.x, S3 * d.y));
    v[0] = cadd2(v[0], s);
    v[1] = cadd2(t, e);
    v[2] = csub2(t, e);
  } else {  // r == 5
    constexpr double C1 = 0.30901699437494742410, C2 = -0.80901699437494742410;  // cos(2π/5), cos(4π/5)
    constexpr double S1 = 0.95105651629515357212, S2 = 0.58778525229247312917;   // sin(2π/5), sin(4π/5)
    const double2 s1 = cadd2(v[1], v[4]), d1 = csub2(v[1], v[4]), s2 = cadd2(v[2], v[3]), d2 = csub2(v[2], v[3]);
    const double2 a1 = make_double2(v[0].x + C1 * s1.x + C2 * s2.x, v[0].y + C1 * s1.y + C2 * s2.y);
    const double2 a2 = make_double2(v[0].x + C2 * s1.x + C1 * s2.x, v[0].y + C2 * s1.y + C1 * s2.y);
    const double2 b1 = rot<DIR>(make_double2(S1 * d1.x + S2 * d2.x, S1 * d1.y + S2 * d2.y));
    const double2 b2 = rot<DIR>(make_double2(S2 * d1.x - S1 * d2.x, S2 * d1.y - S1 * d2.y));
    v[0] = cadd2(v[0], cadd2(s1, s2));
    v[1] = cadd2(a1, b1);
    v[4] = csub2(a1, b1);
    v[2] = cadd2(a2, b2);
    v[3] = csub2(a2, b2);
  }
}

// B lines of n points in LDS (line b at x + b n, ping-pong partner y),
// transformed in place by the block: mixed-radix Stockham, DIF form (the
// r-point DFT over the points p + t m, then the twiddle ω_len^(p u)):
//   y[q + s (r p + u)] = ω_len^(p u) Σ_t x[q + s (p + t m)] ω_r^(t u)
// with len the current sub-transform length (n, n/r₀, …), m = len/r, s the
// stride (1, r₀, …); ω_len^(p u) = tw[p u n/len] (p u < len).  Natural order
// in and out; returns the buffer holding the result.  DIR = -1 forward
// (unnormalised), +1 inverse.
// one r-point butterfly (p, q) of a stage (len = r m, stride s)
template <int DIR>
__device__ __forceinline__ void bfly(const double2* __restrict__ xb, double2* __restrict__ yb, int r, int m, int s,
                                     int step, int p, int q, const double2* __restrict__ tw) {
  double2 v[5];
#pragma unroll
  for (int t = 0; t < 5; ++t)
    if (t < r) v[t] = xb[q + s * (p + t * m)];
  dft_small<DIR>(r, v);
  yb[q + s * r * p] = v[0];
#pragma unroll
  for (int u = 1; u < 5; ++u)
    if (u < r) {
      double2 w = tw[p * u * step];
      if (DIR > 0) w.y = -w.y;
      yb[q + s * (r * p + u)] = cmul2(v[u], w);
    }
}

template <int DIR>
__device__ double2* fft_lds(double2* x, double2* y, const Rad& R, int B, const double2* __restrict__ tw) {
  const int n = R.n;
  int len = n, s = 1;
  for (int pi = 0; pi < R.nr; ++pi) {
    const int r = R.r[pi], m = len / r, nb = m * s, step = n / len;
    for (int idx = threadIdx.x; idx < B * nb; idx += blockDim.x) {
      const int b = idx / nb, i = idx - b * nb, p = i / s, q = i - p * s;
      bfly<DIR>(x + b * n, y + b * n, r, m, s, step, p, q, tw);
    }
    __syncthreads();
    double2* t = x;
    x = y;
    y = t;
    len = m;
    s *= r;
  }
  return x;
}

// ---- compile-time lines (round 6): the same stages for a line length N, B
// lines and NTH threads known at compile time — the radix, the index
// divisions and the thread loops fold (the runtime form spends more VALU on
// its index divisions than on the butterflies); the same butterflies in the
// same order, so bitwise the runtime form's results.
constexpr int ct_nrad(int n) {
  int k = 0;
  while (n % 4 == 0) ++k, n /= 4;
  while (n % 2 == 0) ++k, n /= 2;
  while (n % 3 == 0) ++k, n /= 3;
  while (n % 5 == 0) ++k, n /= 5;
  return k;
}
constexpr int ct_rad(int n, int pi) {  // radices()'s pi-th radix
  int k = 0;
  while (n % 4 == 0) { if (k++ == pi) return 4; n /= 4; }
  while (n % 2 == 0) { if (k++ == pi) return 2; n /= 2; }
  while (n % 3 == 0) { if (k++ == pi) return 3; n /= 3; }
  while (n % 5 == 0) { if (k++ == pi) return 5; n /= 5; }
  return 0;
}
// lines per block / threads per block (host and device: the launch and the kernel agree)
constexpr int ct_lines_per_block(int n) {
  int B = 1;
  while (B < 8 && 2 * B * n <= 2048) B *= 2;
  return B;
}
constexpr int ct_blk_threads(int lines, int n) {
  const int t = (lines * n / 2 + 63) / 64 * 64;
  return t < 64 ? 64 : (t > 1024 ? 1024 : t);
}

// f(idx) for idx < TOT over the block's NTH threads (TOT > 0: unrolled,
// constant trip count), else for idx < tot over blockDim.x threads
template <int TOT, int NTH, typename F>
__device__ __forceinline__ void gfor(int tot, F f) {
  if constexpr (TOT > 0) {
#pragma unroll
    for (int i0 = 0; i0 < TOT; i0 += NTH) {
      const int idx = i0 + (int)threadIdx.x;
      if (TOT % NTH == 0 || idx < TOT) f(idx);
    }
  } else {
    for (int idx = threadIdx.x; idx < tot; idx += blockDim.x) f(idx);
  }
}

template <int DIR, int N, int B, int NTH, int PI = 0, int LEN = N, int S = 1>
__device__ __forceinline__ double2* fft_ct(double2* x, double2* y, const double2* __restrict__ tw) {
  if constexpr (PI == ct_nrad(N)) {
    return x;
  } else {
    constexpr int r = ct_rad(N, PI), m = LEN / r, nb = m * S, step = N / LEN;
    gfor<B * nb, NTH>(0, [&](int idx) {
      const unsigned u = (unsigned)idx;
      const int b = (int)(u / nb), i = idx - b * nb, p = (int)((unsigned)i / S), q = i - p * S;
      bfly<DIR>(x + b * N, y + b * N, r, m, S, step, p, q, tw);
    });
    __syncthreads();
    return fft_ct<DIR, N, B, NTH, PI + 1, m, S * r>(y, x, tw);
  }
}

// N > 0: the compile-time stages; else the runtime ones
template <int DIR, int N, int B, int NTH>
__device__ __forceinline__ double2* fft_any(double2* x, double2* y, const Rad& R, int Br,
                                            const double2* __restrict__ tw) {
  if constexpr (N > 0) return fft_ct<DIR, N, B, NTH>(x, y, tw);
  else return fft_lds<DIR>(x, y, R, Br, tw);
}

// complex lines of R.n points, B per block (adjacent kr: one row of B points
// per load): element e of line kr of field f at data[f·fstride + kr + e·es]
template <int DIR>
__global__ void __launch_bounds__(1024) k_lines(double2* __restrict__ data, Rad R, int B, int nkr, long long fstride,
                                               long long es, const double2* __restrict__ tw) {
  extern __shared__ double2 lds[];
  const int n = R.n, groups = (nkr + B - 1) / B;
  double2 *twl = lds, *x = lds + n, *y = x + B * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) twl[j] = tw[j];
  const int f = blockIdx.x / groups, kr0 = (blockIdx.x - f * groups) * B;
  const int nv = min(B, nkr - kr0);
  double2* d = data + f * fstride + kr0;
  for (int idx = threadIdx.x; idx < B * n; idx += blockDim.x) {
    const int e = idx / B, b = idx - e * B;
    x[b * n + e] = b < nv ? d[e * es + b] : zero2();
  }
  __syncthreads();
  const double2* z = fft_lds<DIR>(x, y, R, B, twl);
  for (int idx = threadIdx.x; idx < B * n; idx += blockDim.x) {
    const int e = idx / B, b = idx - e * B;
    if (b < nv) d[e * es + b] = z[b * n + e];
  }
}

// c2r along x of B stored rows (FF's irfft rule: c2c along l done, then c2r
// along x with the DC and Nyquist bins' imaginary parts dropped, numpy's
// convention): spec rows [nkr] -> phys rows [nx] × scale
__global__ void __launch_bounds__(1024) k_c2r_rows(const double2* __restrict__ spec, double* __restrict__ phys, Rad R,
                                                  int B, int nkr, double scale, const double2* __restrict__ tw) {
  extern __shared__ double2 lds[];
  const int n = R.n;
  double2 *twl = lds, *x = lds + n, *y = x + B * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) twl[j] = tw[j];
  const long long row0 = (long long)blockIdx.x * B;
  const double2* a = spec + row0 * nkr;
  for (int idx = threadIdx.x; idx < B * n; idx += blockDim.x) {
    const int b = idx / n, k = idx - b * n;
    double2 z;
    if (k <= n / 2) {
      z = a[b * nkr + k];
      if (k == 0 || k == n / 2) z.y = 0.0;
    } else {
      const double2 c = a[b * nkr + n - k];
      z = make_double2(c.x, -c.y);
    }
    x[idx] = z;
  }
  __syncthreads();
  const double2* z = fft_lds<+1>(x, y, R, B, twl);
  double* o = phys + row0 * n;
  for (int idx = threadIdx.x; idx < B * n; idx += blockDim.x) o[idx] = z[idx].x * scale;
}

// r2c along x of B rows: phys rows [nx] -> spec rows [nkr] (unnormalised)
__global__ void __launch_bounds__(1024) k_r2c_rows(const double* __restrict__ phys, double2* __restrict__ spec, Rad R,
                                                  int B, int nkr, const double2* __restrict__ tw) {
  extern __shared__ double2 lds[];
  const int n = R.n;
  double2 *twl = lds, *x = lds + n, *y = x + B * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) twl[j] = tw[j];
  const long long row0 = (long long)blockIdx.x * B;
  const double* a = phys + row0 * n;
  for (int idx = threadIdx.x; idx < B * n; idx += blockDim.x) x[idx] = make_double2(a[idx], 0.0);
  __syncthreads();
  const double2* z = fft_lds<-1>(x, y, R, B, twl);
  double2* o = spec + row0 * nkr;
  for (int idx = threadIdx.x; idx < B * nkr; idx += blockDim.x) {
    const int b = idx / nkr, k = idx - b * nkr;
    o[idx] = z[b * n + k];
  }
}

// mode (l, kr) of a full [nl][nkr] field: live under FF's dealias!
__device__ __forceinline__ bool live_mode(const Geom& g, int l, int kr) { return kr < g.kc && (l < g.lc || l >= g.lr2); }

// per mode of X (dealiased on the fly): the 6 spectral fields the products
// need — per layer j: q̂_j, û_j = -il ψ̂_j, v̂_j = ik ψ̂_j (ψ̂ = S⁻¹ q̂,
// streamfunctionfrompv!) — at spec[3 j + {0, 1, 2}]
__global__ void k_prep(Geom g, Phys p, const double2* __restrict__ X, double2* __restrict__ spec) {
  const long long F = (long long)g.nl * g.nkr;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const int l = (int)(i / g.nkr), kr = (int)(i - (long long)l * g.nkr);
  const bool live = live_mode(g, l, kr);
  const double2 q1 = live ? X[i] : zero2(), q2 = live ? X[F + i] : zero2();
  const double k = kr * g.mk, ll = lwav(g, l), K2 = k * k + ll * ll;
  for (int j = 0; j < 2; ++j) {
    double2 ps;
    qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, j, ps.x, ps.y);
    spec[(3 * j) * F + i] = j ? q2 : q1;
    spec[(3 * j + 1) * F + i] = cmul_i(ps, -ll);
    spec[(3 * j + 2) * F + i] = cmul_i(ps, k);
  }
}

// physical products per point: per layer j, (U_j + u_j) q_j and v_j q_j into
// phys[2 j], phys[2 j + 1] (the inputs q_j, u_j, v_j at phys[3 j + {0,1,2}]
// are read first: the outputs overwrite fields 0-3)
__global__ void k_products(Phys p, double* __restrict__ phys, long long np) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  double q[2], u[2], v[2];
  for (int j = 0; j < 2; ++j) {
    q[j] = phys[(3 * j) * np + i];
    u[j] = phys[(3 * j + 1) * np + i];
    v[j] = phys[(3 * j + 2) * np + i];
  }
  for (int j = 0; j < 2; ++j) {
    const double U = j ? p.U2 : p.U1;
    phys[(2 * j) * np + i] = (u[j] + U) * q[j];
    phys[(2 * j + 1) * np + i] = v[j] * q[j];
  }
}

// N_j = -ik Â_j - il B̂_j - Qy_j ik ψ̂_j (+ μ K² ψ̂₂ on the lower layer) on the
// live modes, 0 on the aliased ones: GF's calcN_advection! + bottom drag
// (oracle mlqg_calcN: -rfft(v Qy) is Qy·ik ψ̂ up to the transforms' roundoff)
__global__ void k_assemble(Geom g, Phys p, const double2* __restrict__ X, const double2* __restrict__ spec,
                           double2* __restrict__ N) {
  const long long F = (long long)g.nl * g.nkr;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const int l = (int)(i / g.nkr), kr = (int)(i - (long long)l * g.nkr);
  if (!live_mode(g, l, kr)) {
    N[i] = N[F + i] = zero2();
    return;
  }
  const double k = kr * g.mk, ll = lwav(g, l), K2 = k * k + ll * ll;
  const double2 q1 = X[i], q2 = X[F + i];
  for (int j = 0; j < 2; ++j) {
    double2 ps;
    qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, j, ps.x, ps.y);
    const double Qy = j ? p.Qy2 : p.Qy1;
    double2 r = cscale(cmul_i(ps, k), -Qy);
    r = csub(r, cadd(cmul_i(spec[(2 * j) * F + i], k), cmul_i(spec[(2 * j + 1) * F + i], ll)));
    if (j == 1) r = cadd(r, cscale(ps, p.mu * K2));
    N[j * F + i] = r;
  }
}

// FF FilteredRK4 stage `stage` per mode (op_frk4's arithmetic, L = -ν K^(2nν)):
//   RHS = N + L x;  1: acc = RHS/6, x' = sol + dt/2 RHS;  2: acc += RHS/3,
//   x' = sol + dt/2 RHS;  3: acc += RHS/3, x' = sol + dt RHS;
//   4: sol = (sol + dt (acc + RHS/6)) · filter
// one field of one live mode (o = f·F + i): X the stage input, writes acc
// and the next stage input xo (stages 1-3) or the new state (stage 4);
// returns the stored new state at stage 4 (for the NaN check)
__device__ __forceinline__ double2 frk4_mode(const Geom& g, const Phys& p, int stage, long long o, double k, double ll,
                                             double D, double2 Xv, const double2 nv, double2* __restrict__ sol,
                                             double2* __restrict__ xo, double2* __restrict__ acc) {
#pragma clang fp contract(off)
  const double dt = p.dt;
  const cplx X = cx(Xv.x, Xv.y);
  const cplx u = cx(sol[o].x, sol[o].y);
  const cplx rhs = cx(nv.x + D * X.re, nv.y + D * X.im);
  if (stage < 4) {
    const double h = stage == 3 ? dt : dt / 2;
    const cplx r = stage == 1 ? cx(rhs.re / 6, rhs.im / 6) : cx(rhs.re / 3, rhs.im / 3);
    const cplx a = stage == 1 ? r : cx(acc[o].x + r.re, acc[o].y + r.im);
    acc[o] = make_double2(a.re, a.im);
    xo[o] = make_double2(u.re + h * rhs.re, u.im + h * rhs.im);
    return zero2();
  }
  const double filt = filter_value(g, p, k, ll);
  const cplx s6 = cx(acc[o].x + rhs.re / 6, acc[o].y + rhs.im / 6);
  const cplx r = cx(u.re + dt * s6.re, u.im + dt * s6.im);
  const double2 v = make_double2(r.re * filt, r.im * filt);
  sol[o] = v;
  return v;
}

__device__ __forceinline__ void note_bad(int* nanflag, bool bad) {
  if (!nanflag) return;
  const unsigned long long m = __ballot(bad);
  if (m != 0ull && (int)__lane_id() == __ffsll((long long)m) - 1)
    __hip_atomic_store(nanflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// FF FilteredRK4 stage `stage` per mode (op_frk4's arithmetic, L = -ν K^(2nν)):
//   RHS = N + L x;  1: acc = RHS/6, x' = sol + dt/2 RHS;  2: acc += RHS/3,
//   x' = sol + dt/2 RHS;  3: acc += RHS/3, x' = sol + dt RHS;
//   4: sol = (sol + dt (acc + RHS/6)) · filter
__global__ void k_frk4(Geom g, Phys p, int stage, double2* __restrict__ sol, double2* __restrict__ xs,
                       double2* __restrict__ acc, const double2* __restrict__ N, int* nanflag) {
  const long long F = (long long)g.nl * g.nkr;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (i < F) {
    const int l = (int)(i / g.nkr), kr = (int)(i - (long long)l * g.nkr);
    if (live_mode(g, l, kr)) {
      const double k = kr * g.mk, ll = lwav(g, l);
      const double D = -(p.nu * ipow(k * k + ll * ll, p.nnu));
      for (int f = 0; f < 2; ++f) {
        const long long o = f * F + i;
        const double2 X = stage == 1 ? sol[o] : xs[o];
        const double2 r = frk4_mode(g, p, stage, o, k, ll, D, X, N[o], sol, xs, acc);
        bad = bad || !isfinite(r.x) || !isfinite(r.y);
      }
    }
  }
  note_bad(nanflag, bad);
}

// ---------------------------------------------------------------- fused step
// Three kernels per FilteredRK4 stage (Engine::fused), the power-of-two
// engine's col_inv / row / col_step split on the generic transforms:
//   k_gcol_inv   one spectral field (q_j, u_j, v_j of X, dealiased) per block,
//                formed on load, inverse transform along l;
//   k_grow       one row: the six fields' c2r as three complex lines
//                (q₁ + iu₁, v₁ + iq₂, u₂ + iv₂), the products, their r2c as
//                two complex lines ((U₁+u₁)q₁ + i v₁q₁, (U₂+u₂)q₂ + i v₂q₂)
//                split by Hermitian symmetry;
//   k_gcol_fwd   one layer per block: forward transforms of its two product
//                fields along l, N_j (k_assemble's arithmetic) and the stage
//                update (frk4_mode) per live mode.
// X is read by both layers' blocks, so stages write the next input to the
// other xs buffer (ping-pong).
// (kernel templates: NC > 0 the compile-time line length, BC lines per block,
// NTH threads — launched with exactly those; NC = 0 the runtime form)
template <int NC, int BC, int NTH>
__global__ void __launch_bounds__(NTH > 0 ? NTH : 1024) k_gcol_inv(Geom g, Phys p, const double2* __restrict__ X,
                                                                  double2* __restrict__ spec, Rad R, int Bp,
                                                                  const double2* __restrict__ tw) {
  extern __shared__ double2 lds[];
  const int n = NC > 0 ? NC : R.n, B = NC > 0 ? BC : Bp, groups = (g.nkr + B - 1) / B;
  double2 *twl = lds, *x = lds + n, *y = x + B * n;
  gfor<NC, NTH>(n, [&](int j) { twl[j] = tw[j]; });
  const int fid = blockIdx.x / groups, kr0 = (blockIdx.x - fid * groups) * B;
  const int layer = fid / 3, comp = fid - 3 * layer;
  const long long F = (long long)g.nl * g.nkr;
  gfor<NC * BC, NTH>(B * n, [&](int idx) {
    const int l = (int)((unsigned)idx / B), b = idx - l * B, kr = kr0 + b;
    double2 v = zero2();
    if (kr < g.nkr && live_mode(g, l, kr)) {
      const long long i = (long long)l * g.nkr + kr;
      const double2 q1 = X[i], q2 = X[F + i];
      if (comp == 0) {
        v = layer ? q2 : q1;
      } else {
        const double k = kr * g.mk, ll = lwav(g, l), K2 = k * k + ll * ll;
        double2 ps;
        qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, layer, ps.x, ps.y);
        v = comp == 1 ? cmul_i(ps, -ll) : cmul_i(ps, k);
      }
    }
    x[b * n + l] = v;
  });
  __syncthreads();
  const double2* z = fft_any<+1, NC, BC, NTH>(x, y, R, B, twl);
  double2* d = spec + fid * F + kr0;
  const int nv = min(B, g.nkr - kr0);
  gfor<NC * BC, NTH>(B * n, [&](int idx) {
    const int l = (int)((unsigned)idx / B), b = idx - l * B;
    if (b < nv) d[(long long)l * g.nkr + b] = z[b * n + l];
  });
}

// c2r of two Hermitian half rows A, B (FF/numpy's rule: the DC and Nyquist
// bins' imaginary parts dropped) as one complex line: Z_k = A_k + i B_k over
// the full length, IFFT(Z) = a + i b
__device__ __forceinline__ double2 pack_c2r(const double2* __restrict__ A, const double2* __restrict__ Bv, int k,
                                            int n) {
  if (k <= n / 2) {
    double2 a = A[k], b = Bv[k];
    if (k == 0 || k == n / 2) a.y = b.y = 0.0;
    return make_double2(a.x - b.y, a.y + b.x);
  }
  const double2 a = A[n - k], b = Bv[n - k];
  return make_double2(a.x + b.y, b.x - a.y);
}

template <int NC, int NTH>
__global__ void __launch_bounds__(NTH > 0 ? NTH : 1024) k_grow(Geom g, Phys p, double2* __restrict__ spec, Rad R,
                                                              double scale, const double2* __restrict__ tw) {
  extern __shared__ double2 lds[];
  const int n = NC > 0 ? NC : R.n, row = blockIdx.x;
  const int nkr = NC > 0 ? NC / 2 + 1 : g.nkr;  // (the x transforms: nkr = nx/2 + 1)
  const long long F = (long long)g.nl * nkr;
  double2 *twl = lds, *x = lds + n, *y = x + 3 * n;
  gfor<NC, NTH>(n, [&](int j) { twl[j] = tw[j]; });
  const double2* S = spec + (long long)row * nkr;
  gfor<3 * NC, NTH>(3 * n, [&](int idx) {
    const int c = (int)((unsigned)idx / n), k = idx - c * n;  // lines: (q1, u1), (v1, q2), (u2, v2) = fields (0,1), (2,3), (4,5)
    x[idx] = pack_c2r(S + (2 * c) * F, S + (2 * c + 1) * F, k, n);
  });
  __syncthreads();
  double2* z = fft_any<+1, NC, 3, NTH>(x, y, R, 3, twl);
  double2* w = z == x ? y : x;  // the free buffer
  gfor<NC, NTH>(n, [&](int k) {
    const double2 a = z[k], b = z[n + k], c = z[2 * n + k];
    const double q1 = a.x * scale, u1 = a.y * scale, v1 = b.x * scale, q2 = b.y * scale;
    const double u2 = c.x * scale, v2 = c.y * scale;
    w[k] = make_double2((u1 + p.U1) * q1, v1 * q1);
    w[n + k] = make_double2((u2 + p.U2) * q2, v2 * q2);
  });
  __syncthreads();
  const double2* Z = fft_any<-1, NC, 2, NTH>(w, z, R, 2, twl);
  double2* O = spec + (long long)row * nkr;
  gfor<2 * (NC / 2 + 1) * (NC > 0), NTH>(2 * nkr, [&](int idx) {
    const int c = (int)((unsigned)idx / nkr), k = idx - c * nkr;
    const double2 zk = Z[c * n + k], zm = Z[c * n + (k == 0 ? 0 : n - k)];
    // P = (Z_k + conj Z_{n-k})/2, Q = (Z_k - conj Z_{n-k})/(2i)
    O[(2 * c) * F + k] = make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
    O[(2 * c + 1) * F + k] = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));
  });
}

template <int NC, int BC, int NTH>
__global__ void __launch_bounds__(NTH > 0 ? NTH : 1024)
    k_gcol_fwd(Geom g, Phys p, int stage, const double2* X,  // (= sol at stage 1)
               const double2* __restrict__ spec, double2* __restrict__ sol, double2* __restrict__ xo,
               double2* __restrict__ acc, Rad R, int Bp, const double2* __restrict__ tw, int* nanflag) {
  extern __shared__ double2 lds[];
  const int n = NC > 0 ? NC : R.n, B = NC > 0 ? BC : Bp, groups = (g.nkr + B - 1) / B;
  double2 *twl = lds, *x = lds + n, *y = x + 2 * B * n;
  gfor<NC, NTH>(n, [&](int j) { twl[j] = tw[j]; });
  const int j = blockIdx.x / groups, kr0 = (blockIdx.x - j * groups) * B;
  const long long F = (long long)g.nl * g.nkr;
  const int nv = min(B, g.nkr - kr0);
  // lines 2b: (U_j + u_j) q_j, 2b + 1: v_j q_j of column kr0 + b
  gfor<2 * BC * NC, NTH>(2 * B * n, [&](int idx) {
    const int l = (int)((unsigned)idx / (2 * B)), r = idx - l * (2 * B), b = r >> 1, c = r & 1;
    x[r * n + l] = b < nv ? spec[(2 * j + c) * F + (long long)l * g.nkr + kr0 + b] : zero2();
  });
  __syncthreads();
  const double2* z = fft_any<-1, NC, 2 * BC, NTH>(x, y, R, 2 * B, twl);
  bool bad = false;
  gfor<BC * NC, NTH>(B * n, [&](int idx) {
    const int l = (int)((unsigned)idx / B), b = idx - l * B, kr = kr0 + b;
    if (b >= nv || !live_mode(g, l, kr)) return;
    const long long i = (long long)l * g.nkr + kr, o = j * F + i;
    const double k = kr * g.mk, ll = lwav(g, l), K2 = k * k + ll * ll;
    const double2 q1 = X[i], q2 = X[F + i];
    double2 ps;
    qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, j, ps.x, ps.y);
    const double Qy = j ? p.Qy2 : p.Qy1;
    double2 r = cscale(cmul_i(ps, k), -Qy);
    r = csub(r, cadd(cmul_i(z[(2 * b) * n + l], k), cmul_i(z[(2 * b + 1) * n + l], ll)));
    if (j == 1) r = cadd(r, cscale(ps, p.mu * K2));
    const double D = -(p.nu * ipow(K2, p.nnu));
    const double2 v = frk4_mode(g, p, stage, o, k, ll, D, j ? q2 : q1, r, sol, xo, acc);
    bad = bad || !isfinite(v.x) || !isfinite(v.y);
  });
  if (stage == 4) note_bad(nanflag, bad);
}

__global__ void k_dealias(Geom g, double2* __restrict__ X) {
  const long long F = (long long)g.nl * g.nkr;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const int l = (int)(i / g.nkr), kr = (int)(i - (long long)l * g.nkr);
  if (!live_mode(g, l, kr)) X[i] = X[F + i] = zero2();
}

// updatevars! spectral field (k_make_spec's MultiLayerQG branch on the full array)
__global__ void k_spec_field(Geom g, Phys p, int fid, const double2* __restrict__ X, double2* __restrict__ out) {
  const long long F = (long long)g.nl * g.nkr;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= F) return;
  const int l = (int)(i / g.nkr), kr = (int)(i - (long long)l * g.nkr);
  double2 r = zero2();
  if (live_mode(g, l, kr)) {
    const int layer = fid >> 3, id = fid & 7;
    const double2 q1 = X[i], q2 = X[F + i];
    if (id == 4) {
      r = layer ? q2 : q1;
    } else {
      const double k = kr * g.mk, ll = lwav(g, l), K2 = k * k + ll * ll;
      double2 ps;
      qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, layer, ps.x, ps.y);
      if (id == 5) r = ps;
      else if (id == 3) r = make_double2(-K2 * ps.x, -K2 * ps.y);
      else if (id == 0) r = cmul_i(ps, -ll);
      else if (id == 1) r = cmul_i(ps, k);
    }
  }
  out[i] = r;
}

// MultiLayerQG.energies' Parseval sums per kr column (fixed order, one block
// per column): K²|ψ̂₁|², K²|ψ̂₂|², |ψ̂₂ - ψ̂₁|² over the live modes
__global__ void __launch_bounds__(256) k_energy_cols(Geom g, Phys p, const double2* __restrict__ X,
                                                     double* __restrict__ cols) {
  __shared__ double red[3][256];
  const long long F = (long long)g.nl * g.nkr;
  const int kr = blockIdx.x;
  double a[3] = {0.0, 0.0, 0.0};
  for (int l = threadIdx.x; l < g.nl; l += blockDim.x) {
    if (!live_mode(g, l, kr)) continue;
    const long long i = (long long)l * g.nkr + kr;
    const double k = kr * g.mk, ll = lwav(g, l), K2 = k * k + ll * ll;
    const double2 q1 = X[i], q2 = X[F + i];
    double2 p1, p2;
    qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, 0, p1.x, p1.y);
    qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, 1, p2.x, p2.y);
    a[0] += K2 * (p1.x * p1.x + p1.y * p1.y);
    a[1] += K2 * (p2.x * p2.x + p2.y * p2.y);
    const double dr = p2.x - p1.x, di = p2.y - p1.y;
    a[2] += dr * dr + di * di;
  }
  for (int c = 0; c < 3; ++c) red[c][threadIdx.x] = a[c];
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int c = 0; c < 3; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) cols[kr * 3 + threadIdx.x] = red[threadIdx.x][0];
}

// FF parsevalsum weights (kr = 0 and the Nyquist column once, the others
// twice), columns added in order -> out[0..2]; out[3..SW_NSUM) = 0
__global__ void k_energy_final(Geom g, const double* __restrict__ cols, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s[3] = {0.0, 0.0, 0.0};
  for (int kr = 0; kr < g.nkr; ++kr) {
    const double w = (kr == 0 || kr == g.nx / 2) ? 1.0 : 2.0;
    for (int c = 0; c < 3; ++c) s[c] += w * cols[kr * 3 + c];
  }
  for (int c = 0; c < SW_NSUM; ++c) out[c] = c < 3 ? s[c] : 0.0;
}

__global__ void k_nan(long long n, const double* __restrict__ x, int* flag) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool bad = i < n && !isfinite(x[i]);
  const unsigned long long m = __ballot(bad);
  if (m != 0ull && (int)__lane_id() == __ffsll((long long)m) - 1)
    __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ----------------------------------------------------------------- host side
static Rad rad_of(const int* r, int nr, int n) {
  Rad R{};
  R.n = n;
  R.nr = nr;
  for (int i = 0; i < nr; ++i) R.r[i] = r[i];
  return R;
}
static dim3 modes_grid(const Geom& g) { return dim3((unsigned)(((long long)g.nl * g.nkr + 255) / 256)); }

static int lines_per_block(int n);

int create(Engine*& e, const sw_config& k, const Phys& p, const Geom& g, double2* sol, hipStream_t s,
           std::string& err) {
  e = new Engine();
  e->g = g;
  e->p = p;
  e->s = s;
  e->sol = sol;
  e->nradx = radices(k.nx, e->radx);
  e->nrady = radices(k.ny, e->rady);
  // one line and its ping-pong partner plus the twiddle table in 160 KB of LDS
  if (!e->nradx || !e->nrady || k.nx > 3328 || k.ny > 3328) {
    err = "generic grids: nx, ny even, 16 ... 3328, of the form 2^a 3^b 5^c";
    return SW_E_INVALID;
  }
  const size_t F = (size_t)g.nl * g.nkr, NP = (size_t)g.nx * g.ny;
  void** bufs[] = {(void**)&e->xs, (void**)&e->acc, (void**)&e->N};
  for (void** b : bufs)
    if (hipMalloc(b, 2 * F * sizeof(double2)) != hipSuccess) return SW_E_NOMEM;
  if (hipMalloc((void**)&e->spec, 6 * F * sizeof(double2)) != hipSuccess) return SW_E_NOMEM;
  if (hipMalloc((void**)&e->phys, 6 * NP * sizeof(double)) != hipSuccess) return SW_E_NOMEM;
  if (hipMalloc((void**)&e->cols, 3 * (size_t)g.nkr * sizeof(double)) != hipSuccess) return SW_E_NOMEM;
  for (double2* b : {e->xs, e->acc, e->N}) (void)hipMemsetAsync(b, 0, 2 * F * sizeof(double2), s);
  if (hipMalloc((void**)&e->twx, (size_t)g.nx * sizeof(double2)) != hipSuccess) return SW_E_NOMEM;
  if (hipMalloc((void**)&e->twy, (size_t)g.ny * sizeof(double2)) != hipSuccess) return SW_E_NOMEM;
  SW_LAUNCH(k_twiddles, dim3((g.nx + 255) / 256), dim3(256), 0, s, e->twx, g.nx);
  SW_LAUNCH(k_twiddles, dim3((g.ny + 255) / 256), dim3(256), 0, s, e->twy, g.ny);
  // rows per block: B·nx ≤ 2048 with B dividing ny (ny is even, B a power of two)
  e->bx = lines_per_block(g.nx);
  while (g.ny % e->bx) e->bx /= 2;
  // the fused stages (k_grow holds 3 complex lines of nx points twice: ≤ 96 KB
  // of LDS; k_gcol_fwd 2 lines of ny): nx, ny ≤ 1024; SW_GEN_FUSED=0 forces
  // the separate passes (tests run both)
  const char* fe = std::getenv("SW_GEN_FUSED");
  e->fused = g.nx <= 1024 && g.ny <= 1024 && !(fe && fe[0] == '0');
  const char* ce = std::getenv("SW_GEN_CT");
  e->ct = !(ce && ce[0] == '0');
  const char* ge = std::getenv("SW_GEN_GRAPH");
  e->graph_on = e->fused && ge && ge[0] == '1';
  if (e->fused && hipMalloc((void**)&e->xs2, 2 * F * sizeof(double2)) != hipSuccess) return SW_E_NOMEM;
  return SW_OK;
}

void destroy(Engine* e) {
  if (!e) return;
  if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
  for (void* b : {(void*)e->xs, (void*)e->xs2, (void*)e->acc, (void*)e->N, (void*)e->spec, (void*)e->phys,
                  (void*)e->cols, (void*)e->twx, (void*)e->twy})
    if (b) (void)hipFree(b);
  delete e;
}

// nf spectral fields [nf][nl][nkr] -> physical [nf][ny][nx] (normalised c2r;
// the spectral fields are transformed in place along l first)
// lines per block: B·n ≤ 2048 points (≤ 64 KB of LDS with the ping-pong buffer), at most 8
static int lines_per_block(int n) { return ct_lines_per_block(n); }

// threads of a transform block: one per butterfly of its widest (radix-2)
// stage over its lines, 64 … 1024 (small grids: the latency of each stage
// is spread over more waves)
static int blk_threads(int lines, int n) { return ct_blk_threads(lines, n); }

static void inverse2d(Engine* e, double2* spec, int nf, double* phys) {
  const Geom& g = e->g;
  const Rad Ry = rad_of(e->rady, e->nrady, g.ny), Rx = rad_of(e->radx, e->nradx, g.nx);
  const int By = lines_per_block(g.ny), Bx = e->bx;
  SW_LAUNCH(k_lines<+1>, dim3(nf * ((g.nkr + By - 1) / By)), dim3(blk_threads(By, g.ny)),
            (2 * By + 1) * g.ny * sizeof(double2), e->s, spec,
            Ry, By, g.nkr, (long long)g.nl * g.nkr, (long long)g.nkr, e->twy);
  SW_LAUNCH(k_c2r_rows, dim3(nf * g.ny / Bx), dim3(blk_threads(Bx, g.nx)), (2 * Bx + 1) * g.nx * sizeof(double2), e->s,
            spec, phys, Rx, Bx,
            g.nkr, 1.0 / ((double)g.nx * (double)g.ny), e->twx);
}

// physical [nf][ny][nx] -> spectral [nf][nl][nkr] (unnormalised r2c)
static void forward2d(Engine* e, const double* phys, int nf, double2* spec) {
  const Geom& g = e->g;
  const Rad Ry = rad_of(e->rady, e->nrady, g.ny), Rx = rad_of(e->radx, e->nradx, g.nx);
  const int By = lines_per_block(g.ny), Bx = e->bx;
  SW_LAUNCH(k_r2c_rows, dim3(nf * g.ny / Bx), dim3(blk_threads(Bx, g.nx)), (2 * Bx + 1) * g.nx * sizeof(double2), e->s,
            phys, spec, Rx, Bx,
            g.nkr, e->twx);
  SW_LAUNCH(k_lines<-1>, dim3(nf * ((g.nkr + By - 1) / By)), dim3(blk_threads(By, g.ny)),
            (2 * By + 1) * g.ny * sizeof(double2), e->s, spec,
            Ry, By, g.nkr, (long long)g.nl * g.nkr, (long long)g.nkr, e->twy);
}

void calcN(Engine* e, const double2* X, double2* N) {
  const Geom& g = e->g;
  const long long np = (long long)g.nx * g.ny;
  SW_LAUNCH(k_prep, modes_grid(g), dim3(256), 0, e->s, g, e->p, X, e->spec);
  inverse2d(e, e->spec, 6, e->phys);
  SW_LAUNCH(k_products, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, e->s, e->p, e->phys, np);
  forward2d(e, e->phys, 4, e->spec);
  SW_LAUNCH(k_assemble, modes_grid(g), dim3(256), 0, e->s, g, e->p, X, e->spec, N);
}

// the line lengths with compile-time fused kernels (the 3·2^k family of
// simulation/MattParameters.jl's nx = 384 and the test grids); other lengths
// run the runtime forms.  SW_GEN_CT=0: the runtime forms everywhere (A/B, tests)
#define SW_GEN_CT_LENGTHS(X) X(48) X(96) X(192) X(384) X(768)

template <int NY>
static void gcol_inv_ct(Engine* e, const double2* X, const Rad& Ry, int gi) {
  constexpr int B = ct_lines_per_block(NY), T = ct_blk_threads(B, NY);
  SW_LAUNCH((k_gcol_inv<NY, B, T>), dim3(6 * gi), dim3(T), (2 * B + 1) * NY * sizeof(double2), e->s, e->g, e->p, X,
            e->spec, Ry, B, e->twy);
}
template <int NX>
static void grow_ct(Engine* e, const Rad& Rx, double scale) {
  constexpr int T = ct_blk_threads(3, NX);
  SW_LAUNCH((k_grow<NX, T>), dim3(e->g.ny), dim3(T), 7 * NX * sizeof(double2), e->s, e->g, e->p, e->spec, Rx, scale,
            e->twx);
}
template <int NY>
static void gcol_fwd_ct(Engine* e, int stage, const double2* X, double2* xo, const Rad& Ry, int gf, int* nanflag) {
  constexpr int Bi = ct_lines_per_block(NY), B = Bi > 1 ? Bi / 2 : 1, T = ct_blk_threads(2 * B, NY);
  SW_LAUNCH((k_gcol_fwd<NY, B, T>), dim3(2 * gf), dim3(T), (4 * B + 1) * NY * sizeof(double2), e->s, e->g, e->p,
            stage, X, e->spec, e->sol, xo, e->acc, Ry, B, e->twy, nanflag);
}

// the fused stage sequence (k_gcol_inv, k_grow, k_gcol_fwd; Engine::fused)
static void step_fused(Engine* e, int* nanflag) {
  const Geom& g = e->g;
  const Rad Ry = rad_of(e->rady, e->nrady, g.ny), Rx = rad_of(e->radx, e->nradx, g.nx);
  const int Bi = lines_per_block(g.ny), Bf = Bi > 1 ? Bi / 2 : 1;
  const int gi = (g.nkr + Bi - 1) / Bi, gf = (g.nkr + Bf - 1) / Bf;
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  const double2* X = e->sol;
  for (int stage = 1; stage <= 4; ++stage) {
    // stage inputs: sol, xs, xs2, xs; the next input goes to the other buffer
    double2* xo = stage == 4 ? nullptr : (stage & 1 ? e->xs : e->xs2);
    int* nf = stage == 4 ? nanflag : nullptr;
    bool done = false;
#define SW_GEN_CASE(N) \
  case N:              \
    gcol_inv_ct<N>(e, X, Ry, gi); \
    done = true;       \
    break;
    if (e->ct) switch (g.ny) { SW_GEN_CT_LENGTHS(SW_GEN_CASE) default: break; }
#undef SW_GEN_CASE
    if (!done)
      SW_LAUNCH((k_gcol_inv<0, 0, 0>), dim3(6 * gi), dim3(blk_threads(Bi, g.ny)), (2 * Bi + 1) * g.ny * sizeof(double2),
                e->s, g, e->p, X, e->spec, Ry, Bi, e->twy);
    done = false;
#define SW_GEN_CASE(N)   \
  case N:                \
    grow_ct<N>(e, Rx, scale); \
    done = true;         \
    break;
    if (e->ct) switch (g.nx) { SW_GEN_CT_LENGTHS(SW_GEN_CASE) default: break; }
#undef SW_GEN_CASE
    if (!done)
      SW_LAUNCH((k_grow<0, 0>), dim3(g.ny), dim3(blk_threads(3, g.nx)), 7 * g.nx * sizeof(double2), e->s, g, e->p,
                e->spec, Rx, scale, e->twx);
    done = false;
#define SW_GEN_CASE(N)                              \
  case N:                                           \
    gcol_fwd_ct<N>(e, stage, X, xo, Ry, gf, nf); \
    done = true;                                    \
    break;
    if (e->ct) switch (g.ny) { SW_GEN_CT_LENGTHS(SW_GEN_CASE) default: break; }
#undef SW_GEN_CASE
    if (!done)
      SW_LAUNCH((k_gcol_fwd<0, 0, 0>), dim3(2 * gf), dim3(blk_threads(2 * Bf, g.ny)),
                (4 * Bf + 1) * g.ny * sizeof(double2), e->s, g, e->p, stage, X, e->spec, e->sol, xo, e->acc, Ry, Bf,
                e->twy, nf);
    X = xo;
  }
}

// The fused step as one hipGraph (round 6, SW_GEN_GRAPH=1): at 384² a step
// is twelve kernels of 9-13 µs and the gaps between them were 7 % of the step
// (trace span 135.9 against a kernel sum of 126.1 µs per step).  Every launch
// of the step has the same arguments each step (the stage buffers, the flag),
// so the step is captured once per flag pointer and replayed.  Measured
// slower (tools/ab/ab_env.sh, three rounds): 7919-7936 → 7592-7613 steps/s,
// TwoLayerSimulation's cadence at 384² 4717 → 3779: off (direct launches).
static bool graph_step(Engine* e, int* nanflag) {
  if (!e->graph_on || ::sw::prof_ev.stop) return false;
  if (!e->gexec || e->gflag != nanflag) {
    if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
    e->gexec = nullptr;
    hipGraph_t gr = nullptr;
    if (hipStreamBeginCapture(e->s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
      e->graph_on = false;
      return false;
    }
    step_fused(e, nanflag);
    const bool ok = hipStreamEndCapture(e->s, &gr) == hipSuccess && gr &&
                    hipGraphInstantiate(&e->gexec, gr, nullptr, nullptr, 0) == hipSuccess;
    if (gr) (void)hipGraphDestroy(gr);
    if (!ok) {  // (nothing was launched: the captured step runs directly)
      e->gexec = nullptr;
      e->graph_on = false;
      return false;
    }
    e->gflag = nanflag;
  }
  return hipGraphLaunch(e->gexec, e->s) == hipSuccess;
}

void step(Engine* e, int* nanflag) {
  const Geom& g = e->g;
  if (e->fused) {
    if (!graph_step(e, nanflag)) step_fused(e, nanflag);
    return;
  }
  for (int stage = 1; stage <= 4; ++stage) {
    calcN(e, stage == 1 ? e->sol : e->xs, e->N);
    SW_LAUNCH(k_frk4, modes_grid(g), dim3(256), 0, e->s, g, e->p, stage, e->sol, e->xs, e->acc, e->N,
                       stage == 4 ? nanflag : nullptr);
  }
}

void dealias(Engine* e, double2* X) { SW_LAUNCH(k_dealias, modes_grid(e->g), dim3(256), 0, e->s, e->g, X); }

void physical(Engine* e, const double2* X, int fid, double* out) {
  SW_LAUNCH(k_spec_field, modes_grid(e->g), dim3(256), 0, e->s, e->g, e->p, fid, X, e->spec);
  inverse2d(e, e->spec, 1, out);
}

void energy_sums(Engine* e, const double2* X, double* out) {
  SW_LAUNCH(k_energy_cols, dim3(e->g.nkr), dim3(256), 0, e->s, e->g, e->p, X, e->cols);
  SW_LAUNCH(k_energy_final, dim3(1), dim3(64), 0, e->s, e->g, e->cols, out);
}

void nan_scan(Engine* e, const double2* X, int* flag) {
  const long long n = 4LL * e->g.nl * e->g.nkr;  // 2 fields of complex doubles
  SW_LAUNCH(k_nan, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->s, n,
                     reinterpret_cast<const double*>(X), flag);
}

}  // namespace gen
}  // namespace sw
