// libsw device kernels for gfx950 (MI355X).  One pseudo-spectral step is
//   col_inv  (compact spectral state -> y-inverse columns, "mixed" space)
//   row      (x c2r of every field, physical products, x r2c; physical space
//             never touches HBM)
//   col_fwd  (y-forward columns -> N on live modes)
//   update   (stepper combination over live modes)
// See DESIGN.md for layouts, the roofline of each kernel and the reference
// lines each one replaces.
#include "sw_internal.hpp"
#include "sw_fft.hpp"

namespace sw {

// block -> column mapping for the column kernels.  When one line per block and
// the grid is a multiple of 64, the 8 columns that share each 128-B chunk of
// the mixed layout (kr>>3 equal) are placed on blocks b, b+8, …, b+56, which
// the dispatcher deals to one XCD, so they meet in one L2 (speed only).
__device__ __forceinline__ int col_of_block(int b, int nb) {
  if ((nb & 63) == 0) {
    const int q = b >> 6, j = (b >> 3) & 7, x = b & 7;
    return (q << 6) + (x << 3) + j;
  }
  return b;
}

// minimum waves per SIMD requested from the register allocator
#ifndef SW_MINW_FFT
#define SW_MINW_FFT 2
#endif
#define SW_MINW(L) (Blk<L>::THREADS >= 1024 ? 4 : SW_MINW_FFT)

// threads per block: one line of NT = N/8 threads, or several short lines
// packed into 256 threads
template <int LOG2N>
struct Blk {
  static constexpr int NT = FftPlan<LOG2N>::NT;
  // at most 32 lines, so that NB divides ny (>= 32) and kcP (multiple of 64)
  static constexpr int NB = NT >= 256 ? 1 : (256 / NT > 32 ? 32 : 256 / NT);
  static constexpr int THREADS = NB * NT;
};

struct LineCtx {
  int ln, t;
};
template <int LOG2N>
__device__ __forceinline__ LineCtx line_ctx() {
  constexpr int NT = FftPlan<LOG2N>::NT;
  LineCtx c;
  c.ln = threadIdx.x / NT;
  c.t = threadIdx.x - c.ln * NT;
  return c;
}

__device__ __forceinline__ double2 zero2() { return make_double2(0.0, 0.0); }

// ===========================================================================
// col_inv: for column kr, build the y-spectra the row pass needs, inverse FFT
// along y (scaled by 1/(nx ny), FF's normalised c2r), store to mixed space.
//   RSW  outputs (rsw/RotatingShallowWater.jl:147-214): 0 U, 1 V, 2 H, 3 Uy=il U, 4 Vy=il V
//   QG2  outputs (swqg/TwoLayerQG.jl:155-176):          0 Q1, 1 Q2, 2 Ψ1, 3 Ψ2, 4 Ψy1, 5 Ψy2
// grid: (columns, groups); RSW group f reads field f; QG2 group = layer.
// ===========================================================================
template <int MODEL, int LOG2N>
__global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_col_inv(Geom g, Phys p, const double2* __restrict__ X, double2* __restrict__ M,
              const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int kr = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
  const int grp = blockIdx.y;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  const bool live = kr < g.kc;
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  const double k = kr * g.mk;
  double2 v[8];

  auto store = [&](int o) {  // fft_line leaves Y[t + s*NT] in v[s]
    if (live) {
      double2* Mo = M + (long long)o * g.mfield;
#pragma unroll
      for (int s = 0; s < 8; ++s) Mo[midx(g, kr, c.t + s * NT)] = v[s];
    }
  };

  // loads are unconditional from a clamped in-bounds address, then selected:
  // a branch around each load would serialise them (one vmcnt(0) per element)
  const int krc = live ? kr : g.kc - 1;
  if constexpr (MODEL == MODEL_RSW) {
    const double2* Xf = X + (long long)grp * g.cfield + (long long)krc * g.LrP;
    double2 x[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int m = c.t + s * NT;
      const int j = compact_of(g, m);
      const double2 t = Xf[j >= 0 ? j : 0];
      x[s] = (live && j >= 0) ? t : zero2();
      v[s] = cscale(x[s], scale);
    }
    fft_line<LOG2N, +1>(v, c.t, tws, line);
    store(grp);
    if (grp < 2) {  // ∂y: Uy, Vy
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cmul_i(x[s], lwav(g, c.t + s * NT) * scale);
      fft_line<LOG2N, +1>(v, c.t, tws, line);
      store(3 + grp);
    }
  } else {
    // streamfunctionfrompv! (swqg/TwoLayerQG.jl:101-111)
    const double2* X1 = X + (long long)krc * g.LrP;
    const double2* X2 = X1 + g.cfield;
    double2 psi[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int m = c.t + s * NT;
      const int j = compact_of(g, m);
      const int jc = j >= 0 ? j : 0;
      double2 q1 = X1[jc], q2 = X2[jc];
      if (!(live && j >= 0)) {
        q1 = zero2();
        q2 = zero2();
      }
      const double l = lwav(g, m);
      const double K2 = k * k + l * l;
      const double iK2 = K2 == 0.0 ? 0.0 : 1.0 / K2;
      const double den = K2 + 2.0 * p.F;
      const double2 qs = cadd(q1, q2);
      const double2 qg = grp == 0 ? q1 : q2;
      double2 ps = make_double2(-(K2 * qg.x + p.F * qs.x), -(K2 * qg.y + p.F * qs.y));
      psi[s] = make_double2((ps.x / den) * iK2, (ps.y / den) * iK2);
      v[s] = cscale(qg, scale);
    }
    fft_line<LOG2N, +1>(v, c.t, tws, line);
    store(grp);
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = cscale(psi[s], scale);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
    store(2 + grp);
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = cmul_i(psi[s], lwav(g, c.t + s * NT) * scale);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
    store(4 + grp);
  }
}

// ===========================================================================
// row: one physical row y per line.  Real fields travel in pairs a + i b
// through one complex FFT of length nx (Z[k] = A[k] + i B[k] for k <= nx/2,
// Z[nx-k] = conj(A[k]) + i conj(B[k]); the DC bin keeps real parts only —
// numpy's c2r rule).
// ===========================================================================
template <int LOG2N>
__device__ __forceinline__ void load_pair(double2 (&v)[8], int t, const Geom& g,
                                          const double2* __restrict__ A,
                                          const double2* __restrict__ B, int y, bool deriv) {
  constexpr int N = 1 << LOG2N, NT = N / 8, half = N / 2;
  double2 a[8], b[8];
  int kk[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {  // issue every load first (clamped, unconditional)
    const int m = t + s * NT;
    kk[s] = m <= half ? m : N - m;
    const int o = midx(g, kk[s] < g.kc ? kk[s] : 0, y);
    a[s] = A[o];
    b[s] = B ? B[o] : zero2();
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int m = t + s * NT;
    double2 aa = a[s], bb = b[s];
    if (deriv) {
      const double kw = kk[s] * g.mk;
      aa = cmul_i(aa, kw);
      bb = cmul_i(bb, kw);
    }
    if (kk[s] == 0) {
      aa.y = 0.0;
      bb.y = 0.0;
    }
    if (m > half) {
      aa = cconj(aa);
      bb = cconj(bb);
    }
    const double2 z = make_double2(aa.x - bb.y, aa.y + bb.x);  // a + i b
    v[s] = kk[s] < g.kc ? z : zero2();
  }
}

// After a forward FFT of z = a + i b (Z[t + s*NT] in v), write Â[k], B̂[k]
// for k < kc.  Needs Z[nx-k] from a mirror thread: one LDS round trip.
template <int LOG2N>
__device__ __forceinline__ void store_pair(const double2 (&v)[8], int t, const Geom& g,
                                           double2* line, double2* __restrict__ A,
                                           double2* __restrict__ B, int y) {
  constexpr int N = 1 << LOG2N, NT = N / 8;
  lds_barrier();  // previous LDS readers are done
#pragma unroll
  for (int s = 0; s < 8; ++s) line[LP(t + s * NT)] = v[s];
  lds_barrier();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = t + s * NT;
    if (k < g.kc) {
      const double2 zk = v[s];
      const double2 zn = line[LP((N - k) & (N - 1))];
      const int o = midx(g, k, y);
      A[o] = make_double2(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
      // (zk - conj zn) / (2i)
      B[o] = make_double2(0.5 * (zk.y + zn.y), -0.5 * (zk.x - zn.x));
    }
  }
}

template <int MODEL, int LOG2N>
__global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_row(Geom g, Phys p, const double2* __restrict__ Mi, double2* __restrict__ Mo,
          const double2* __restrict__ tw) {
  using Bk = Blk<LOG2N>;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int y = blockIdx.x * Bk::NB + c.ln;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  const long long MF = g.mfield;
  double2 v[8];

  if constexpr (MODEL == MODEL_RSW) {
    const double2 *U = Mi, *V = Mi + MF, *H = Mi + 2 * MF, *Uy = Mi + 3 * MF, *Vy = Mi + 4 * MF;
    double2 uv[8], ab[8];
    // u + i v   (fft_line leaves z[x = t + s*NT] in v[s])
    load_pair<LOG2N>(v, c.t, g, U, V, y, false);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) uv[s] = v[s];
    // ux + i vx:  A = u ux, B = u vx   (:172, :204)
    load_pair<LOG2N>(v, c.t, g, U, V, y, true);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) ab[s] = make_double2(uv[s].x * v[s].x, uv[s].x * v[s].y);
    // uy + i vy:  A += v uy, B += v vy   (:181, :195)
    load_pair<LOG2N>(v, c.t, g, Uy, Vy, y, false);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s)
      v[s] = make_double2(ab[s].x + uv[s].y * v[s].x, ab[s].y + uv[s].y * v[s].y);
    fft_line<LOG2N, -1>(v, c.t, tws, line);
    store_pair<LOG2N>(v, c.t, g, line, Mo, Mo + MF, y);
    // η:  C = u η, D = v η   (:218, :224)
    load_pair<LOG2N>(v, c.t, g, H, nullptr, y, false);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = make_double2(uv[s].x * v[s].x, uv[s].y * v[s].x);
    fft_line<LOG2N, -1>(v, c.t, tws, line);
    store_pair<LOG2N>(v, c.t, g, line, Mo + 2 * MF, Mo + 3 * MF, y);
  } else {
    const double2 *Q1 = Mi, *Q2 = Mi + MF, *P1 = Mi + 2 * MF, *P2 = Mi + 3 * MF,
                  *Py1 = Mi + 4 * MF, *Py2 = Mi + 5 * MF;
    double2 q[8];
    // q1 + i q2
    load_pair<LOG2N>(v, c.t, g, Q1, Q2, y, false);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) q[s] = v[s];
    // ψx1 + i ψx2;  ψx q per layer (swqg/TwoLayerQG.jl:169)
    load_pair<LOG2N>(v, c.t, g, P1, P2, y, true);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = make_double2(v[s].x * q[s].x, v[s].y * q[s].y);
    fft_line<LOG2N, -1>(v, c.t, tws, line);
    store_pair<LOG2N>(v, c.t, g, line, Mo, Mo + MF, y);
    // ψy q per layer (:177)
    load_pair<LOG2N>(v, c.t, g, Py1, Py2, y, false);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = make_double2(v[s].x * q[s].x, v[s].y * q[s].y);
    fft_line<LOG2N, -1>(v, c.t, tws, line);
    store_pair<LOG2N>(v, c.t, g, line, Mo + 2 * MF, Mo + 3 * MF, y);
  }
}

// ===========================================================================
// col_fwd: forward FFT along y of the row outputs, combine into N (live rows).
//   RSW (rsw/RotatingShallowWater.jl:174-226):
//     N0 = -F(A), N1 = -F(B), N2 = -ik F(C) - il F(D)
//   QG2 (swqg/TwoLayerQG.jl:171,179): N_l = -il F(A_l) + ik F(B_l)
// ===========================================================================
template <int MODEL, int LOG2N>
__global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_col_fwd(Geom g, Phys p, const double2* __restrict__ Mf, double2* __restrict__ N,
              const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int kr = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
  const int grp = blockIdx.y;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  const bool live = kr < g.kc;
  const double k = kr * g.mk;
  const long long MF = g.mfield;
  double2 v[8], acc[8];

  auto load_col = [&](const double2* Mfield) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double2 t = Mfield[midx(g, kr, c.t + s * NT)];  // kr < kcP: always in bounds
      v[s] = live ? t : zero2();
    }
  };

  int fa, fb;
  if constexpr (MODEL == MODEL_RSW) {
    fa = grp < 2 ? grp : 2;
    fb = grp < 2 ? -1 : 3;
  } else {
    fa = grp;      // A_l
    fb = 2 + grp;  // B_l
  }
  // fft_line leaves F[m = t + s*NT] in v[s]; only live rows are written
  load_col(Mf + fa * MF);
  fft_line<LOG2N, -1>(v, c.t, tws, line);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const double2 a = v[s];
    if constexpr (MODEL == MODEL_RSW) {
      acc[s] = (grp < 2) ? make_double2(-a.x, -a.y) : cmul_i(a, -k);
    } else {
      acc[s] = cmul_i(a, -lwav(g, c.t + s * NT));
    }
  }
  if (fb >= 0) {
    load_col(Mf + fb * MF);
    fft_line<LOG2N, -1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int m = c.t + s * NT;
      if constexpr (MODEL == MODEL_RSW) {
        acc[s] = cadd(acc[s], cmul_i(v[s], -lwav(g, m)));
      } else {
        acc[s] = cadd(acc[s], cmul_i(v[s], k));
      }
    }
  }
  if (live) {
    double2* Nf = N + (long long)grp * g.cfield + (long long)kr * g.LrP;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = compact_of(g, c.t + s * NT);
      if (j >= 0) Nf[j] = acc[s];
    }
  }
}

// ===========================================================================
// stepper updates over live modes (one thread per mode, all fields)
// ===========================================================================
__device__ __forceinline__ bool mode_of(const Geom& g, long long i, int& kr, int& j) {
  kr = (int)(i / g.LrP);
  j = (int)(i - (long long)kr * g.LrP);
  return kr < g.kc && j < g.Lr;
}

template <int NF>
__device__ __forceinline__ void model_L(int model, const Phys& p, double k, double l, cplx L[NF][NF]) {
  if constexpr (NF == 3) {
    rsw_L(p, k, l, L);
  } else {
    qg2_L(p, k, l, L);
  }
}

// FF FilteredAB3: RHS = N + L·sol; Euler for step < 3, else AB3;
// sol .*= filter.  RHS overwrites N in place (it becomes history).
template <int NF>
__global__ void k_upd_fab3(Geom g, Phys p, double2* __restrict__ sol, double2* __restrict__ NR,
                           const double2* __restrict__ Rm1, const double2* __restrict__ Rm2,
                           int euler) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
  cplx L[NF][NF];
  model_L<NF>(0, p, k, l, L);
  cplx s[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const double2 t = sol[f * g.cfield + i];
    s[f] = cx(t.x, t.y);
  }
  const double filt = filter_value(g, p, k, l);
  const double dt = p.dt;
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    cplx Ls = cx(0.0);
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) Ls = Ls + L[r][cc] * s[cc];
    const double2 n = NR[r * g.cfield + i];
    const cplx rhs = cx(n.x + Ls.re, n.y + Ls.im);
    cplx upd;
    if (euler) {
      upd = dt * rhs;
    } else {
      const double2 a = Rm1[r * g.cfield + i], b = Rm2[r * g.cfield + i];
      upd = dt * cx(23.0 / 12 * rhs.re - 16.0 / 12 * a.x + 5.0 / 12 * b.x,
                    23.0 / 12 * rhs.im - 16.0 / 12 * a.y + 5.0 / 12 * b.y);
    }
    NR[r * g.cfield + i] = make_double2(rhs.re, rhs.im);
    const cplx ns = s[r] + upd;
    sol[r * g.cfield + i] = make_double2(ns.re * filt, ns.im * filt);
  }
}

template <int NF>
__device__ __forceinline__ void load_mat(const double2* __restrict__ E, long long cf, long long i,
                                         cplx M[NF][NF]) {
#pragma unroll
  for (int r = 0; r < NF; ++r)
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) {
      const double2 t = E[(r * NF + cc) * cf + i];
      M[r][cc] = cx(t.x, t.y);
    }
}

template <int NF>
__device__ __forceinline__ void load_vec(const double2* __restrict__ X, long long cf, long long i,
                                         cplx x[NF]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const double2 t = X[f * cf + i];
    x[f] = cx(t.x, t.y);
  }
}

template <int NF>
__device__ __forceinline__ void matvec(const cplx M[NF][NF], const cplx x[NF], cplx y[NF]) {
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    cplx s = cx(0.0);
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) s = s + M[r][cc] * x[cc];
    y[r] = s;
  }
}

// utils/IFMAB3.jl:129-160: Euler for step < 3, else AB3 with E N₋₁, E2 N₋₂;
// then sol = E·(…); filter.
template <int NF>
__global__ void k_upd_ifmab3(Geom g, Phys p, double2* __restrict__ sol, const double2* __restrict__ N,
                             const double2* __restrict__ Nm1, const double2* __restrict__ Nm2,
                             const double2* __restrict__ E, const double2* __restrict__ E2,
                             int euler) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const long long cf = g.cfield;
  cplx M[NF][NF], s[NF], n[NF], x[NF], y[NF];
  load_mat<NF>(E, cf, i, M);
  load_vec<NF>(sol, cf, i, s);
  load_vec<NF>(N, cf, i, n);
  const double dt = p.dt;
  if (euler) {
#pragma unroll
    for (int f = 0; f < NF; ++f) x[f] = s[f] + dt * n[f];
  } else {
    cplx a[NF], b[NF], e1[NF], e2[NF], M2[NF][NF];
    load_vec<NF>(Nm1, cf, i, a);
    load_vec<NF>(Nm2, cf, i, b);
    load_mat<NF>(E2, cf, i, M2);
    matvec<NF>(M, a, e1);
    matvec<NF>(M2, b, e2);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const cplx comb = cx(23.0 / 12 * n[f].re - 16.0 / 12 * e1[f].re + 5.0 / 12 * e2[f].re,
                           23.0 / 12 * n[f].im - 16.0 / 12 * e1[f].im + 5.0 / 12 * e2[f].im);
      x[f] = s[f] + dt * comb;
    }
  }
  matvec<NF>(M, x, y);
  double filt = 1.0;
  if (p.use_filter) {
    const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
    filt = filter_value(g, p, k, l);
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) sol[f * cf + i] = make_double2(y[f].re * filt, y[f].im * filt);
}

// Lawson IF-RK4 stage inputs:
//   which 1: x = H (u + dt/2 k1);  2: x = H u + dt/2 k2;  3: x = E u + dt H k3
template <int NF>
__global__ void k_rk4_stage(Geom g, Phys p, int which, const double2* __restrict__ u,
                            const double2* __restrict__ kk, const double2* __restrict__ E,
                            const double2* __restrict__ H, double2* __restrict__ x) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const long long cf = g.cfield;
  const double dt = p.dt;
  cplx uu[NF], kv[NF], M[NF][NF], t[NF], o[NF];
  load_vec<NF>(u, cf, i, uu);
  load_vec<NF>(kk, cf, i, kv);
  if (which == 1) {
    load_mat<NF>(H, cf, i, M);
#pragma unroll
    for (int f = 0; f < NF; ++f) t[f] = uu[f] + (0.5 * dt) * kv[f];
    matvec<NF>(M, t, o);
  } else if (which == 2) {
    load_mat<NF>(H, cf, i, M);
    matvec<NF>(M, uu, t);
#pragma unroll
    for (int f = 0; f < NF; ++f) o[f] = t[f] + (0.5 * dt) * kv[f];
  } else {
    cplx M2[NF][NF], hk[NF];
    load_mat<NF>(E, cf, i, M);
    load_mat<NF>(H, cf, i, M2);
    matvec<NF>(M, uu, t);
    matvec<NF>(M2, kv, hk);
#pragma unroll
    for (int f = 0; f < NF; ++f) o[f] = t[f] + dt * hk[f];
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) x[f * cf + i] = make_double2(o[f].re, o[f].im);
}

// u <- E u + dt/6 (E k1 + 2 H (k2 + k3) + k4); filter
template <int NF>
__global__ void k_rk4_final(Geom g, Phys p, double2* __restrict__ u, const double2* __restrict__ k1,
                            const double2* __restrict__ k2, const double2* __restrict__ k3,
                            const double2* __restrict__ k4, const double2* __restrict__ E,
                            const double2* __restrict__ H) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const long long cf = g.cfield;
  const double dt = p.dt;
  cplx uu[NF], a[NF], b[NF], c3[NF], d[NF], ME[NF][NF], MH[NF][NF], Eu[NF], Ek1[NF], s23[NF], H23[NF];
  load_vec<NF>(u, cf, i, uu);
  load_vec<NF>(k1, cf, i, a);
  load_vec<NF>(k2, cf, i, b);
  load_vec<NF>(k3, cf, i, c3);
  load_vec<NF>(k4, cf, i, d);
  load_mat<NF>(E, cf, i, ME);
  load_mat<NF>(H, cf, i, MH);
  matvec<NF>(ME, uu, Eu);
  matvec<NF>(ME, a, Ek1);
#pragma unroll
  for (int f = 0; f < NF; ++f) s23[f] = b[f] + c3[f];
  matvec<NF>(MH, s23, H23);
  double filt = 1.0;
  if (p.use_filter) filt = filter_value(g, p, kr * g.mk, lwav(g, lrow_of(g, j)));
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const cplx comb = Ek1[f] + 2.0 * H23[f] + d[f];
    const cplx r = Eu[f] + (dt / 6) * comb;
    u[f * cf + i] = make_double2(r.re * filt, r.im * filt);
  }
}

// per-mode exp(factor·dt·L) (utils/IFMAB3.jl:32-41), stored [r][c] planes
template <int NF>
__global__ void k_setup_expm(Geom g, Phys p, double factor, double2* __restrict__ E) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
  cplx L[NF][NF], A[NF][NF], X[NF][NF];
  model_L<NF>(0, p, k, l, L);
  const double sdt = factor * p.dt;
#pragma unroll
  for (int r = 0; r < NF; ++r)
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) A[r][cc] = sdt * L[r][cc];
  expm<NF>(A, X);
#pragma unroll
  for (int r = 0; r < NF; ++r)
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) E[(r * NF + cc) * g.cfield + i] = make_double2(X[r][cc].re, X[r][cc].im);
}

// ===========================================================================
// state I/O: Julia column-major (nkr, nl, nf) <-> compact live columns
// ===========================================================================
__global__ void k_gather(Geom g, int nf, const double2* __restrict__ full, double2* __restrict__ cmp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)g.kc * g.Lr;
  if (i >= per * nf) return;
  const int f = (int)(i / per);
  const long long r = i - f * per;
  const int j = (int)(r / g.kc), kr = (int)(r - (long long)j * g.kc);
  const int m = lrow_of(g, j);
  cmp[f * g.cfield + (long long)kr * g.LrP + j] = full[((long long)f * g.nl + m) * g.nkr + kr];
}

__global__ void k_scatter(Geom g, int nf, const double2* __restrict__ cmp, double2* __restrict__ full) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)g.nkr * g.nl;
  if (i >= per * nf) return;
  const int f = (int)(i / per);
  const long long r = i - f * per;
  const int m = (int)(r / g.nkr), kr = (int)(r - (long long)m * g.nkr);
  const int j = compact_of(g, m);
  double2 v = zero2();
  if (kr < g.kc && j >= 0) v = cmp[f * g.cfield + (long long)kr * g.LrP + j];
  full[i] = v;
}

__global__ void k_nan_check(Geom g, int nf, const double2* __restrict__ cmp, int* flag) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  int bad = 0;
  if (i < g.cfield && mode_of(g, i, kr, j)) {
    for (int f = 0; f < nf; ++f) {
      const double2 v = cmp[f * g.cfield + i];
      if (!isfinite(v.x) || !isfinite(v.y)) bad = 1;
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// ===========================================================================
// updatevars! support: one spectral field -> physical
// ===========================================================================
// field ids: RSW 0 u, 1 v, 2 η, 3 ζ = ik v - il u - f η (rsw/RotatingShallowWater.jl:108)
//            QG2 layer*8 + {4 q, 5 ψ, 3 ζ = -K² ψ, 0 u = -il ψ, 1 v = ik ψ} (swqg/TwoLayerQG.jl:117-121)
__global__ void k_make_spec(Geom g, Phys p, int model, int fid, const double2* __restrict__ sol,
                            double2* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const long long cf = g.cfield;
  const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
  double2 r = zero2();
  if (model == MODEL_RSW) {
    if (fid <= 2) {
      r = sol[fid * cf + i];
    } else {
      const double2 u = sol[i], v = sol[cf + i], e = sol[2 * cf + i];
      const double2 a = cmul_i(v, k), b = cmul_i(u, l);
      r = make_double2(a.x - b.x - p.f * e.x, a.y - b.y - p.f * e.y);
    }
  } else {
    const int layer = fid >> 3, id = fid & 7;
    const double2 q1 = sol[i], q2 = sol[cf + i];
    const double2 qg = layer ? q2 : q1;
    if (id == 4) {  // q
      r = qg;
    } else {
      const double K2 = k * k + l * l;
      const double iK2 = K2 == 0.0 ? 0.0 : 1.0 / K2;
      const double den = K2 + 2.0 * p.F;
      const double2 qs = cadd(q1, q2);
      double2 ps = make_double2(-(K2 * qg.x + p.F * qs.x), -(K2 * qg.y + p.F * qs.y));
      ps = make_double2((ps.x / den) * iK2, (ps.y / den) * iK2);
      if (id == 5) r = ps;
      else if (id == 3) r = make_double2(-K2 * ps.x, -K2 * ps.y);
      else if (id == 0) r = cmul_i(ps, -l);
      else if (id == 1) r = cmul_i(ps, k);
    }
  }
  out[i] = r;
}

template <int LOG2N>
__global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_col_inv1(Geom g, const double2* __restrict__ X, double2* __restrict__ M,
               const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int kr = blockIdx.x * B::NB + c.ln;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  const bool live = kr < g.kc;
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  const double2* Xf = X + (long long)(live ? kr : g.kc - 1) * g.LrP;
  double2 v[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int j = compact_of(g, c.t + s * NT);
    const double2 t = Xf[j >= 0 ? j : 0];
    v[s] = (live && j >= 0) ? cscale(t, scale) : zero2();
  }
  fft_line<LOG2N, +1>(v, c.t, tws, line);
  if (live) {
#pragma unroll
    for (int s = 0; s < 8; ++s) M[midx(g, kr, c.t + s * NT)] = v[s];
  }
}

template <int LOG2N>
__global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_row_c2r1(Geom g, const double2* __restrict__ M, double* __restrict__ out,
               const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int y = blockIdx.x * B::NB + c.ln;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  double2 v[8];
  load_pair<LOG2N>(v, c.t, g, M, nullptr, y, false);
  fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
  for (int s = 0; s < 8; ++s) out[(long long)y * g.nx + c.t + s * NT] = v[s].x;
}

// Energies by Parseval over live modes (FF parsevalsum2 / parsevalsum:
// weight 2 for 0 < kr < nx/2, 1 for kr = 0).  acc[0] = KE-sum, acc[1] = PE-sum.
__global__ void k_energy(Geom g, Phys p, int model, const double2* __restrict__ sol, double* acc) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  double ke = 0.0, pe = 0.0;
  if (i < g.cfield && mode_of(g, i, kr, j)) {
    const long long cf = g.cfield;
    const double w = kr == 0 ? 1.0 : 2.0;
    if (model == MODEL_RSW) {
      const double2 u = sol[i], v = sol[cf + i], e = sol[2 * cf + i];
      ke = w * (u.x * u.x + u.y * u.y + v.x * v.x + v.y * v.y);
      pe = w * (e.x * e.x + e.y * e.y);
    } else {
      const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
      const double K2 = k * k + l * l;
      const double iK2 = K2 == 0.0 ? 0.0 : 1.0 / K2;
      const double den = K2 + 2.0 * p.F;
      const double2 q1 = sol[i], q2 = sol[cf + i];
      const double2 qs = cadd(q1, q2);
      double2 p1 = make_double2(-(K2 * q1.x + p.F * qs.x), -(K2 * q1.y + p.F * qs.y));
      double2 p2 = make_double2(-(K2 * q2.x + p.F * qs.x), -(K2 * q2.y + p.F * qs.y));
      p1 = make_double2((p1.x / den) * iK2, (p1.y / den) * iK2);
      p2 = make_double2((p2.x / den) * iK2, (p2.y / den) * iK2);
      ke = w * K2 * (p1.x * p1.x + p1.y * p1.y + p2.x * p2.x + p2.y * p2.y);
      const double dx_ = p1.x - p2.x, dy_ = p1.y - p2.y;
      pe = w * (dx_ * dx_ + dy_ * dy_);
    }
  }
  // wave reduction
  for (int off = 32; off > 0; off >>= 1) {
    ke += __shfl_down(ke, off, 64);
    pe += __shfl_down(pe, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(acc, ke);
    atomicAdd(acc + 1, pe);
  }
}

// ===========================================================================
// launchers
// ===========================================================================
// host-side: dispatch the LOG2N instantiation (N = 32 … 8192)
#define SW_LOG2_CASES(X) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13)

template <template <int> class F, typename... Args>
static void dispatch_log2(int log2n, Args&&... args) {
  switch (log2n) {
#define SW_CASE(L) \
  case L:          \
    F<L>::run(args...); \
    break;
    SW_LOG2_CASES(SW_CASE)
#undef SW_CASE
    default:
      break;
  }
}

template <int L>
static int col_blocks(const Geom& g) {
  return (g.kcP + Blk<L>::NB - 1) / Blk<L>::NB;
}
template <int L>
static int row_blocks(const Geom& g) {
  return g.ny / Blk<L>::NB;
}
template <int L>
static size_t lds_bytes() {
  return (size_t)Blk<L>::NB * FftPlan<L>::LDS * sizeof(double2);
}

template <int L>
struct ColInvL {
  static void run(int model, const Geom& g, const Phys& p, const double2* X, double2* M,
                  const double2* tw, hipStream_t s) {
    const dim3 grid(col_blocks<L>(g), model == MODEL_RSW ? 3 : 2);
    if (model == MODEL_RSW)
      hipLaunchKernelGGL((k_col_inv<MODEL_RSW, L>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M, tw);
    else
      hipLaunchKernelGGL((k_col_inv<MODEL_QG2, L>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M, tw);
  }
};
template <int L>
struct RowL {
  static void run(int model, const Geom& g, const Phys& p, const double2* Mi, double2* Mo,
                  const double2* tw, hipStream_t s) {
    if (model == MODEL_RSW)
      hipLaunchKernelGGL((k_row<MODEL_RSW, L>), dim3(row_blocks<L>(g)), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, Mi, Mo, tw);
    else
      hipLaunchKernelGGL((k_row<MODEL_QG2, L>), dim3(row_blocks<L>(g)), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, Mi, Mo, tw);
  }
};
template <int L>
struct ColFwdL {
  static void run(int model, const Geom& g, const Phys& p, const double2* Mf, double2* N,
                  const double2* tw, hipStream_t s) {
    const dim3 grid(col_blocks<L>(g), model == MODEL_RSW ? 3 : 2);
    if (model == MODEL_RSW)
      hipLaunchKernelGGL((k_col_fwd<MODEL_RSW, L>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, Mf, N, tw);
    else
      hipLaunchKernelGGL((k_col_fwd<MODEL_QG2, L>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, Mf, N, tw);
  }
};
template <int L>
struct ColInv1L {
  static void run(const Geom& g, const double2* X, double2* M, const double2* tw, hipStream_t s) {
    hipLaunchKernelGGL((k_col_inv1<L>), dim3(col_blocks<L>(g)), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, X, M, tw);
  }
};
template <int L>
struct RowC2r1L {
  static void run(const Geom& g, const double2* M, double* out, const double2* tw, hipStream_t s) {
    hipLaunchKernelGGL((k_row_c2r1<L>), dim3(row_blocks<L>(g)), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, M, out, tw);
  }
};

void launch_col_inv(int model, const Geom& g, const Phys& p, const double2* X, double2* Minv,
                    const double2* tw_y, hipStream_t s) {
  dispatch_log2<ColInvL>(g.log2ny, model, g, p, X, Minv, tw_y, s);
}
void launch_row(int model, const Geom& g, const Phys& p, const double2* Minv, double2* Mfwd,
                const double2* tw_x, hipStream_t s) {
  dispatch_log2<RowL>(g.log2nx, model, g, p, Minv, Mfwd, tw_x, s);
}
void launch_col_fwd(int model, const Geom& g, const Phys& p, const double2* Mfwd, double2* N,
                    const double2* tw_y, hipStream_t s) {
  dispatch_log2<ColFwdL>(g.log2ny, model, g, p, Mfwd, N, tw_y, s);
}

static inline dim3 mode_grid(const Geom& g) { return dim3((unsigned)((g.cfield + 255) / 256)); }

void launch_upd_fab3(int model, const Geom& g, const Phys& p, double2* sol, double2* NR,
                     const double2* Rm1, const double2* Rm2, int euler, hipStream_t s) {
  if (model == MODEL_RSW)
    hipLaunchKernelGGL(k_upd_fab3<3>, mode_grid(g), dim3(256), 0, s, g, p, sol, NR, Rm1, Rm2, euler);
  else
    hipLaunchKernelGGL(k_upd_fab3<2>, mode_grid(g), dim3(256), 0, s, g, p, sol, NR, Rm1, Rm2, euler);
}

void launch_upd_ifmab3(int nf, const Geom& g, const Phys& p, double2* sol, const double2* N,
                       const double2* Nm1, const double2* Nm2, const double2* E, const double2* E2,
                       int euler, hipStream_t s) {
  if (nf == 3)
    hipLaunchKernelGGL(k_upd_ifmab3<3>, mode_grid(g), dim3(256), 0, s, g, p, sol, N, Nm1, Nm2, E, E2, euler);
  else
    hipLaunchKernelGGL(k_upd_ifmab3<2>, mode_grid(g), dim3(256), 0, s, g, p, sol, N, Nm1, Nm2, E, E2, euler);
}

void launch_rk4_stage(int nf, int which, const Geom& g, const Phys& p, const double2* u,
                      const double2* k, const double2* E, const double2* H, double2* x,
                      hipStream_t s) {
  if (nf == 3)
    hipLaunchKernelGGL(k_rk4_stage<3>, mode_grid(g), dim3(256), 0, s, g, p, which, u, k, E, H, x);
  else
    hipLaunchKernelGGL(k_rk4_stage<2>, mode_grid(g), dim3(256), 0, s, g, p, which, u, k, E, H, x);
}

void launch_rk4_final(int nf, const Geom& g, const Phys& p, double2* u, const double2* k1,
                      const double2* k2, const double2* k3, const double2* k4, const double2* E,
                      const double2* H, hipStream_t s) {
  if (nf == 3)
    hipLaunchKernelGGL(k_rk4_final<3>, mode_grid(g), dim3(256), 0, s, g, p, u, k1, k2, k3, k4, E, H);
  else
    hipLaunchKernelGGL(k_rk4_final<2>, mode_grid(g), dim3(256), 0, s, g, p, u, k1, k2, k3, k4, E, H);
}

void launch_setup_expm(int model, const Geom& g, const Phys& p, double factor, double2* E,
                       hipStream_t s) {
  if (model == MODEL_RSW)
    hipLaunchKernelGGL(k_setup_expm<3>, mode_grid(g), dim3(256), 0, s, g, p, factor, E);
  else
    hipLaunchKernelGGL(k_setup_expm<2>, mode_grid(g), dim3(256), 0, s, g, p, factor, E);
}

void launch_gather(int nf, const Geom& g, const double2* full, double2* cmp, hipStream_t s) {
  const long long n = (long long)g.kc * g.Lr * nf;
  hipLaunchKernelGGL(k_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, nf, full, cmp);
}

void launch_scatter(int nf, const Geom& g, const double2* cmp, double2* full, hipStream_t s) {
  const long long n = (long long)g.nkr * g.nl * nf;
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, nf, cmp, full);
}

void launch_nan_check(int nf, const Geom& g, const double2* cmp, int* flag, hipStream_t s) {
  hipLaunchKernelGGL(k_nan_check, mode_grid(g), dim3(256), 0, s, g, nf, cmp, flag);
}

void launch_make_spec(int model, int fid, const Geom& g, const Phys& p, const double2* sol,
                      double2* out, hipStream_t s) {
  hipLaunchKernelGGL(k_make_spec, mode_grid(g), dim3(256), 0, s, g, p, model, fid, sol, out);
}

void launch_col_inv1(const Geom& g, const double2* X, double2* M, const double2* tw_y, hipStream_t s) {
  dispatch_log2<ColInv1L>(g.log2ny, g, X, M, tw_y, s);
}

void launch_row_c2r1(const Geom& g, const double2* M, double* out, const double2* tw_x, hipStream_t s) {
  dispatch_log2<RowC2r1L>(g.log2nx, g, M, out, tw_x, s);
}

void launch_energy(int model, const Geom& g, const Phys& p, const double2* sol, double* acc,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_energy, mode_grid(g), dim3(256), 0, s, g, p, model, sol, acc);
}

}  // namespace sw
