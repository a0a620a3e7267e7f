// Shared host/device definitions for libsw (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

// No implicit FMA contraction in libsw: the same formula rounds the same way
// in every kernel (and on the host), so kernel fusion never changes results.
#pragma clang fp contract(off)

namespace sw {

enum { MODEL_RSW = 0, MODEL_QG2 = 1 };
enum { ST_FAB3 = 0, ST_IFMAB3 = 1, ST_IFMRK4 = 2 };

// Grid geometry of one slab in the layouts of DESIGN.md §2 and §6.
// Slab s of P owns kr columns [kr0, kr0 + kcl) in the column passes and
// physical rows [y0, y0 + nyl) in the row pass (P = 1: kr0 = y0 = 0,
// kcl = roundup(kc, 64), nyl = ny).
//  compact spectral field: [krl][j], krl < kcn live local columns, j < Lr live
//    rows, column stride LrP
//  mixed fields: midx/midc (forward direction), midx_i/midc_i (inverse
//    direction) below.  Block q of a column-phase array (rows of slab q) is
//    exactly the block slab q holds for this slab's columns in its row-phase
//    array, so the transpose between the passes is a plain all-to-all of
//    contiguous blocks.
struct Geom {
  int nx, ny, log2nx, log2ny;
  int nkr, nl;
  int kc;             // global live kr columns [0, kc)
  int lc, lr2, Lr, LrP;  // live l rows [0, lc) ∪ [lr2, ny); count Lr; stride LrP
  double mk, ml;      // kr = i*mk, l = (signed j)*ml
  double dx, dy, Lx, Ly;
  // slab decomposition
  int nslab, slab;    // P, this slab
  int kr0, kcn, kcl, ntl;  // first global column, live local columns, local columns (multiple of 8), kcl/8
  int y0, nyl, log2nyl;    // first row, local rows
  long long cfield;   // elements per compact field  = max(kcn,1)*LrP
  long long mfield;   // elements per mixed field    = kcl*ny = (P*kcl)*nyl
};

struct Phys {
  double f, Cg2, nu;  // RSW
  int nnu;
  double U, mu, F;    // QG2
  // filter (FF makefilter)
  int use_filter, forder;
  double innerK, decay;
  double dt;
};

__host__ __device__ inline int lrow_of(const Geom& g, int j) { return j < g.lc ? j : j - g.lc + g.lr2; }
__host__ __device__ inline int compact_of(const Geom& g, int m) {
  return m < g.lc ? m : (m >= g.lr2 ? m - g.lr2 + g.lc : -1);
}
__host__ __device__ inline double lwav(const Geom& g, int m) {
  return (double)(m < (g.ny >> 1) ? m : m - g.ny) * g.ml;
}
// Element offsets inside one mixed field (< 2^31 for nx, ny <= 8192).  A
// 128-B line holds a tile of A columns kr × B = 8/A rows y (16-B elements, kr
// fastest).  The row pass touches 16·A bytes of a line, the column pass
// 16·B; the blocks that share a line are placed on one XCD (col_of_block),
// where L2 stitches the line.  Measured on MI355X at 2048² (tools/sweep.sh,
// DESIGN.md §2): 2×4 tiles in both directions beat whole-line rows (8×1) or
// whole-line columns (1×8) by 11 % per step, because a pass that touches
// 16 B of each line pays for the whole line in L1 fills and L2 requests.
//  column phase (local column krl, any y): block q = y / nyl, then the tile
//    offset of (krl, y % nyl) inside the block
//  row phase (global kr = p kcl + krl, local row yl): block p, then the tile
//    offset of (krl, yl)
//  so block q of the column-phase array (rows of slab q) is byte for byte
//  block p of slab q's row-phase array.
// The forward fields (row outputs) use A = SW_TILE_F with their lines in
// column order, the inverse fields (column outputs) A = SW_TILE_I with their
// lines in row order.
#ifndef SW_TILE_F
#define SW_TILE_F 2
#endif
#ifndef SW_TILE_I
#define SW_TILE_I 2
#endif
// line order: 0 = [y / B][kr / A] (a row's lines contiguous), 1 = [kr / A][y / B]
#ifndef SW_LORD_F
#define SW_LORD_F 1
#endif
#ifndef SW_LORD_I
#define SW_LORD_I 0
#endif
template <int A, int ORD>
__host__ __device__ inline int mtile_local(const Geom& g, int krl, int yl) {
  // (krl, yl) inside one slab-pair block of kcl columns × nyl rows
  constexpr int B = 8 / A;
  const int line = ORD == 0 ? (yl / B) * (g.kcl / A) + krl / A : (krl / A) * (g.nyl / B) + yl / B;
  return line * 8 + (yl % B) * A + krl % A;
}
template <int A, int ORD>
__host__ __device__ inline int mtile_c(const Geom& g, int krl, int y) {
  return (y >> g.log2nyl) * g.nyl * g.kcl + mtile_local<A, ORD>(g, krl, y & (g.nyl - 1));
}
template <int A, int ORD>
__host__ __device__ inline int mtile_x(const Geom& g, int kr, int yl) {
  int p = 0, krl = kr;
  if (g.nslab > 1) {
    p = kr / g.kcl;
    krl = kr - p * g.kcl;
  }
  return p * g.nyl * g.kcl + mtile_local<A, ORD>(g, krl, yl);
}
// forward fields: row phase / column phase
__host__ __device__ inline int midx(const Geom& g, int kr, int yl) { return mtile_x<SW_TILE_F, SW_LORD_F>(g, kr, yl); }
__host__ __device__ inline int midc(const Geom& g, int krl, int y) { return mtile_c<SW_TILE_F, SW_LORD_F>(g, krl, y); }
// inverse fields: column phase / row phase
__host__ __device__ inline int midc_i(const Geom& g, int krl, int y) { return mtile_c<SW_TILE_I, SW_LORD_I>(g, krl, y); }
__host__ __device__ inline int midx_i(const Geom& g, int kr, int yl) { return mtile_x<SW_TILE_I, SW_LORD_I>(g, kr, yl); }

// integer power x^n (n >= 0) by repeated squaring
__host__ __device__ inline double ipow(double x, int n) {
  double r = 1.0;
  while (n > 0) {
    if (n & 1) r *= x;
    x *= x;
    n >>= 1;
  }
  return r;
}

// FF makefilter value at (k, l): K = sqrt((k dx/π)² + (l dy/π)²),
// filt = exp(-decay (K-innerK)^order) for K >= innerK, else 1.
__host__ __device__ inline double filter_value(const Geom& g, const Phys& p, double k, double l) {
#pragma clang fp contract(off)
  const double a = k * g.dx / 3.14159265358979323846, b = l * g.dy / 3.14159265358979323846;
  const double K = sqrt(a * a + b * b);
  if (K < p.innerK) return 1.0;
  return exp(-p.decay * ipow(K - p.innerK, p.forder));
}

struct cplx {
  double re, im;
};
__host__ __device__ inline cplx cx(double r, double i = 0.0) { return cplx{r, i}; }
__host__ __device__ inline cplx operator+(cplx a, cplx b) { return cplx{a.re + b.re, a.im + b.im}; }
__host__ __device__ inline cplx operator-(cplx a, cplx b) { return cplx{a.re - b.re, a.im - b.im}; }
__host__ __device__ inline cplx operator*(cplx a, cplx b) {
  return cplx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__host__ __device__ inline cplx operator*(double s, cplx a) { return cplx{s * a.re, s * a.im}; }
__host__ __device__ inline cplx cdiv(cplx a, cplx b) {
  // Smith's algorithm
  if (fabs(b.re) >= fabs(b.im)) {
    double r = b.im / b.re, d = b.re + b.im * r;
    return cplx{(a.re + a.im * r) / d, (a.im - a.re * r) / d};
  } else {
    double r = b.re / b.im, d = b.re * r + b.im;
    return cplx{(a.re * r + a.im) / d, (a.im * r - a.re) / d};
  }
}

// ---------------------------------------------------------------------------
// Per-mode linear operators
// ---------------------------------------------------------------------------
// RSW L (rsw/RotatingShallowWater.jl:242-260, D = -ν Krsq^nν at :263/277)
__host__ __device__ inline void rsw_L(const Phys& p, double k, double l, cplx L[3][3]) {
#pragma clang fp contract(off)
  const double D = -(p.nu * ipow(k * k + l * l, p.nnu));
  L[0][0] = cx(D);           L[0][1] = cx(p.f);          L[0][2] = cx(0.0, -k * p.Cg2);
  L[1][0] = cx(-p.f);        L[1][1] = cx(D);            L[1][2] = cx(0.0, -l * p.Cg2);
  L[2][0] = cx(0.0, -k);     L[2][1] = cx(0.0, -l);      L[2][2] = cx(D);
}

// QG2 L (swqg/TwoLayerQG.jl:184-198) with the Complex{Float32} literal quirk
// (SURVEY A11): PV_term, drag_term and the Sinv numerators are rounded to fp32.
__host__ __device__ inline void qg2_L(const Phys& p, double k, double l, cplx L[2][2]) {
#pragma clang fp contract(off)
  const double K2 = k * k + l * l;
  const double K2inv = (K2 == 0.0) ? 0.0 : 1.0 / K2;
  const double pv1 = (double)(float)(((-2.0 * k) * p.F) * p.U);
  const double pv2 = (double)(float)(((2.0 * k) * p.F) * p.U);
  const double drag2 = (double)(float)(p.mu * K2);
  const double a = (double)(float)((-K2) - p.F);
  const double b = (double)(float)(-p.F);
  const double den = K2 + 2.0 * p.F;
  const double Saa = (a / den) * K2inv, Sab = (b / den) * K2inv;
  // psi_terms = (0 + i pv1, drag2 + i pv2) ; L[r][c] = psi[r] * S[r][c]
  L[0][0] = cx(0.0 * Saa, pv1 * Saa);
  L[0][1] = cx(0.0 * Sab, pv1 * Sab);
  L[1][0] = cx(drag2 * Sab, pv2 * Sab);
  L[1][1] = cx(drag2 * Saa, pv2 * Saa);
  const double D = -(p.nu * ipow(K2, p.nnu));
  L[0][0] = cx(L[0][0].re + D, L[0][0].im + (-k * p.U));
  L[1][1] = cx(L[1][1].re + D, L[1][1].im + (k * p.U));
}

// ---------------------------------------------------------------------------
// Matrix exponential of a small complex matrix: Padé-13 scaling and squaring
// (Higham 2005), the algorithm behind Julia's exp for matrices that
// utils/IFMAB3.jl:26-41 calls per mode.
// ---------------------------------------------------------------------------
template <int n>
__host__ __device__ inline void mm(const cplx A[n][n], const cplx B[n][n], cplx C[n][n]) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      cplx s = cx(0.0);
      for (int k = 0; k < n; ++k) s = s + A[i][k] * B[k][j];
      C[i][j] = s;
    }
}

template <int n>
__host__ __device__ inline void expm(const cplx Ain[n][n], cplx E[n][n]) {
  const double b[14] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                        1187353796428800.0,  129060195264000.0,   10559470521600.0,
                        670442572800.0,      33522128640.0,       1323241920.0,
                        40840800.0,          960960.0,            16380.0,
                        182.0,               1.0};
  const double theta13 = 5.371920351148152;
  double nrm = 0.0;  // 1-norm
  for (int j = 0; j < n; ++j) {
    double c = 0.0;
    for (int i = 0; i < n; ++i) c += hypot(Ain[i][j].re, Ain[i][j].im);
    nrm = c > nrm ? c : nrm;
  }
  int s = 0;
  if (nrm > theta13) s = (int)ceil(log2(nrm / theta13));
  const double sc = ldexp(1.0, -s);
  cplx A[n][n], A2[n][n], A4[n][n], A6[n][n], T[n][n], Uo[n][n], V[n][n];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) A[i][j] = sc * Ain[i][j];
  mm<n>(A, A, A2);
  mm<n>(A2, A2, A4);
  mm<n>(A4, A2, A6);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) T[i][j] = b[13] * A6[i][j] + b[11] * A4[i][j] + b[9] * A2[i][j];
  mm<n>(A6, T, Uo);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      Uo[i][j] = Uo[i][j] + b[7] * A6[i][j] + b[5] * A4[i][j] + b[3] * A2[i][j];
      if (i == j) Uo[i][j] = Uo[i][j] + cx(b[1]);
    }
  mm<n>(A, Uo, T);  // T = U
  cplx W[n][n];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) W[i][j] = b[12] * A6[i][j] + b[10] * A4[i][j] + b[8] * A2[i][j];
  mm<n>(A6, W, V);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      V[i][j] = V[i][j] + b[6] * A6[i][j] + b[4] * A4[i][j] + b[2] * A2[i][j];
      if (i == j) V[i][j] = V[i][j] + cx(b[0]);
    }
  // solve (V - U) X = (V + U) by Gaussian elimination with partial pivoting
  cplx P[n][n], Q[n][n];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      P[i][j] = V[i][j] - T[i][j];
      Q[i][j] = V[i][j] + T[i][j];
    }
  for (int c = 0; c < n; ++c) {
    int piv = c;
    double best = hypot(P[c][c].re, P[c][c].im);
    for (int r = c + 1; r < n; ++r) {
      double v = hypot(P[r][c].re, P[r][c].im);
      if (v > best) { best = v; piv = r; }
    }
    if (piv != c) {
      for (int j = 0; j < n; ++j) {
        cplx t1 = P[c][j]; P[c][j] = P[piv][j]; P[piv][j] = t1;
        cplx t2 = Q[c][j]; Q[c][j] = Q[piv][j]; Q[piv][j] = t2;
      }
    }
    for (int r = c + 1; r < n; ++r) {
      cplx fct = cdiv(P[r][c], P[c][c]);
      for (int j = c; j < n; ++j) P[r][j] = P[r][j] - fct * P[c][j];
      for (int j = 0; j < n; ++j) Q[r][j] = Q[r][j] - fct * Q[c][j];
    }
  }
  for (int c = n - 1; c >= 0; --c) {
    for (int j = 0; j < n; ++j) {
      cplx s2 = Q[c][j];
      for (int k = c + 1; k < n; ++k) s2 = s2 - P[c][k] * Q[k][j];
      Q[c][j] = cdiv(s2, P[c][c]);
    }
  }
  for (int it = 0; it < s; ++it) {
    mm<n>(Q, Q, T);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) Q[i][j] = T[i][j];
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) E[i][j] = Q[i][j];
}

// ---------------------------------------------------------------------------
// launchers (sw_kernels.hip)
// ---------------------------------------------------------------------------
struct Bufs;  // fwd

void launch_col_inv(int model, const Geom& g, const Phys& p, const double2* X, double2* Minv,
                    const double2* tw_y, hipStream_t s);
void launch_row(int model, const Geom& g, const Phys& p, const double2* Minv, double2* Mfwd,
                const double2* tw_x, hipStream_t s);
void launch_col_fwd(int model, const Geom& g, const Phys& p, const double2* Mfwd, double2* N,
                    const double2* tw_y, hipStream_t s);
// Pointers of one stepper stage (see sw_kernels.hip).
struct StepPtrs {
  const double2* sol;  // state in
  double2* sol_out;    // state out (FilteredAB3: the other buffer; else == sol)
  double2* h0;
  const double2* h1;
  const double2* h2;
  const double2* E;
  const double2* E2;
  double2* xs;        // IFMRK4 stages 1-3: the stage input written for the next calcN
  int euler;
  int stage;
};
enum { OP_FAB3 = 0, OP_IFMAB3 = 1, OP_RK4 = 2 };
void launch_col_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                     const double2* Mf, double2* Minv, const double2* tw_y, hipStream_t s);
void launch_step_elem(int nf, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                      const double2* N, double2* xs, hipStream_t s);
void launch_setup_expm(int model, const Geom& g, const Phys& p, double factor, double2* E,
                       hipStream_t s);
void launch_gather(int nf, const Geom& g, const double2* full, double2* compact, hipStream_t s);
void launch_scatter(int nf, const Geom& g, int lo, int hi, const double2* compact, double2* full,
                    hipStream_t s);
void launch_nan_check(int nf, const Geom& g, const double2* compact, int* flag, hipStream_t s);
void launch_make_spec(int model, int field_id, const Geom& g, const Phys& p, const double2* sol,
                      double2* out, hipStream_t s);
void launch_col_inv1(const Geom& g, const double2* X, double2* M, const double2* tw_y, hipStream_t s);
void launch_row_c2r1(const Geom& g, const double2* M, double* out, const double2* tw_x, hipStream_t s);
// energy sums of a compact state (sw_kernels.hip k_energy_cols): one triple
// per local column into cols[3 krl + 0..2]; k_energy_final adds ncols
// triples in order into out[0..2]
void launch_energy_cols(int model, const Geom& g, const Phys& p, const double2* sol, double* cols,
                        hipStream_t s);
void launch_energy_final(const double* cols, int ncols, double* out, hipStream_t s);
void launch_absmax(const double* f, long long n, unsigned long long* out, hipStream_t s);

}  // namespace sw
