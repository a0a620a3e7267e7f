// Shared host/device definitions for libsw (not part of the public ABI).
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

// The SW_EXP_* knobs time the cost of one resource by removing it and give
// wrong results by design: only experiment builds (-DSW_EXPERIMENTS,
// tools/build_variants.sh) may define them; a production translation unit
// cannot compile them in.
#if !defined(SW_EXPERIMENTS) &&                                                                   \
    (defined(SW_EXP_NOHBM) || defined(SW_EXP_NOLOAD) || defined(SW_EXP_NOSTORE) ||                \
     defined(SW_EXP_CS_NOMIX) || defined(SW_EXP_CS_NOUPD) || defined(SW_EXP_NOBAR) ||             \
     defined(SW_EXP_NOTW) || defined(SW_EXP_NOLDS) || defined(SW_EXP_NOFILT))
#error "SW_EXP_* knobs give wrong results: experiment builds only (-DSW_EXPERIMENTS)"
#endif

// No implicit FMA contraction in libsw: the same formula rounds the same way
// in every kernel (and on the host), so kernel fusion never changes results.
#pragma clang fp contract(off)

// Short lines (N/8 threads each) are packed into blocks of up to this many
// threads (kernels and host geometry must agree).  64: one
// line per block from N = 512 up, the most blocks on small grids (measured,
// sw_kernels.hip row_tgt)
#ifndef SW_BLK_THREADS
#define SW_BLK_THREADS 64
#endif

// Parseval sums per energy evaluation (k_energy_cols; 3 for RSW/QG2/MLQG,
// 7 for TY with its wave/balanced split)
#define SW_NSUM 7

#include <hip/hip_ext.h>

namespace sw {

// sw_profile_steps' kernel timing (sw_api.cpp Timer): while `stop` is set,
// every launch is a hipExtLaunchKernel whose events take the dispatch's own
// start/end timestamps — the first launch of a timed scope `start`, each
// launch `stop` (the last one holds) — so a scope's interval is its kernels'
// execution, as the kernel trace reports it, without the event markers'
// own packets in it.
struct ProfEv {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local ProfEv prof_ev;
#define SW_LAUNCH(k, gr, bl, sh, st, ...)                                                             \
  do {                                                                                               \
    if (::sw::prof_ev.stop) {                                                                        \
      hipExtLaunchKernelGGL(k, gr, bl, sh, st, ::sw::prof_ev.start, ::sw::prof_ev.stop, 0, __VA_ARGS__); \
      ::sw::prof_ev.start = nullptr;                                                                 \
    } else {                                                                                         \
      hipLaunchKernelGGL(k, gr, bl, sh, st, __VA_ARGS__);                                            \
    }                                                                                                \
  } while (0)

// MODEL_MLQG (GeophysicalFlows MultiLayerQG, 2 layers) runs the MODEL_QG2
// kernels; Phys::model selects its streamfunction and linear terms at run time
enum { MODEL_RSW = 0, MODEL_QG2 = 1, MODEL_TY = 2, MODEL_MLQG = 3 };
// kernel family only: RSW's calcN in the reference's advective form
// (aliased_fraction = 0, where the vorticity form of MODEL_RSW is not exact)
enum { MODEL_RSWA = 4 };
enum { ST_FAB3 = 0, ST_IFMAB3 = 1, ST_IFMRK4 = 2, ST_ETDRK4 = 3, ST_FRK4 = 4 };

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
  int tcm;            // inverse mixed fields: column-major tiles (mtile_local)
  // forward mixed fields (A = 2^fa columns × B = 8/A rows per tile): line
  // stride per B rows and per A columns — (1, nyl/B): lines in column order
  // (one slab); (kcl/A, 1): in row order (several slabs: a chunk of rows is
  // contiguous per block, so the forward transposes can follow the row pass
  // chunk by chunk).  fa = 1 (2×4 tiles) but for the 2LQG half-length rows
  // at 8192 points (fa = 2: 4×2, sw_api.cpp make_geom)
  int fsy, fsk, fa;
  int isplit;         // 2LQG/MLQG/TY column inverse: one output per block (k_col_inv SPLIT)
  int rsplit;         // RSW/2LQG/MLQG/TY row over 2 / 4 blocks (k_row SPLIT)
  int rsp;            // RSW decimated row over 2 one-line blocks (k_row_rsw_sp, SW_ROW_SP)
};

struct Phys {
  double f, Cg2, nu;  // RSW
  int nnu;
  double U, mu, F;    // QG2
  double Ro;          // TY Rossby number
  int model;          // MODEL_* of the problem (MLQG shares the QG2 kernels)
  // MLQG: F1 = F (above), F2, per-layer mean flow and background PV gradient
  double F2, U1, U2, Qy1, Qy2;
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
// where L2 stitches the line.  Measured on MI355X at 2048² (tools/ab/sweep.sh,
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
// Inside a line: cm = 0 row-major (a row's A elements contiguous), cm = 1
// column-major (a column's B elements contiguous).  The inverse fields are
// written by the column pass and read by the row pass: column-major, each
// column block writes one contiguous 64-B half of every line it touches
// (row-major: four 16-B pieces, every 32-B sector partly written; where the
// neighbouring column's half arrives after the line left L2 the sectors go
// out twice).  Measured (MI355X, steps/s): RSW 2048² FilteredAB3 6226 →
// 6363 (col_step 87.8 → 85.7 µs), 1024² +0.7 %, 4096² +1.2 %, 2LQG 2048²
// IFMAB3 +1.2 %, 2LQG 8192² IFMRK4 60.5 → 63.0 (col_inv 1117 → 937 µs).
// Geom::tcm (SW_TILE_CM=0 selects row-major, for comparison); the forward
// fields, written by the row pass, are row-major.
template <int A, int ORD>
__host__ __device__ inline int mtile_local(const Geom& g, int krl, int yl, int cm = 0) {
  // (krl, yl) inside one slab-pair block of kcl columns × nyl rows
  constexpr int B = 8 / A;
  const int line = ORD == 0 ? (yl / B) * (g.kcl / A) + krl / A : (krl / A) * (g.nyl / B) + yl / B;
  return line * 8 + (cm ? (krl % A) * B + yl % B : (yl % B) * A + krl % A);
}
template <int A, int ORD>
__host__ __device__ inline int mtile_c(const Geom& g, int krl, int y, int cm = 0) {
  return (y >> g.log2nyl) * g.nyl * g.kcl + mtile_local<A, ORD>(g, krl, y & (g.nyl - 1), cm);
}
template <int A, int ORD>
__host__ __device__ inline int mtile_x(const Geom& g, int kr, int yl, int cm = 0) {
  int p = 0, krl = kr;
  if (g.nslab > 1) {
    p = kr / g.kcl;
    krl = kr - p * g.kcl;
  }
  return p * g.nyl * g.kcl + mtile_local<A, ORD>(g, krl, yl, cm);
}
// forward fields: row phase / column phase (A = 2^fa: tile and line order
// from Geom)
#if SW_TILE_F == 2
__host__ __device__ inline int mtile_f_local(const Geom& g, int krl, int yl) {
  const int fb = 3 - g.fa;
  return ((yl >> fb) * g.fsy + (krl >> g.fa) * g.fsk) * 8 + ((yl & ((1 << fb) - 1)) << g.fa) +
         (krl & ((1 << g.fa) - 1));
}
__host__ __device__ inline int midx(const Geom& g, int kr, int yl) {
  int p = 0, krl = kr;
  if (g.nslab > 1) {
    p = kr / g.kcl;
    krl = kr - p * g.kcl;
  }
  return p * g.nyl * g.kcl + mtile_f_local(g, krl, yl);
}
__host__ __device__ inline int midc(const Geom& g, int krl, int y) {
  return (y >> g.log2nyl) * g.nyl * g.kcl + mtile_f_local(g, krl, y & (g.nyl - 1));
}
#else
__host__ __device__ inline int midx(const Geom& g, int kr, int yl) { return mtile_x<SW_TILE_F, SW_LORD_F>(g, kr, yl); }
__host__ __device__ inline int midc(const Geom& g, int krl, int y) { return mtile_c<SW_TILE_F, SW_LORD_F>(g, krl, y); }
#endif
// Aliased-state tracking: the row pass's x-spectra kr in [kc, nx/2] of its
// NFA forward outputs (Ma).  One block per slab q of the stored rows,
// [q][f][kr - kc][yl] (stored row m = q nyl + yl), so that one slab's rows
// are one contiguous piece (one all-gather assembles them on the slab holding
// the aliased columns, sw_api.cpp); one slab: [f][kr - kc][y].  Field f of
// block q starts at Ma + ma_off(g, NFA, 0, q nyl) + f · ma_field(g).
__host__ __device__ inline long long ma_field(const Geom& g) { return (long long)(g.nkr - g.kc) * g.nyl; }
__host__ __device__ inline long long ma_off(const Geom& g, int nfa, int col, int m) {
  const int q = m >> g.log2nyl, yl = m & (g.nyl - 1);
  return ((long long)q * nfa * (g.nkr - g.kc) + col) * g.nyl + yl;
}
// fields of Ma per kernel family (the row pass's forward outputs)
__host__ __device__ constexpr int ma_nfa(int model) { return model == MODEL_TY ? 7 : 4; }

// inverse fields: column phase / row phase
__host__ __device__ inline int midc_i(const Geom& g, int krl, int y) { return mtile_c<SW_TILE_I, SW_LORD_I>(g, krl, y, g.tcm); }
__host__ __device__ inline int midx_i(const Geom& g, int kr, int yl) { return mtile_x<SW_TILE_I, SW_LORD_I>(g, kr, yl, g.tcm); }

// integer power x^n (0 <= n < 256, sw_create checks) by repeated squaring:
// the products of the loop `while (n) { if (n & 1) r *= x; x *= x; n >>= 1; }`
// in the same order, unrolled over 8 bits with selects, so the update
// kernels have no control flow here (loads of several modes issue together)
__host__ __device__ inline double ipow(double x, int n) {
  double r = 1.0;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    r = ((n >> b) & 1) ? r * x : r;
    x = x * x;
  }
  return r;
}

// FF makefilter value at (k, l): K = sqrt((k dx/π)² + (l dy/π)²),
// filt = exp(-decay (K-innerK)^order) for K >= innerK, else 1.
__host__ __device__ inline double filter_value(const Geom& g, const Phys& p, double k, double l) {
#pragma clang fp contract(off)
#ifdef SW_EXP_NOFILT  // experiment: filter evaluation cost (wrong results)
  return 1.0 + k * l;
#endif
  const double a = k * g.dx / 3.14159265358979323846, b = l * g.dy / 3.14159265358979323846;
  const double K = sqrt(a * a + b * b);
#ifdef SW_FILT_SELECT
  const double f = exp(-p.decay * ipow(K - p.innerK, p.forder));
  return K < p.innerK ? 1.0 : f;  // select, no branch
#else
  // exp only where the filter acts (a wave whose modes are all inside
  // innerK skips it: most waves of the low-wavenumber columns)
  double f = 1.0;
  if (K >= p.innerK) f = exp(-p.decay * ipow(K - p.innerK, p.forder));
  return f;
#endif
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

// Streamfunction of layer `layer` from the PV pair at K² (0 at K = 0):
//  2LQG streamfunctionfrompv! (swqg/TwoLayerQG.jl:101-111, its op order);
//  MLQG ψ̂ = S⁻¹ q̂, S⁻¹ = [[-(K²+F₂), -F₁], [-F₂, -(K²+F₁)]] / (K²(K²+F₁+F₂))
__host__ __device__ inline void qg_psi(const Phys& p, double K2, double q1r, double q1i, double q2r, double q2i,
                                       int layer, double& pr, double& pi) {
#pragma clang fp contract(off)
  if (p.model == MODEL_MLQG) {
    const double inv = K2 == 0.0 ? 0.0 : 1.0 / (K2 * (K2 + p.F + p.F2));
    if (layer == 0) {
      pr = (-(K2 + p.F2) * q1r - p.F * q2r) * inv;
      pi = (-(K2 + p.F2) * q1i - p.F * q2i) * inv;
    } else {
      pr = (-p.F2 * q1r - (K2 + p.F) * q2r) * inv;
      pi = (-p.F2 * q1i - (K2 + p.F) * q2i) * inv;
    }
    return;
  }
  const double iK2 = K2 == 0.0 ? 0.0 : 1.0 / K2;
  const double den = K2 + 2.0 * p.F;
  const double qsr = q1r + q2r, qsi = q1i + q2i;
  const double qgr = layer ? q2r : q1r, qgi = layer ? q2i : q1i;
  pr = (-(K2 * qgr + p.F * qsr) / den) * iK2;
  pi = (-(K2 * qgi + p.F * qsi) / den) * iK2;
}

// ---------------------------------------------------------------------------
// Per-mode integrating factors exp(τ L) (utils/IFMAB3.jl:26-41 computes them
// with Julia's matrix exp per mode and stores E, E2 arrays).  libsw evaluates
// them in closed form on the fly inside the stepper update instead — exact
// up to rounding, like the reference's Padé-13 — so no (nf×nf) operator
// planes are stored or streamed from HBM (36 F per RSW IFMAB3 step).
// ---------------------------------------------------------------------------
__host__ __device__ inline cplx cconj_(cplx a) { return cplx{a.re, -a.im}; }
__host__ __device__ inline cplx cexp_(cplx z) {
  const double e = exp(z.re);
  return cplx{e * cos(z.im), e * sin(z.im)};
}
__host__ __device__ inline cplx csqrt_(cplx z) {
  const double r = hypot(z.re, z.im);
  if (r == 0.0) return cplx{0.0, 0.0};
  double a = sqrt(0.5 * (r + fabs(z.re))), b = 0.5 * z.im / a;
  if (z.re < 0.0) {
    const double t = a;
    a = fabs(b);
    b = (z.im < 0.0 ? -t : t);
  }
  return cplx{a, b};
}

// RSW (rsw/RotatingShallowWater.jl:242-260): L = D I + A with the scalar
// D = -ν K^(2nν) and A = [[0, f, -ik Cg²], [-f, 0, -il Cg²], [-ik, -il, 0]],
// whose characteristic polynomial is λ³ + ω² λ (ω² = f² + Cg² K²), so
//   exp(τ L) = e^(Dτ) (I + sin(ωτ)/ω A + 2 sin²(ωτ/2)/ω² A²).
struct RswExp {
  double k, l, e, s, c;
};
__host__ __device__ inline RswExp rsw_exp(const Phys& p, double k, double l, double tau) {
#pragma clang fp contract(off)
  const double K2 = k * k + l * l;
  const double D = -(p.nu * ipow(K2, p.nnu));
  const double w = sqrt(p.f * p.f + p.Cg2 * K2);
  RswExp E;
  E.k = k;
  E.l = l;
  E.e = exp(D * tau);
  if (w * tau < 1e-8) {  // A ≈ 0 (f = 0, K = 0): series limits
    E.s = tau;
    E.c = 0.5 * tau * tau;
  } else {
    const double h = sin(0.5 * w * tau);
    E.s = sin(w * tau) / w;
    E.c = 2.0 * h * h / (w * w);
  }
  return E;
}
__host__ __device__ inline void rsw_A_mul(const Phys& p, double k, double l, const cplx x[3], cplx y[3]) {
#pragma clang fp contract(off)
  // y = A x (complex entries -ik Cg², -il Cg², -ik, -il applied as i·(real))
  y[0] = cx(p.f * x[1].re + k * p.Cg2 * x[2].im, p.f * x[1].im - k * p.Cg2 * x[2].re);
  y[1] = cx(-p.f * x[0].re + l * p.Cg2 * x[2].im, -p.f * x[0].im - l * p.Cg2 * x[2].re);
  y[2] = cx(k * x[0].im + l * x[1].im, -(k * x[0].re) - l * x[1].re);
}
__host__ __device__ inline void exp_apply(const Phys& p, const RswExp& E, const cplx x[3], cplx y[3]) {
#pragma clang fp contract(off)
  cplx a[3], b[3];
  rsw_A_mul(p, E.k, E.l, x, a);
  rsw_A_mul(p, E.k, E.l, a, b);
  for (int r = 0; r < 3; ++r) {
    const cplx t = x[r] + E.s * a[r] + E.c * b[r];
    y[r] = E.e * t;
  }
}

// 2LQG (swqg/TwoLayerQG.jl:184-206, incl. the Float32 literals of qg2_L):
// M = τL = m I + B with m = τ tr(L)/2, B traceless, B² = δ² I,
//   exp(M) = e^m (cosh δ I + sinh(δ)/δ B).
struct Qg2Exp {
  cplx E[2][2];
};
// cosh z and sinh(z)/z: for |z| < 0.5 their Taylor series to z^20 (no
// transcendental; the terms past it are < 1e-24), else from sinh/cosh of z.re
// and sin/cos of z.im
__host__ __device__ inline void ccosh_sinhc(cplx z, cplx& ch, cplx& sc) {
#pragma clang fp contract(off)
  if (z.re * z.re + z.im * z.im < 0.25) {
    const cplx z2 = z * z;
    cplx rs = cx(1.0), ts = cx(1.0), rc = cx(1.0), tc = cx(1.0);
    for (int n = 1; n <= 10; ++n) {
      ts = (1.0 / ((2.0 * n) * (2.0 * n + 1.0))) * (ts * z2);  // z^(2n)/(2n+1)!
      tc = (1.0 / ((2.0 * n - 1.0) * (2.0 * n))) * (tc * z2);  // z^(2n)/(2n)!
      rs = rs + ts;
      rc = rc + tc;
    }
    sc = rs;
    ch = rc;
    return;
  }
  const double shr = sinh(z.re), chr = cosh(z.re), sn = sin(z.im), cs = cos(z.im);
  ch = cx(chr * cs, shr * sn);
  sc = cdiv(cx(shr * cs, chr * sn), z);
}
__host__ __device__ inline Qg2Exp qg2_exp(const Phys& p, double k, double l, double tau) {
#pragma clang fp contract(off)
  cplx L[2][2];
  qg2_L(p, k, l, L);
  const cplx m = (0.5 * tau) * (L[0][0] + L[1][1]);
  const cplx b00 = (0.5 * tau) * (L[0][0] - L[1][1]);
  const cplx b01 = tau * L[0][1], b10 = tau * L[1][0];
  const cplx d = csqrt_(b00 * b00 + b01 * b10);
  // tr L is real for the 2LQG operator (pv₂ = -pv₁, ∓kU): e^m without the
  // sin/cos of 0 (cos 0 = 1 and sin 0 = 0 exactly)
  const cplx em = m.im == 0.0 ? cx(exp(m.re), 0.0) : cexp_(m);
  cplx ch, sc;
  ccosh_sinhc(d, ch, sc);
  Qg2Exp X;
  X.E[0][0] = em * (ch + sc * b00);
  X.E[1][1] = em * (ch - sc * b00);
  X.E[0][1] = em * (sc * b01);
  X.E[1][0] = em * (sc * b10);
  return X;
}
__host__ __device__ inline void exp_apply(const Phys&, const Qg2Exp& X, const cplx x[2], cplx y[2]) {
#pragma clang fp contract(off)
  y[0] = X.E[0][0] * x[0] + X.E[0][1] * x[1];
  y[1] = X.E[1][0] * x[0] + X.E[1][1] * x[1];
}

// exp(2τL) from exp(τL): RSW re-evaluates its cheap closed form; 2LQG squares
// the 2×2 matrix (one evaluation of the complex transcendental form per mode)
__host__ __device__ inline RswExp exp_double(const Phys& p, const RswExp& E, double tau) {
  return rsw_exp(p, E.k, E.l, 2.0 * tau);
}
__host__ __device__ inline Qg2Exp exp_double(const Phys&, const Qg2Exp& X, double) {
#pragma clang fp contract(off)
  Qg2Exp Y;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) Y.E[i][j] = X.E[i][0] * X.E[0][j] + X.E[i][1] * X.E[1][j];
  return Y;
}

template <int NF>
struct ExpOf;
template <>
struct ExpOf<3> {
  using T = RswExp;
  __host__ __device__ static T make(const Phys& p, double k, double l, double tau) { return rsw_exp(p, k, l, tau); }
};
template <>
struct ExpOf<2> {
  using T = Qg2Exp;
  __host__ __device__ static T make(const Phys& p, double k, double l, double tau) { return qg2_exp(p, k, l, tau); }
};

// ---------------------------------------------------------------------------
// launchers (sw_kernels.hip)
// ---------------------------------------------------------------------------
struct Bufs;  // fwd

// column-pass launches over a range of groups (col_inv: output groups, see
// k_col_inv; col_fwd / col_step: fields); n < 0 = from the first to the last
int col_inv_groups(int model);
int col_fields(int model);
// transform length 2^log2n instantiated in this build (a one-length
// experiment build, SW_ONLY_LOG2, holds one; sw_create rejects the others)
bool length_built(int log2n);
void launch_col_inv(int model, const Geom& g, const Phys& p, const double2* X, double2* Minv,
                    const double2* tw_y, hipStream_t s, int g0 = 0, int ng = -1);
// local rows [y0, y0 + nrows) (nrows < 0: to the last); nrows a multiple of
// row_lines_per_block (and of 4, the mixed tiles' height)
// Ma (2LQG on lines up to 4096, or RSW's advective form; one slab): also the
// x-spectra k in [kc, nx/2] of the forward fields, [field][k - kc][y] (the
// aliased-state tracking)
void launch_row(int model, const Geom& g, const Phys& p, const double2* Minv, double2* Mfwd,
                const double2* tw_x, hipStream_t s, int y0 = 0, int nrows = -1, double2* Ma = nullptr);
bool row_alias_built(int model, int log2nx);
// N at the aliased modes of region ga (sw_api.cpp alias_geom; model QG2 or
// RSWA): region 0 the columns kr >= kc from the row pass's Ma, region 1 the
// aliased rows of the live columns from the forward mixed fields Mfwd; N
// compact in ga
void launch_col_fwd_alias(int model, const Geom& g, const Geom& ga, int region, const Phys& p, const double2* Mfwd,
                          const double2* Ma, double2* N, const double2* tw_y, hipStream_t s);
// compact modes of ga <-> the full (nkr, nl, nf) array (only those modes)
void launch_scatter_modes(int nf, const Geom& ga, const double2* compact, double2* full, hipStream_t s);
void launch_gather_modes(int nf, const Geom& ga, const double2* full, double2* compact, hipStream_t s);
int row_lines_per_block(int model, int log2nx);
// X: the compact calcN input (TY adds its linear terms from it; unused otherwise)
// T1, T2 (short columns, sw_api.cpp fsplit): one term of N per block, terms
// 1-2 into T1 / T2, completed by the consuming update (StepPtrs nt1, nt2)
void launch_col_fwd(int model, const Geom& g, const Phys& p, const double2* Mfwd, double2* N,
                    const double2* X, const double2* tw_y, hipStream_t s, int f0 = 0, int nfl = -1,
                    double2* T1 = nullptr, double2* T2 = nullptr);
// Pointers of one stepper stage (see sw_kernels.hip).
struct StepPtrs {
  const double2* sol;  // state in
  double2* sol_out;    // state out (FilteredAB3: the other buffer; else == sol)
  double2* h0;
  const double2* h1;
  const double2* h2;
  double2* xs;        // IFMRK4 stages 1-3: the stage input written for the next calcN
  int euler;
  int stage;
  int stream;  // state/history accesses non-temporal (step traffic beyond the Infinity Cache)
  // ETDRK4 (FF ETDRK4TimeStepper): N₁, N₂, the second stage input s₂ and
  // the per-mode coefficient table [E, E2, ζ, α, β, Γ][cfield]
  double2* n1;
  double2* n2;
  double2* xs2;
  const double* etd;
  // a split N (launch_col_fwd T1/T2): its terms 1-2 and the calcN input for
  // the linear terms, completed per mode before the op (assemble_terms)
  const double2* nt1;
  const double2* nt2;
  const double2* xin;
  // sw_step's NaN/Inf scan folded into the update: the ops
  // that store the new state set *nan when one of its live values is not
  // finite (nullptr: no scan — the aliased-mode updates, profiling)
  int* nan;
};
enum { OP_FAB3 = 0, OP_IFMAB3 = 1, OP_RK4 = 2, OP_ETDRK4 = 3, OP_FRK4 = 4 };
enum { ETD_E = 0, ETD_E2, ETD_ZETA, ETD_ALPHA, ETD_BETA, ETD_GAMMA, ETD_N };
void launch_col_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                     const double2* Mf, double2* Minv, const double2* tw_y, hipStream_t s, int f0 = 0,
                     int nfl = -1);
// the launches of one transform length L = log2 N (sw_kernels.hip; one
// translation unit per length in the split build, dispatched by log2 N)
template <int L>
struct LenOps {
  static void col_inv(int model, const Geom& g, const Phys& p, const double2* X, double2* M, const double2* tw,
                      hipStream_t s, int g0, int ng);
  static void row(int model, const Geom& g, const Phys& p, const double2* Mi, double2* Mo, const double2* tw,
                  hipStream_t s, int y0, int nrows, double2* Ma);
  static void col_fwd_alias(int model, const Geom& g, const Geom& ga, int region, const Phys& p,
                            const double2* Mf, const double2* Ma, double2* N, const double2* tw, hipStream_t s);
  static void col_fwd(int model, const Geom& g, const Phys& p, const double2* Mf, double2* N, const double2* X,
                      const double2* tw, hipStream_t s, int f0, int nfl, double2* T1, double2* T2);
  static void col_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a, const double2* Mf,
                       double2* Minv, const double2* tw, hipStream_t s, int f0, int nfl);
  static void col_fwd_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a, const double2* Mf,
                           const double2* tw, hipStream_t s, bool lds);
  static size_t fwd_step_lds_bytes(int model, const Geom& g);
  static void col_inv1(const Geom& g, const double2* X, double2* M, const double2* tw, hipStream_t s);
  static void row_c2r1(const Geom& g, const double2* M, double* out, const double2* tw, hipStream_t s);
};
// k_col_fwd + k_step_elem in one column pass (all fields of a column per
// block, N in registers): RSW IFMAB3/IFMRK4, 2LQG FilteredAB3/IFMAB3/IFMRK4
// lds: N parked in LDS, the update loop rolled (k_col_fwd_step_lds), needs
// fwd_step_lds_bytes(model, g) of LDS per block
void launch_col_fwd_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                         const double2* Mf, const double2* tw_y, hipStream_t s, bool lds = false);
size_t fwd_step_lds_bytes(int model, const Geom& g);
void launch_step_elem(int nf, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                      const double2* N, double2* xs, hipStream_t s);
// a split N completed in place (a.nt1, a.nt2, a.xin)
void launch_assemble_terms(int nf, const Geom& g, const Phys& p, const StepPtrs& a, double2* N, hipStream_t s);
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
// max |f| (sgn = 0) or max f (sgn = 1) as an order-preserving integer key
void launch_absmax(const double* f, long long n, unsigned long long* out, int sgn, hipStream_t s);
// fp32 caller buffers (SW_PREC_F32): n reals widened / rounded
void launch_widen(const float* in, double* out, long long n, hipStream_t s);
void launch_narrow(const double* in, float* out, long long n, hipStream_t s);
// ETDRK4 coefficient table of the real diagonal L = -ν K^(2nν) (FF getetdcoeffs)
void launch_etd_coeffs(const Geom& g, const Phys& p, double* etd, hipStream_t s);

}  // namespace sw
