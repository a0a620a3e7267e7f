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

// Cache policy.  A step streams ≈ 2.5× the 256 MB Infinity Cache (MALL) at
// 2048²; what is worth keeping there is a mixed field between the kernel
// that writes it and the next one, which reads it.  Data read or written
// once per step (the stepper state and history) and mixed fields once read
// go non-temporal, so they do not evict the mixed fields in flight.
__device__ __forceinline__ double2 ld_nt(const double2* p) {
  return make_double2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
}
__device__ __forceinline__ void st_nt(double2* p, double2 v) {
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
}
// stepper state / history (read and written once per step): non-temporal
// when NT — the launchers set it (StepPtrs::stream) where a step's traffic
// exceeds what the Infinity Cache holds (sw_api.cpp); below that the state
// itself stays cached from one step to the next and temporal wins (1024²
// FilteredAB3: 19.2k temporal vs 17.6k non-temporal steps/s; 2048²: 5.5k vs
// 5.9k).  SW_STATE_T forces temporal (experiments).
template <bool NT>
__device__ __forceinline__ double2 state_ld(const double2* p) {
#ifndef SW_STATE_T
  if constexpr (NT) return ld_nt(p);
#endif
  return *p;
}
template <bool NT>
__device__ __forceinline__ void state_st(double2* p, double2 v) {
#ifndef SW_STATE_T
  if constexpr (NT) {
    st_nt(p, v);
    return;
  }
#endif
  *p = v;
}
// sw_step's blow-up check (rsw/RSWDriver.jl:213-218) at the store of the new
// state, whose values are in registers there: one flag per call instead of a
// separate pass over the state after the steps (k_nan_check, 44.8 MB at
// 2048²).  `bad` = some value this lane stored is not finite; the first such
// active lane of the wave stores 1 (a plain vector store: every writer writes
// the same value, and the flag may be pinned host memory, sw_api.cpp hflag).
__device__ __forceinline__ bool nonfinite(double2 v) { return !isfinite(v.x) || !isfinite(v.y); }
__device__ __forceinline__ bool nonfinite(cplx v) { return !isfinite(v.re) || !isfinite(v.im); }
__device__ __forceinline__ void note_nonfinite(int* flag, bool bad) {
  if (flag == nullptr) return;
  const unsigned long long m = __ballot(bad);
  if (m != 0ull && (int)__lane_id() == __ffsll((long long)m) - 1)
    __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int NF>
__device__ __forceinline__ void note_state(const StepPtrs& a, const cplx* x) {
  bool bad = false;
#pragma unroll
  for (int f = 0; f < NF; ++f) bad |= nonfinite(x[f]);
  note_nonfinite(a.nan, bad);
}

// mixed-field reads: the row pass's inverse inputs, the column pass's
// forward inputs (read once; their writer's stores stay temporal)
__device__ __forceinline__ double2 mix_ld_row(const double2* p) {
#ifdef SW_MIX_NT_ROW
  return ld_nt(p);
#else
  return *p;
#endif
}
__device__ __forceinline__ double2 mix_ld_col(const double2* p) {
#ifdef SW_MIX_NT_COL
  return ld_nt(p);
#else
  return *p;
#endif
}

// MultiLayerQG calcN!'s terms linear in the calcN input q (layer grp): the
// mean flow and background gradient -ik U_j q_j - ik Qy_j ψ_j, and the
// bottom drag μ K² ψ_2 on the lower layer, added to the Jacobian part r.
// One definition for k_col_fwd and the fused forward + update passes, so
// both round alike.
__device__ __forceinline__ double2 mlqg_linear_terms(const Phys& p, double k, double l, double2 q1, double2 q2,
                                                     int grp, double2 r) {
#pragma clang fp contract(off)
  const double K2 = k * k + l * l;
  double2 ps;
  qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, grp, ps.x, ps.y);
  const double2 qg = grp ? q2 : q1;
  r = csub(csub(r, cmul_i(qg, k * (grp ? p.U2 : p.U1))), cmul_i(ps, k * (grp ? p.Qy2 : p.Qy1)));
  if (grp == 1) r = cadd(r, cscale(ps, p.mu * K2));
  return r;
}

// block -> line mapping.  When one line per block and the grid is a multiple
// of 64, the 8 lines (columns, or rows in the row pass) that share each 128-B
// chunk of a mixed layout are placed on blocks b, b+8, …, b+56, which the
// dispatcher deals to one XCD, so they meet in one L2 (speed only).
__device__ __forceinline__ int col_of_block(int b, int nb) {
  if ((nb & 63) == 0) {
    const int q = b >> 6, j = (b >> 3) & 7, x = b & 7;
    return (q << 6) + (x << 3) + j;
  }
  return b;
}

// Row pass with two rows per block (RSW, nx = 1024): the four rows that share
// the 128-B lines of a 2×4 mixed tile span two blocks; dealt in dispatch
// order they would land on two XCDs, and each XCD's L2 would fetch the lines
// (round 2 PMC: the 1024² row read 2.1× its bytes).  With the grid a multiple
// of 16, blocks b and b+8 (one XCD label) take the two row pairs of a tile
// row group (speed only).  Returns the first row of block b.
template <int NB>
__device__ __forceinline__ int row0_of_block(int b, int nb) {
#ifndef SW_ROW_NOXCD
  if (NB == 2 && (nb & 15) == 0) {
    const int q = b >> 4, j = (b >> 3) & 1, x = b & 7;
    return ((q << 4) + (x << 1) + j) * 2;
  }
#endif
  return b * NB;
}

// Column-pass store offset of inverse-field element (krl, y = t + s NT): with
// one slab in closed form (A = 2, rows' lines contiguous: a per-thread term
// plus a per-s constant), otherwise midc_i
template <int NT>
__device__ __forceinline__ int midc_i_col_base(const Geom& g, int krl, int t) {
  asm volatile("" : "+v"(t));  // formed at the store, not hoisted over the kernel
  const int pos = g.tcm ? ((krl & 1) << 2) + (t & 3) : ((t & 3) << 1) + (krl & 1);
  return ((t >> 2) * (g.kcl >> 1) + (krl >> 1)) * 8 + pos;
}
template <int NT, typename F>
__device__ __forceinline__ void store_col_i(const Geom& g, int krl, int t, F put) {
  if (SW_TILE_I == 2 && SW_LORD_I == 0 && NT % 4 == 0 && g.nslab == 1) {
    const int b = midc_i_col_base<NT>(g, krl, t);
#pragma unroll
    for (int s = 0; s < 8; ++s) put(s, b + s * (NT >> 2) * (g.kcl >> 1) * 8);
  } else {
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int s = 0; s < 8; ++s) put(s, midc_i(g, krl, t + s * NT));
  }
}

// minimum waves per SIMD requested from the register allocator
#ifndef SW_MINW_FFT
#define SW_MINW_FFT 2
#endif
#define SW_MINW(L) (Blk<L>::THREADS >= 1024 ? 4 : SW_MINW_FFT)
// the column passes of the RSW/2LQG families: blocks of 512 threads (4096-
// point lines) at 4 waves per SIMD too (128 VGPRs: two blocks per CU; round 3,
// sw_fft.hpp SW_OPAQUE_LOG2); Thomas-Yamada's hold more per line and keep 2
#define SW_MINW_M(M, L) (Blk<L>::THREADS >= (M == MODEL_TY ? 1024 : 512) ? 4 : SW_MINW_FFT)
#ifndef SW_MINW_ROW
#define SW_MINW_ROW 2
#endif
#ifndef SW_MINW_ROW_QG  // the 2LQG/MultiLayerQG row
#define SW_MINW_ROW_QG 2
#endif

// threads per block: one line of NT = N/8 threads, or several short lines
// packed into 256 threads
template <int LOG2N, int TGT = SW_BLK_THREADS>
struct Blk {
  static constexpr int NT = FftPlan<LOG2N>::NT;
  // at most 32 lines, so that NB divides the local rows (>= 32) and the local
  // columns (a multiple of NB)
  static constexpr int NB = NT >= TGT ? 1 : (TGT / NT > 32 ? 32 : TGT / NT);
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

// ---------------------------------------------------------------------------
// Decimated column transforms (round 4).  From 2^SW_COL_DEC_MIN points the
// column passes' y-transforms are the wave-decimated ones (sw_fft.hpp:
// fftw_dif/fftw_dit for W = N/512 <= 8, fft16_dif/fft16_dit at 8192): one
// workgroup exchange per transform, the rest inside each wave.  Their
// physical-space side is in the decimated order, and the mixed fields keep it:
// slot s of thread t (wave w = t/64, lane j) is the stored row
//   p = 512 w + j + 64 s,   physical row y = (N/512) (p mod 512) + p / 512,
// contiguous across the lanes as the natural order's p = t + s NT.  The row
// pass is order-blind (it transforms whole stored rows; the slab exchange
// moves blocks of stored rows), so nothing else changes: k_col_inv writes
// that order (DIF: natural spectrum in), k_col_fwd / k_col_step read it (DIT:
// natural spectrum out); the physical-space output (k_col_inv1, k_row_c2r1)
// keeps the natural order.  Aliased-state tracking's row-pass x-spectra
// (Ma, indexed by the stored row) follow the same order.
// ---------------------------------------------------------------------------
#ifndef SW_COL_DEC_MIN
#define SW_COL_DEC_MIN 12
#endif
// the 2LQG/MultiLayerQG column kernels from 2048 points (config 3, 2LQG
// 2048² IFMAB3: col_fwd 30.0 -> 28.0 µs, 5332-5358 -> 5435-5583 steps/s; the
// RSW fused column step there: 82.4 -> 83.8 µs, so RSW keeps SW_COL_DEC_MIN;
// profiles/r04/ab_coldec.md)
#ifndef SW_COL_DEC_MIN_QG
#define SW_COL_DEC_MIN_QG 11
#endif
// MODEL: the kernel family whose column passes write and read the mixed
// fields (one order per family: its col_inv, col_fwd, col_step, alias pass)
template <int LOG2N, int MODEL = -1>
__host__ __device__ constexpr bool col_dec() {
  return LOG2N >= (MODEL == MODEL_QG2 ? SW_COL_DEC_MIN_QG : SW_COL_DEC_MIN) && LOG2N >= 10 && LOG2N <= 13;
}
// stored row of slot s of thread t
template <int LOG2N, bool DEC = col_dec<LOG2N>()>
__device__ __forceinline__ int cpos(int t, int s) {
  if constexpr (DEC) return ((t >> 6) << 9) + (t & 63) + (s << 6);
  else return t + s * FftPlan<LOG2N>::NT;
}
template <int LOG2N, bool DEC = col_dec<LOG2N>()>
struct ColTw {
  Twiddles<LOG2N> tws;
  __device__ __forceinline__ void load(int t, const double2* __restrict__ tw) { tws.load(t, tw); }
};
template <int LOG2N>
struct ColTw<LOG2N, true> {
  static constexpr bool FLY = LOG2N >= 12;
  Twiddles<9, FLY> tq;
  const double2* tab;
  __device__ __forceinline__ void load(int t, const double2* __restrict__ tw) {
    tq.load(t & 63, tw, LOG2N - 9);
    tab = tw;
  }
};
// the column passes' y-transform: DIR = +1 natural spectrum -> stored rows,
// DIR = -1 stored rows -> natural spectrum (v[s] = X[t + s NT])
template <int LOG2N, int DIR, bool DEC = col_dec<LOG2N>()>
__device__ __forceinline__ void col_fft(double2 (&v)[8], int t, const ColTw<LOG2N, DEC>& c, double2* __restrict__ line) {
  if constexpr (!DEC) {
    fft_line<LOG2N, DIR>(v, t, c.tws, line);
  } else if constexpr (LOG2N == 13) {
    if constexpr (DIR > 0) fft16_dif<DIR>(v, t, c.tq, c.tab, line);
    else fft16_dit<DIR>(v, t, c.tq, c.tab, line);
  } else {
    constexpr int W = 1 << (LOG2N - 9);
    constexpr bool FLY = ColTw<LOG2N, true>::FLY;
    using V1 = double2(&)[1][8];
    const double2 wt = c.tab[t];  // W_N^t, read per transform (not held)
    if constexpr (DIR > 0) fftw_dif<W, DIR, 1, true, FLY>(reinterpret_cast<V1>(v), t, wt, c.tq, line, 0);
    else fftw_dit<W, DIR, 1, FLY, true>(reinterpret_cast<V1>(v), t, wt, c.tq, line, 0);
  }
}
// the inverse-field stores of a column line at the stored rows cpos (as
// store_col_i: closed form with one slab)
template <int LOG2N, bool DEC = col_dec<LOG2N>(), typename F>
__device__ __forceinline__ void store_col_p(const Geom& g, int krl, int t, F put) {
  constexpr int PS = DEC ? 64 : FftPlan<LOG2N>::NT;  // stored-row stride of the slots
  if (SW_TILE_I == 2 && SW_LORD_I == 0 && PS % 4 == 0 && g.nslab == 1) {
    const int b = midc_i_col_base<PS>(g, krl, cpos<LOG2N, DEC>(t, 0));
#pragma unroll
    for (int s = 0; s < 8; ++s) put(s, b + s * (PS >> 2) * (g.kcl >> 1) * 8);
  } else {
    asm volatile("" : "+v"(t));
#pragma unroll
    for (int s = 0; s < 8; ++s) put(s, midc_i(g, krl, cpos<LOG2N, DEC>(t, s)));
  }
}

// ===========================================================================
// col_inv: for column kr, build the y-spectra the row pass needs, inverse FFT
// along y (scaled by 1/(nx ny), FF's normalised c2r), store to mixed space.
//   RSW  outputs (rsw/RotatingShallowWater.jl:147-214): 0 U, 1 V, 2 H, 3 Uy=il U
//        (the row pass forms ζ̂ = ik V - Uy itself: ik is constant along a row)
//   QG2  outputs (swqg/TwoLayerQG.jl:155-176):          0 Q1, 1 Q2, 2 Ψ1, 3 Ψ2, 4 Ψy1, 5 Ψy2
// grid: (columns, groups); RSW group f reads field f; QG2 group = layer.
// ===========================================================================
template <int MODEL>
__host__ __device__ constexpr int inv_split_per() { return MODEL == MODEL_QG2 ? 3 : 2; }
// SPLIT: one output per block — grid (columns, 3 × groups) for 2LQG /
// MultiLayerQG (a layer's q, ψ or ∂yψ), (columns, 2 × groups) for
// Thomas–Yamada and RSW (a group's one or two outputs) — so that small grids, whose
// one-line blocks are a single wave, put 2-3 times the waves on the chip (the
// same arithmetic per output; Geom::isplit, sw_api.cpp make_geom)
// The column kernels' live-row band at compile time (round 6): BAND = 1 the
// 2/3 rule (lc = N/3, lr2 = N − N/3 for every power-of-two column), 2
// aliased_fraction = 0 (lc = N/2, lr2 = N/2 + 1), 0 the run-time g.lc, g.lr2.
// A local copy of the geometry carries the constants into every inlined
// helper (compact_of, the slot tests), so wholly live or dead slots resolve at
// compile time.  Measured (tools/ab/r6_colband.sh, two interleaved rounds,
// bitwise equal on eight configurations): RSWDriver 512² IFMAB3 33077-33173 →
// 34640-34648 steps/s, TYdriver 512² 6797-6818 → 6920-6925, TwoLayerSimulation
// 512² 7518-7604 → 7664-7682, the headline 6570-6587 → 6597-6622 (col_step
// −1 µs), config 3 5662-5674 → 5715-5718, config 5 71.6 → 71.8-72.3 (col_inv
// 887 → 853 µs).  SW_COL_BAND=0: never (A/B).
#ifndef SW_COL_BAND
#define SW_COL_BAND 1
#endif
template <int LOG2N, int BAND>
__device__ __forceinline__ void band_fix(Geom& g) {
  constexpr int N = 1 << LOG2N;
  if constexpr (BAND == 1) {
    g.lc = N / 3;
    g.lr2 = N - N / 3;
  } else if constexpr (BAND == 2) {
    g.lc = N / 2;
    g.lr2 = N / 2 + 1;
  }
}

template <int MODEL, int LOG2N, bool SPLIT = false, int BAND = 0>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW_M(MODEL, LOG2N))
    k_col_inv(Geom g, Phys p, const double2* __restrict__ X, double2* __restrict__ M,
              const double2* __restrict__ tw, int gbase) {
  band_fix<LOG2N, BAND>(g);
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  int krl, grp;
  if (MODEL == MODEL_QG2 && gbase < 0) {
    // both layers, 1-D grid of 2*kcl blocks (NB == 1, kcl a multiple of 64):
    // the two layer blocks of a column are consecutive on one XCD label
    // (b % 8), so the second one's reads of q1, q2 (each layer needs both for
    // ψ) come from that L2 rather than HBM; the 8 columns sharing a 128-B
    // chunk of the mixed layout stay on one label (speed only)
    const int b = blockIdx.x, q = b >> 7, r = b & 127, x = r & 7, jj = r >> 3;
    grp = jj & 1;
    krl = (q << 6) + (x << 3) + (jj >> 1);
  } else {
    krl = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
    grp = gbase + (SPLIT ? (int)blockIdx.y / inv_split_per<MODEL>() : (int)blockIdx.y);
  }
  const int out = SPLIT ? (int)blockIdx.y % inv_split_per<MODEL>() : -1;  // -1: every output
  if (MODEL == MODEL_TY && out == 1 && grp == 3) return;  // (vc: one output)
  if ((MODEL == MODEL_RSW || MODEL == MODEL_RSWA) && out == 1 && !(grp == 0 || (MODEL == MODEL_RSWA && grp == 1)))
    return;  // (V, H: one output; the advective form's V: two)
  const bool live = krl < g.kcn;
  if (B::NB == 1 && !live) return;  // padding column: nobody reads it
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  constexpr bool CD = col_dec<LOG2N, MODEL>();  // the family's stored-row order
  ColTw<LOG2N, CD> tws;
  tws.load(c.t, tw);
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  const double k = (g.kr0 + krl) * g.mk;
  double2 v[8];

  auto store = [&](int o) {  // fft_line leaves Y[t + s*NT] in v[s]
    if (live) {
      double2* Mo = M + (long long)o * g.mfield;
      store_col_p<LOG2N, CD>(g, krl, c.t, [&](int s, int o) { Mo[o] = v[s]; });
    }
  };

  // loads are unconditional from a clamped in-bounds address, then selected:
  // a branch around each load would serialise them (one vmcnt(0) per element)
  const int krc = live ? krl : 0;
  if constexpr (MODEL == MODEL_RSW || MODEL == MODEL_RSWA) {
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
    if (out <= 0) {
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(grp);
    }
    if (out != 0 && (grp == 0 || (MODEL == MODEL_RSWA && grp == 1))) {  // ∂y u: Uy (advective form: and ∂y v: Vy)
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cmul_i(x[s], lwav(g, c.t + s * NT) * scale);
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(3 + grp);
    }
  } else if constexpr (MODEL == MODEL_TY) {
    // thomasyamada/ThomasYamada.jl:129-262.  Group → (input field, outputs):
    //   0: ζ  → 0 ζ, 1 ψ = -ζ/K²        1: ζ  → 2 ût = -il ψ, 3 ∂y ut = l² ψ
    //   2: uc → 4 uc, 5 il uc           3: vc → 6 vc
    //   4: pc → 7 pc, 8 il pc
    // (x-derivatives ik·… are formed in the row pass, where k is constant)
    const int fin = grp <= 1 ? 0 : grp - 1;
    const double2* Xf = X + (long long)fin * g.cfield + (long long)krc * g.LrP;
    double2 x[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int m = c.t + s * NT;
      const int j = compact_of(g, m);
      const double2 t = Xf[j >= 0 ? j : 0];
      x[s] = (live && j >= 0) ? t : zero2();
      if (grp <= 1) {  // ψ = -ζ invKrsq (:125-127)
        const double l = lwav(g, m);
        const double K2 = k * k + l * l;
        const double iK2 = K2 == 0.0 ? 0.0 : 1.0 / K2;
        const double2 ps = make_double2(-x[s].x * iK2, -x[s].y * iK2);
        if (grp == 1) x[s] = ps;
        else v[s] = ps;
      }
    }
    if (grp == 0) {
      double2 psi[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        psi[s] = v[s];
        v[s] = cscale(x[s], scale);
      }
      if (out <= 0) {
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(0);
      }
      if (out != 0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = cscale(psi[s], scale);
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(1);
      }
    } else if (grp == 1) {  // x = ψ
      if (out <= 0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = cmul_i(x[s], -lwav(g, c.t + s * NT) * scale);
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(2);
      }
      if (out != 0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          const double l = lwav(g, c.t + s * NT);
          v[s] = cscale(x[s], (l * l) * scale);
        }
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(3);
      }
    } else {
      const int o = grp == 2 ? 4 : (grp == 3 ? 6 : 7);
      if (out <= 0) {
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = cscale(x[s], scale);
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(o);
      }
      if (grp != 3 && out != 0) {  // ∂y uc, ∂y pc
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = cmul_i(x[s], lwav(g, c.t + s * NT) * scale);
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(o + 1);
      }
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
      const double2 qg = grp == 0 ? q1 : q2;
      qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, grp, psi[s].x, psi[s].y);
      v[s] = cscale(qg, scale);
    }
    if (out <= 0) {
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(grp);
    }
    if (out < 0 || out == 1) {
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cscale(psi[s], scale);
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(2 + grp);
    }
    if (out < 0 || out == 2) {
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cmul_i(psi[s], lwav(g, c.t + s * NT) * scale);
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(4 + grp);
    }
  }
}

// ===========================================================================
// row: one physical row y per line.  Real fields travel in pairs a + i b
// through one complex FFT of length nx (Z[k] = A[k] + i B[k] for k <= nx/2,
// Z[nx-k] = conj(A[k]) + i conj(B[k]); the DC bin keeps real parts only —
// numpy's c2r rule).
// ===========================================================================
// Row-pass addressing (k_row, k_row_c2r1).  Element s of thread t of a row
// is the x-wavenumber kk_s = t + s·NT for s < 4 and the Hermitian mirror
// N − t − s·NT for s >= 4 (inverse transforms' inputs), or k = t + s·NT
// (forward transforms' outputs).  A row's mixed-field offsets are the same
// for every field, so they are formed once per row: with one slab in closed
// form (a per-thread term plus a per-s constant, which folds into the scalar
// base of each load and store), with several slabs from the tile offsets.
// Dead inputs (kk >= kc) read column 0 of the row (in bounds) and are zeroed;
// s-slots dead on every thread of the row are skipped (uniform branch).
#if SW_TILE_I == 2 && SW_LORD_I == 0 && SW_TILE_F == 2 && SW_LORD_F == 1
#define SW_ROW_CLOSED true
#else
#define SW_ROW_CLOSED false
#endif
// LEAN: the row kernel runs at 128 VGPRs (row_fly): per-use offsets
template <int LOG2N, bool LEAN = false>
struct RowIdx {
  static constexpr int N = 1 << LOG2N, NT = N / 8;
  // 8192-point lines (128 VGPRs): only t, y are kept; the per-thread terms
  // are re-derived at each use from an opaque copy of t (SW_OPAQUE_T)
  static constexpr bool kStore = LOG2N < SW_OPAQUE_LOG2 && !LEAN;
  int oi[kStore ? 8 : 1];
  int f0s;  // kStore: forward-layout term of k = t
  int t, y;
  __device__ __forceinline__ static int kk(int t, int s) { return s < 4 ? t + s * NT : N - t - s * NT; }
  // some thread of the row holds a live inverse input s (uniform)
  __device__ __forceinline__ static bool inv_any(const Geom& g, int s) {
    return s < 4 ? s * NT < g.kc : (7 - s) * NT + 1 < g.kc;
  }
  // some thread holds a live forward output s, k = t + s NT < kc (uniform)
  __device__ __forceinline__ static bool fwd_any(const Geom& g, int s) { return s * NT < g.kc; }
  // one slab: inverse layout 8 (kk >> 1) + 4 (kk & 1) + row term (column-major
  // tiles; row-major: (kk & 1) and twice the row term), forward layout
  // 2 ny (k >> 1) + (k & 1) + row term (mtile_local, A = 2)
  __device__ __forceinline__ static int row_inv(const Geom& g, int y) {
    return (y >> 2) * (g.kcl >> 1) * 8 + (y & 3) * (g.tcm ? 1 : 2);
  }
  // (A = 2^fa columns per tile: k = t + s NT adds s NT nyl, NT a multiple of A)
  __device__ __forceinline__ static int fwd0(const Geom& g, int t, int y) {
    const int fb = 3 - g.fa;
    return (y >> fb) * 8 + ((y & ((1 << fb) - 1)) << g.fa) + (((t >> g.fa) * g.nyl) << g.fa) +
           (t & ((1 << g.fa) - 1));
  }
  __device__ __forceinline__ int oinv_calc(const Geom& g, int s) const {
    int tt = t;
    if constexpr (LOG2N >= SW_OPAQUE_LOG2 || LEAN) asm volatile("" : "+v"(tt));
    const int k = kk(tt, s);
    if (SW_ROW_CLOSED && g.nslab == 1) {
      const int r0 = row_inv(g, y);
      if (k >= g.kc) return r0;
      // mirror kk = (8 - s) NT - tt: 8 (kk >> 1) + KI (kk & 1) = 4 (8 - s) NT - 4 tt + (KI - 4) (tt & 1)
      const int KI = g.tcm ? 4 : 1;  // offset of an odd kk
      return s < 4 ? r0 + 8 * (tt >> 1) + KI * (tt & 1) + 4 * NT * s
                   : r0 - 4 * tt + (KI - 4) * (tt & 1) + 4 * NT * (8 - s);
    }
    return midx_i(g, k < g.kc ? k : 0, y);
  }
  __device__ __forceinline__ void init(const Geom& g, int t_, int y_) {
    t = t_;
    y = y_;
    if constexpr (kStore) {
#pragma unroll
      for (int s = 0; s < 8; ++s) oi[s] = oinv_calc(g, s);
      f0s = fwd0(g, t, y);
    }
  }
  __device__ __forceinline__ int oinv(const Geom& g, int s) const {
#if defined(SW_EXP_NOHBM) || defined(SW_EXP_NOLOAD)  // experiment: every load from one address (L1 hits)
    return 0;
#endif
    if constexpr (kStore) return oi[s];
    else return oinv_calc(g, s);
  }
  // forward-layout offset of output s (k = t + s NT)
  __device__ __forceinline__ int ofwd(const Geom& g, int s) const {
#if defined(SW_EXP_NOHBM) || defined(SW_EXP_NOSTORE)  // experiment: every store to two addresses
    return t & 1;
#endif
    int tt = t;
    if constexpr (LOG2N >= SW_OPAQUE_LOG2 || LEAN) asm volatile("" : "+v"(tt));
    if (SW_ROW_CLOSED && g.nslab == 1) return (kStore ? f0s : fwd0(g, tt, y)) + s * NT * g.nyl;
    return midx(g, tt + s * NT, y);
  }
};

// a + i b from the x-spectra of a row: z[kk] = a + i b for kk <= N/2,
// conj(a) + i conj(b) at the mirror (the DC bin keeps real parts only —
// numpy's c2r rule); dead kk give 0
__device__ __forceinline__ double2 pair_z(double2 aa, double2 bb, int kk, bool mirror, bool live) {
  if (kk == 0) {
    aa.y = 0.0;
    bb.y = 0.0;
  }
  if (mirror) {
    aa = cconj(aa);
    bb = cconj(bb);
  }
  return live ? make_double2(aa.x - bb.y, aa.y + bb.x) : zero2();
}

template <int LOG2N, bool LEAN = false>
__device__ __forceinline__ void load_pair(double2 (&v)[8], const RowIdx<LOG2N, LEAN>& ri, const Geom& g,
                                          const double2* __restrict__ A,
                                          const double2* __restrict__ B, bool deriv) {
  using R = RowIdx<LOG2N, LEAN>;
  double2 a[8], b[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {  // issue every load first
    a[s] = b[s] = zero2();
    if (R::inv_any(g, s)) {
      const int o = ri.oinv(g, s);
      a[s] = mix_ld_row(A + o);
      if (B) b[s] = mix_ld_row(B + o);
    }
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int kk = R::kk(ri.t, s);
    double2 aa = a[s], bb = b[s];
    if (deriv) {
      const double kw = kk * g.mk;
      aa = cmul_i(aa, kw);
      bb = cmul_i(bb, kw);
    }
    v[s] = pair_z(aa, bb, kk, s >= 4 && kk != (R::N >> 1), kk < g.kc);
  }
}

// load_pair with a per-field x-multiplier m: 0 → 1, 1 → ik, 2 → (ik)² = -k²
// (B may be null: b = 0)
template <int LOG2N, bool LEAN = false>
__device__ __forceinline__ void load_pair_m(double2 (&v)[8], const RowIdx<LOG2N, LEAN>& ri, const Geom& g,
                                            const double2* __restrict__ A, int ma,
                                            const double2* __restrict__ B, int mb) {
  using R = RowIdx<LOG2N, LEAN>;
  double2 a[8], b[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    a[s] = b[s] = zero2();
    if (R::inv_any(g, s)) {
      const int o = ri.oinv(g, s);
      a[s] = mix_ld_row(A + o);
      if (B) b[s] = mix_ld_row(B + o);
    }
  }
  auto mul = [](double2 x, int mm, double kw) {
    return mm == 0 ? x : (mm == 1 ? cmul_i(x, kw) : cscale(x, -(kw * kw)));
  };
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int kk = R::kk(ri.t, s);
    const double kw = kk * g.mk;
    v[s] = pair_z(mul(a[s], ma, kw), mul(b[s], mb, kw), kk, s >= 4 && kk != (R::N >> 1), kk < g.kc);
  }
}

// RSW second inverse pair: a = Ĥ, b = ζ̂ = ik V̂ - Uy (x-spectral, per element)
template <int LOG2N, bool LEAN = false>
__device__ __forceinline__ void load_eta_zeta(double2 (&v)[8], const RowIdx<LOG2N, LEAN>& ri, const Geom& g,
                                              const double2* __restrict__ H,
                                              const double2* __restrict__ V,
                                              const double2* __restrict__ Uy) {
  using R = RowIdx<LOG2N, LEAN>;
  double2 h[8], vv[8], uy[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    h[s] = vv[s] = uy[s] = zero2();
    if (R::inv_any(g, s)) {
      const int o = ri.oinv(g, s);
      h[s] = mix_ld_row(H + o);
      vv[s] = mix_ld_row(V + o);
      uy[s] = mix_ld_row(Uy + o);
    }
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int kk = R::kk(ri.t, s);
    v[s] = pair_z(h[s], csub(cmul_i(vv[s], kk * g.mk), uy[s]), kk, s >= 4 && kk != (R::N >> 1), kk < g.kc);
  }
}

// RSW inverse pairs u + i v and η + i ζ from one read of U, V, H, Uy
template <int LOG2N, bool LEAN = false>
__device__ __forceinline__ void load_uv_eta_zeta(double2 (&w)[2][8], const RowIdx<LOG2N, LEAN>& ri, const Geom& g,
                                                 const double2* __restrict__ U, const double2* __restrict__ V,
                                                 const double2* __restrict__ H, const double2* __restrict__ Uy) {
  using R = RowIdx<LOG2N, LEAN>;
  double2 u[8], vv[8], h[8], uy[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    u[s] = vv[s] = h[s] = uy[s] = zero2();
    if (R::inv_any(g, s)) {
      const int o = ri.oinv(g, s);
      u[s] = mix_ld_row(U + o);
      vv[s] = mix_ld_row(V + o);
      h[s] = mix_ld_row(H + o);
      uy[s] = mix_ld_row(Uy + o);
    }
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int kk = R::kk(ri.t, s);
    const bool mir = s >= 4 && kk != (R::N >> 1), live = kk < g.kc;
    w[0][s] = pair_z(u[s], vv[s], kk, mir, live);
    w[1][s] = pair_z(h[s], csub(cmul_i(vv[s], kk * g.mk), uy[s]), kk, mir, live);
  }
}

// After a forward FFT of z = a + i b (Z[t + s*NT] in v), hand Â[k], B̂[k] for
// k = t + s NT < kc to emit(k, s, Â, B̂).  Needs Z[nx-k] from a mirror
// thread: one LDS round trip.
// PRUNE: slots 3 and 4 are never read as a mirror (sw_fft.hpp prune_slot):
// not written
template <int LOG2N, bool LEAN = false, bool PRUNE = false, typename Emit>
__device__ __forceinline__ void split_pair(const double2 (&v)[8], int t, const Geom& g,
                                           double2* line, Emit emit) {
  if constexpr (LOG2N >= SW_OPAQUE_LOG2 || LEAN) asm volatile("" : "+v"(t));
  constexpr int N = 1 << LOG2N, NT = N / 8;
  lds_barrier();  // previous LDS readers are done
#pragma unroll
  for (int s = 0; s < 8; ++s)
    if (!(PRUNE && prune_slot(s))) line[LP<LOG2N>(t + s * NT)] = v[s];
  lds_barrier();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = t + s * NT;
    if (RowIdx<LOG2N>::fwd_any(g, s) && k < g.kc) {
      const double2 zk = v[s];
      const double2 zn = line[LP<LOG2N>((N - k) & (N - 1))];
      // A = (zk + conj zn) / 2,  B = (zk - conj zn) / (2i)
      emit(k, s, make_double2(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y)),
           make_double2(0.5 * (zk.y + zn.y), -0.5 * (zk.x - zn.x)));
    }
  }
}

// split_pair for C transforms at once (C line buffers `stride` apart, one
// barrier pair): emit(c, k, s, Â, B̂).
template <int LOG2N, int C, bool PRUNE = false, typename Emit>
__device__ __forceinline__ void split_pairs(const double2 (&v)[C][8], int t, const Geom& g,
                                            double2* line, int stride, Emit emit) {
  SW_OPAQUE_T(t);
  constexpr int N = 1 << LOG2N, NT = N / 8;
  lds_barrier();
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (!(PRUNE && prune_slot(s))) line[c * stride + LP<LOG2N>(t + s * NT)] = v[c][s];
  lds_barrier();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = t + s * NT;
    if (RowIdx<LOG2N>::fwd_any(g, s) && k < g.kc) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const double2 zk = v[c][s];
        const double2 zn = line[c * stride + LP<LOG2N>((N - k) & (N - 1))];
        emit(c, k, s, make_double2(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y)),
             make_double2(0.5 * (zk.y + zn.y), -0.5 * (zk.x - zn.x)));
      }
    }
  }
}

template <int LOG2N, bool LEAN = false, bool PRUNE = false>
__device__ __forceinline__ void store_pair(const double2 (&v)[8], const RowIdx<LOG2N, LEAN>& ri, const Geom& g,
                                           double2* line, double2* __restrict__ A,
                                           double2* __restrict__ B) {
  split_pair<LOG2N, LEAN, PRUNE>(v, ri.t, g, line, [&](int, int s, double2 a, double2 b) {
    const int o = ri.ofwd(g, s);
    A[o] = a;
    B[o] = b;
  });
}

// LDS line buffers per row of k_row: RSW transforms pairs of lines together
// where two buffers per row fit the 160 KB of LDS (nx <= 4096)
// Threads per block of the row pass.  Measured (tools/ab/sweep_sizes.sh): the
// RSW row (two line buffers) runs best with up to 256 threads per block
// (1024²: 29 vs 36 µs at 128), every other kernel with one line per block
// down to 64 threads (512² TY / MultiLayerQG steps +11-14 %, 1024² RSW
// col_step 31 -> 28 µs) — more, smaller blocks spread a small grid over the
// 256 CUs.
// On lines of at most 512 points (the drivers' 512² grids) the RSW row takes
// one line per 64-thread block like the other kernels (SW_RSW_ROW_TGT_SHORT;
// round 6, tools/ab/r6_rowtgt.sh: RSWDriver 512² IFMAB3 31669-32020 →
// 32333-32573 steps/s at 64 against 256 threads, 128 between; bitwise equal)
#ifndef SW_RSW_ROW_TGT_SHORT
#define SW_RSW_ROW_TGT_SHORT 64
#endif
template <int MODEL, int LOG2N>
__host__ __device__ constexpr int row_tgt() {
  return MODEL == MODEL_RSW ? (LOG2N <= 9 ? SW_RSW_ROW_TGT_SHORT : 256) : SW_BLK_THREADS;
}
template <int MODEL, int LOG2N>
using BlkRow = Blk<LOG2N, row_tgt<MODEL, LOG2N>()>;

// the 2LQG / MultiLayerQG row on the decimated lines with two line buffers,
// as the RSW row (round 6, SW_QG_ROW_PAIR): q and ψx inverse-transformed as
// a pipelined pair, ψy alone, the two products' forward transforms as a
// pipelined pair — two blocks per CU, twiddles held, instead of one buffer,
// four blocks and per-stage twiddle reads.  Measured (tools/ab/r6_qgpair.sh):
// 2048 row 69.9-70.5 -> 73.3-75.1 µs, config 3 -2 %: off (parity green; not
// bitwise the default at 2048, whose twiddle powers are formed as a chain)
#ifndef SW_QG_ROW_PAIR
#define SW_QG_ROW_PAIR 0
#endif
template <int LOG2N>
__host__ __device__ constexpr bool qg_row_pair() {
  return SW_QG_ROW_PAIR && LOG2N >= 10 && LOG2N <= 12;  // (the decimated lines: roww)
}
template <int MODEL, int LOG2N>
__host__ __device__ constexpr int row_lds_lines() {
#ifdef SW_ROW_CB1  // sweep knob: one line buffer per row
  return 1;
#else
  if (MODEL == MODEL_QG2 && qg_row_pair<LOG2N>()) return 2;
  return (MODEL == MODEL_RSW && 2 * BlkRow<MODEL, LOG2N>::NB * FftPlan<LOG2N>::LDS * 16 <= 160 * 1024) ? 2 : 1;
#endif
}
// C = 2: both transforms per barrier; C = 1: one after the other
template <int LOG2N, int DIR, int C>
__device__ __forceinline__ void fft_pair(double2 (&w)[2][8], int t, const Twiddles<LOG2N>& tws,
                                         double2* line, int stride) {
  if constexpr (C == 2) {
    fft_lines<LOG2N, DIR, 2>(w, t, tws, line, stride);
  } else {
    fft_line<LOG2N, DIR>(w[0], t, tws, line);
    fft_line<LOG2N, DIR>(w[1], t, tws, line);
  }
}

// After split_pair (LDS still holds Z): the aliased x-spectra kc <= k <= nx/2
// of the pair, A[k] and B[k], into (k - kc, stored row y) of the Ma fields A
// and B (aliased-state tracking, sw_config.aliased_state; ma_off)
template <int LOG2N, int NFA, bool NIK_A = false>
__device__ __forceinline__ void store_alias_pair(const double2 (&v)[8], int t, const Geom& g, const double2* line,
                                                 double2* __restrict__ A, double2* __restrict__ B, int y) {
  constexpr int N = 1 << LOG2N, NT = N / 8;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = t + s * NT;
    if (k >= g.kc && k <= N / 2) {
      const double2 zk = v[s];
      const double2 zn = line[LP<LOG2N>((N - k) & (N - 1))];
      const long long o = ma_off(g, NFA, k - g.kc, y);
      const double2 a = make_double2(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
      A[o] = NIK_A ? cmul_i(a, -(k * g.mk)) : a;  // as the live outputs: Q = -ik (uη)^ (RSW)
      B[o] = make_double2(0.5 * (zk.y + zn.y), -0.5 * (zk.x - zn.x));
    }
  }
}

// store_alias_pair with the outputs formed by the caller: emit(o, k, Â, B̂)
// for the aliased kc <= k <= nx/2 of the pair in LDS, o = the offset of
// (k - kc, y) in one Ma field (Thomas–Yamada's seven outputs)
template <int LOG2N, int NFA, typename Emit>
__device__ __forceinline__ void store_alias_with(const double2 (&v)[8], int t, const Geom& g, const double2* line,
                                                 int y, Emit emit) {
  constexpr int N = 1 << LOG2N, NT = N / 8;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = t + s * NT;
    if (k >= g.kc && k <= N / 2) {
      const double2 zk = v[s];
      const double2 zn = line[LP<LOG2N>((N - k) & (N - 1))];
      emit(ma_off(g, NFA, k - g.kc, y), k, make_double2(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y)),
           make_double2(0.5 * (zk.y + zn.y), -0.5 * (zk.x - zn.x)));
    }
  }
}

// The 2LQG row from 2048-point lines (SW_QG_ROW_FLY_MIN): stage twiddles read
// per stage and the thread index opaque per transform (Twiddles<…, FLY>), 116
// VGPRs, 4 waves per SIMD — 2048²: 85 -> 76 µs, config 3 +2-3 %
// (tools/ab/ab_lean11.sh); the same measures slow the RSW kernels there (row
// 77 -> 82, col_step 85 -> 92 µs), which keep theirs.
#ifndef SW_QG_ROW_FLY_MIN
#define SW_QG_ROW_FLY_MIN 11
#endif
// Row transforms of 1024-4096 points (the full-length RSW/2LQG rows; the
// half-length rows' M = nx/2 lines with SW_ROWH_W) run decimated across the
// line's W waves (sw_fft.hpp fftw_*: one workgroup exchange per transform
// instead of three; SW_ROW4W=0: the Stockham fft_lines).  Returns W, or 0.
#ifndef SW_ROW4W
#define SW_ROW4W 1
#endif
template <int LOG2N>
__host__ __device__ constexpr int roww() {
  return (SW_ROW4W && LOG2N >= 10 && LOG2N <= 12) ? (1 << (LOG2N - 9)) : 0;
}
// the half-length rows' M-point lines: the RSW row (k_row_rsw_h, 2 waves
// per SIMD) at 4096² (M = 2048, W = 4: row 401-407 -> 398 µs, config 4 one
// GPU 1274 -> 1286 steps/s); the 2LQG row (k_row_qg_h, 128 VGPRs) spilled
// with them (4096²: row 426 -> 525 µs; 8192², W = 8: 1823 -> 3150 µs, 54
// spills: the hoisted twiddle powers, round 4: 8) and keeps Stockham, as does
// the RSW row at 8192² (unmeasured).
// SW_ROWH_W=1: every half row.
#ifndef SW_ROWH_W
#define SW_ROWH_W 0
#endif
// the rows' pair splits folded into the decimated forward transforms
// (sw_fft.hpp fftw_dit_split): bitwise-tested (GPU parity at 2048) but
// measured slower — RSW row 73.7 -> 74.7, 2LQG row 74.3 -> 76.7 µs (the
// radix-W combination done twice costs more VALU than the second exchange)
#ifndef SW_SPLIT_FOLD
#define SW_SPLIT_FOLD 0
#endif
// the RSW row (two blocks per CU, set by its LDS) keeping the wave-local
// stage twiddle powers for all its transforms (fft_lines SHARE: 218 VGPRs,
// 3 % fewer fp64 instructions): measured neutral (71.4-73.3 vs 71.0-71.5
// µs), off
#ifndef SW_ROW_TW_SHARE
#define SW_ROW_TW_SHARE 0
#endif
// the 2LQG half row on the decimated transforms from 2^(SW_ROWH_W_QG_MIN + 1)
// -point rows: at 8192 the radix-8 decimation (W = 8) fits 128 VGPRs (8
// spilled) once its twiddle powers are formed per call (sw_fft.hpp
// tw_powers), but measured neutral (row 1601-1603 against 1601-1606 µs,
// tools/ab/r4_batch14.sh): the Stockham form stays (13: off)
#ifndef SW_ROWH_W_QG_MIN
#define SW_ROWH_W_QG_MIN 13
#endif
template <int LM, bool RSW = false>
__host__ __device__ constexpr int roww_h() {
  return (SW_ROWH_W || (RSW && LM == 11) || (!RSW && LM >= SW_ROWH_W_QG_MIN)) ? roww<LM>() : 0;
}
template <int MODEL, int LOG2N>
__host__ __device__ constexpr bool row_fly() {
  return LOG2N >= SW_TWFLY_LOG2 || (MODEL == MODEL_QG2 && LOG2N >= SW_QG_ROW_FLY_MIN && !qg_row_pair<LOG2N>());
}
// PRUNE: a live band kc <= 3N/8 (row_prunable): the decimated transforms
// skip the zero inputs and unused outputs of slots 3 and 4 (sw_fft.hpp)
// SPLIT: more blocks per row on short rows (Geom::rsplit), each running a
// subset of the row's transforms on the same pairs (bitwise the same
// outputs): 2LQG / MultiLayerQG grid (rows, 2), block y = 0 forms ψx q, 1
// forms ψy q, each with its own q transform (three transforms per block
// instead of five); Thomas–Yamada grid (rows, 4), the parts of its branch;
// RSW (two line buffers, undecimated lines) grid (rows, 2), the two forward
// lines apart
// KC > 0: the live band kc known at compile time (the 2/3 rule's N/3; a local
// copy of the geometry with that kc, so every inlined helper's slot and lane
// tests against it fold where they can — as the half rows' live_kc)
template <int MODEL, int LOG2N, bool ALIAS = false, bool PRUNE = false, bool SPLIT = false, int KC = 0>
static __global__ void __launch_bounds__((BlkRow<MODEL, LOG2N>::THREADS),
                                         (BlkRow<MODEL, LOG2N>::THREADS >= 1024 ? 4
                                          : (MODEL == MODEL_QG2 ? (row_fly<MODEL, LOG2N>() ? 4 : SW_MINW_ROW_QG)
                                                                : SW_MINW_ROW)))
    k_row(Geom g_in, Phys p, const double2* __restrict__ Mi, double2* __restrict__ Mo,
          const double2* __restrict__ tw, int yoff, double2* __restrict__ Ma) {
  Geom g = g_in;
  // (KC is launched only on one slab: the closed-form tile offsets, no slab
  // division — tools/ab/r6_slab1.sh: RSW 2048 row 65.7-66.7 → 64.0-65.2 µs,
  // the drivers' 512² rows +1.3..+2.5 %)
  if constexpr (KC > 0) {
    g.kc = KC;
    g.nslab = 1;
  }
  using Bk = BlkRow<MODEL, LOG2N>;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  // local rows [yoff, yoff + NB gridDim.x): all of them, or one chunk of a
  // row-chunked launch (the pipelined slab exchange)
  const int y = yoff + ((Bk::NB == 1) ? col_of_block(blockIdx.x, gridDim.x)
                                      : row0_of_block<Bk::NB>(blockIdx.x, gridDim.x) + c.ln);
  constexpr int CB = row_lds_lines<MODEL, LOG2N>();
  double2* line = smem + c.ln * CB * FftPlan<LOG2N>::LDS;
  RowIdx<LOG2N, row_fly<MODEL, LOG2N>()> ri;
  ri.init(g, c.t, y);
  Twiddles<LOG2N, row_fly<MODEL, LOG2N>()> tws;
  tws.load(c.t, tw);
  const long long MF = g.mfield;
  double2 v[8];

  if constexpr (MODEL == MODEL_RSW) {
    // rsw/RotatingShallowWater.jl:140-230 in vorticity form:
    //   u ux + v uy = ∂x K - ζ v,  u vx + v vy = ∂y K + ζ u,
    //   K = (u² + v²)/2, ζ = vx - uy.
    // Both sides agree exactly on the live (2/3-rule) modes, where every
    // product's aliases vanish.  Outputs (x-spectral, k < kc):
    //   0 P = -ik K̂ + (ζv)^   -> N_u = F_y(P)
    //   1 K̂, 2 (ζu)^          -> N_v = -il F_y(K̂) - F_y((ζu)^)
    //   3 Q = -ik (uη)^, 4 (vη)^ -> N_η = F_y(Q) - il F_y((vη)^)
    const double2 *U = Mi, *V = Mi + MF, *H = Mi + 2 * MF, *Uy = Mi + 3 * MF;
    constexpr int LS = FftPlan<LOG2N>::LDS;  // two line buffers per row
    double2 w[2][8];
    // the decimated transforms (roww): physical x in the DIF's order
    constexpr int W = CB == 2 ? roww<LOG2N>() : 0;
    Twiddles<9> tq;
    double2 wt = zero2();
    if constexpr (W > 0) {
      tq.load(c.t & 63, tw, LOG2N - 9);
      wt = tw[c.t];
    }
    // u + i v and η + i ζ, transformed together (fft_lines leaves z[x = t + s*NT])
    if constexpr (SPLIT && CB == 2 && W == 0) {
      // short rows in two blocks (Geom::rsplit): both inverse pairs, then
      // block y = 0 the ζu + i ζv line and K (outputs 0-2), y = 1 the
      // uη + i vη line (outputs 3-4)
      load_pair<LOG2N>(w[0], ri, g, U, V, false);
      load_eta_zeta<LOG2N>(w[1], ri, g, H, V, Uy);
      fft_pair<LOG2N, +1, CB>(w, c.t, tws, line, LS);
      const int part = blockIdx.y;
      double kk[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const double u = w[0][s].x, vv = w[0][s].y, eta = w[1][s].x, zeta = w[1][s].y;
        kk[s] = 0.5 * (u * u + vv * vv);
        w[0][s] = make_double2(zeta * u, zeta * vv);  // ζu + i ζv
        w[1][s] = make_double2(u * eta, vv * eta);    // uη + i vη
      }
      if (part == 1) {
        fft_line<LOG2N, -1>(w[1], c.t, tws, line);
        split_pairs<LOG2N, 1>(reinterpret_cast<const double2(&)[1][8]>(w[1]), c.t, g, line, LS,
                              [&](int, int k, int s, double2 a, double2 b) {
                                const int o = ri.ofwd(g, s);
                                Mo[3 * MF + o] = cmul_i(a, -(k * g.mk));
                                Mo[4 * MF + o] = b;
                              });
        return;
      }
      fft_line<LOG2N, -1>(w[0], c.t, tws, line);
      double2 zv[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) zv[s] = zero2();
      split_pairs<LOG2N, 1>(reinterpret_cast<const double2(&)[1][8]>(w[0]), c.t, g, line, LS,
                            [&](int, int, int s, double2 a, double2 b) {
                              Mo[2 * MF + ri.ofwd(g, s)] = a;
                              zv[s] = b;
                            });
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = make_double2(kk[s], 0.0);
      lds_barrier();  // split_pairs' mirror reads are done
      fft_line<LOG2N, -1>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int k = c.t + s * Bk::NT;
        if (RowIdx<LOG2N>::fwd_any(g, s) && k < g.kc) {
          const int o = ri.ofwd(g, s);
          Mo[o] = cadd(cmul_i(v[s], -(k * g.mk)), zv[s]);
          Mo[MF + o] = v[s];
        }
      }
      return;
    }
    if constexpr (W > 0) {
      load_uv_eta_zeta<LOG2N>(w, ri, g, U, V, H, Uy);  // V read once (row 74.9 -> 73.5 µs)
      fftw_dif<W, +1, 2, false, false, SW_ROW_TW_SHARE, PRUNE>(w, c.t, wt, tq, line, LS);
    } else if constexpr (CB == 2) {
      load_pair<LOG2N>(w[0], ri, g, U, V, false);
      load_eta_zeta<LOG2N>(w[1], ri, g, H, V, Uy);
      fft_pair<LOG2N, +1, CB>(w, c.t, tws, line, LS);
    } else {
      // nx = 8192 (128 VGPRs per thread): one pair at a time, the second
      // pair's loads issued after the first transform; η + iζ (three loads)
      // first, while nothing else is live
      load_eta_zeta<LOG2N>(w[1], ri, g, H, V, Uy);
      fft_line<LOG2N, +1>(w[1], c.t, tws, line);
      load_pair<LOG2N>(w[0], ri, g, U, V, false);
      fft_line<LOG2N, +1>(w[0], c.t, tws, line);
    }
    // The forward pairs hold lines of one magnitude class: a pair's split
    // leaves each half an absolute error ~ eps × the pair's norm, and ζu
    // (~ k u² at wavenumber k) beside uη, K beside ζv put the larger line's
    // roundoff into the smaller.  ζu + i ζv and uη + i vη pair; K, the real
    // line, goes alone last, and P = -ik K̂ + (ζv)^ takes (ζv)^ from the
    // registers (white-noise state, tests/test_gpu_invariants.py: the
    // ⟨u, N_u⟩, ⟨v, N_v⟩ budgets 9e-18 -> 4e-19).  The inverse pair η + iζ
    // keeps that roundoff in η (its budget ~1e-13 there, 1e-19 on the oracle).
    double kk[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double u = w[0][s].x, vv = w[0][s].y, eta = w[1][s].x, zeta = w[1][s].y;
      kk[s] = 0.5 * (u * u + vv * vv);
      w[0][s] = make_double2(zeta * u, zeta * vv);  // ζu + i ζv
      w[1][s] = make_double2(u * eta, vv * eta);    // uη + i vη
    }
    if constexpr (W > 0) fftw_dit<W, -1, 2, false, false, SW_ROW_TW_SHARE, PRUNE>(w, c.t, wt, tq, line, LS);
    else fft_pair<LOG2N, -1, CB>(w, c.t, tws, line, LS);
    double2 zv[8];  // (ζv)^ of the live slots
#pragma unroll
    for (int s = 0; s < 8; ++s) zv[s] = zero2();
    auto emit = [&](int cc, int k, int s, double2 a, double2 b) {
      const int o = ri.ofwd(g, s);
      if (cc == 0) {
        Mo[2 * MF + o] = a;
        zv[s] = b;
      } else {
        Mo[3 * MF + o] = cmul_i(a, -(k * g.mk));
        Mo[4 * MF + o] = b;
      }
    };
    if constexpr (CB == 2) {
      split_pairs<LOG2N, 2, PRUNE && (W > 0)>(w, c.t, g, line, LS, emit);
    } else {
      split_pairs<LOG2N, 1>(reinterpret_cast<const double2(&)[1][8]>(w[0]), c.t, g, line, LS, emit);
      split_pairs<LOG2N, 1>(reinterpret_cast<const double2(&)[1][8]>(w[1]), c.t, g, line, LS,
                            [&](int, int k, int s, double2 a, double2 b) { emit(1, k, s, a, b); });
    }
    // K (real input: the transform is the spectrum itself)
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = make_double2(kk[s], 0.0);
    lds_barrier();  // split_pairs' mirror reads are done
    if constexpr (W > 0)
      fftw_dit<W, -1, 1, false, false, SW_ROW_TW_SHARE, PRUNE>(reinterpret_cast<double2(&)[1][8]>(v), c.t, wt, tq,
                                                                line, LS);
    else fft_line<LOG2N, -1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = c.t + s * Bk::NT;
      if (RowIdx<LOG2N>::fwd_any(g, s) && k < g.kc) {
        const int o = ri.ofwd(g, s);
        Mo[o] = cadd(cmul_i(v[s], -(k * g.mk)), zv[s]);
        Mo[MF + o] = v[s];
      }
    }
  } else if constexpr (MODEL == MODEL_RSWA) {
    // rsw/RotatingShallowWater.jl:140-230 as written (advective form, the
    // reference's products on every mode; aliased_fraction = 0):
    //   N_u = -(u ux)^ - (v uy)^,  N_v = -(v vy)^ - (u vx)^,  N_η = -ik (uη)^ - il (vη)^
    // Inputs (k_col_inv): 0 U, 1 V, 2 H, 3 Uy, 4 Vy.  Outputs (x-spectral):
    //   0 (u ux + v uy)^, 1 (u vx + v vy)^ -> N_u, N_v = -F_y(…)
    //   2 Q = -ik (uη)^, 3 (vη)^          -> N_η = F_y(Q) - il F_y((vη)^)
    const double2 *U = Mi, *V = Mi + MF, *H = Mi + 2 * MF, *Uy = Mi + 3 * MF, *Vy = Mi + 4 * MF;
    double2 uv[8], pr[8];
    load_pair<LOG2N>(uv, ri, g, U, V, false);  // u + i v
    fft_line<LOG2N, +1>(uv, c.t, tws, line);
    load_pair<LOG2N>(v, ri, g, U, V, true);  // ux + i vx
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) pr[s] = make_double2(uv[s].x * v[s].x, uv[s].x * v[s].y);
    load_pair<LOG2N>(v, ri, g, Uy, Vy, false);  // uy + i vy
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) pr[s] = make_double2(pr[s].x + uv[s].y * v[s].x, pr[s].y + uv[s].y * v[s].y);
    fft_line<LOG2N, -1>(pr, c.t, tws, line);
    store_pair<LOG2N>(pr, ri, g, line, Mo, Mo + MF);
    const long long MA = ma_field(g);  // aliased columns × rows per field
    if constexpr (ALIAS) store_alias_pair<LOG2N, ma_nfa(MODEL)>(pr, c.t, g, line, Ma, Ma + MA, y + g.y0);
    load_pair<LOG2N>(v, ri, g, H, nullptr, false);  // η
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = make_double2(uv[s].x * v[s].x, uv[s].y * v[s].x);  // uη + i vη
    fft_line<LOG2N, -1>(v, c.t, tws, line);
    split_pair<LOG2N>(v, c.t, g, line, [&](int k, int s, double2 a, double2 b) {
      const int o = ri.ofwd(g, s);
      Mo[2 * MF + o] = cmul_i(a, -(k * g.mk));
      Mo[3 * MF + o] = b;
    });
    if constexpr (ALIAS) store_alias_pair<LOG2N, ma_nfa(MODEL), true>(v, c.t, g, line, Ma + 2 * MA, Ma + 3 * MA, y + g.y0);
  } else if constexpr (MODEL == MODEL_TY) {
    // thomasyamada/ThomasYamada.jl:129-262.  Inputs (k_col_inv): 0 ζ, 1 ψ,
    // 2 ût, 3 ∂y ut, 4 uc, 5 ∂y uc, 6 vc, 7 pc, 8 ∂y pc.  Physical fields in
    // pairs through complex x-FFTs, products formed as soon as their factors
    // exist, forward pairs split and combined on the x-spectral side:
    //   p1 = vt ζ, p2 = ut ζ, p3 = uc vc, p4 = uc² - vc², p6 = ut uc,
    //   p7 = vt vc, p8 = vt ∂y uc + vc ∂y ut, p9 = ut ∂x vc + uc ∂x vt,
    //   p10 = ut ∂x pc + vt ∂y pc
    // Outputs (×(-Ro); k_col_fwd applies the y-multiplier in brackets):
    //   0 ik p̂2 - k² p̂3 [1]   1 i p̂1 + k p̂4 [l]   2 p̂3 [l²]   → N_ζ
    //   3 ik p̂6 + p̂8 [1]                                      → N_uc
    //   4 p̂7 [il]   5 p̂9 [1]                                   → N_vc
    //   6 p̂10 [1]                                              → N_pc
    const double2* F[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) F[i] = Mi + i * MF;
    const double nRo = -p.Ro;
    // SPLIT: grid (rows, 4), block y = part: 0 outputs 0-2 (transforms I1-I3),
    // 1 output 3 (I1-I4), 2 outputs 4-5 (I1-I5), 3 output 6 (I1, I2, I5, I6);
    // each part runs the same transforms of the same pairs as the whole row
    const int part = SPLIT ? (int)blockIdx.y : -1;
    auto want = [&](int q) { return part < 0 || part == q; };
    double zt[8], ut[8], vt[8], uc[8], vc[8], p6[8], p7[8], p8[8], p9[8], p10[8];
    if constexpr (SPLIT) {  // (a part skipping a transform leaves its products unused; defined anyway)
#pragma unroll
      for (int s = 0; s < 8; ++s) vc[s] = p7[s] = p8[s] = p9[s] = 0.0;
    }
    // I1: ζ + i ut, I2: vt + i uc
    load_pair_m<LOG2N>(v, ri, g, F[0], 0, F[2], 0);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      zt[s] = v[s].x;
      ut[s] = v[s].y;
    }
    load_pair_m<LOG2N>(v, ri, g, F[1], 1, F[4], 0);
    fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      vt[s] = v[s].x;
      uc[s] = v[s].y;
      p6[s] = ut[s] * uc[s];
    }
    // aliased-state tracking: the x-spectra kc <= k <= nx/2 of every output
    // into Ma (ma_off: field, k - kc, stored row; k_col_fwd_alias), as the live ones
    const long long MA = ma_field(g);
    const int yg = y + g.y0;
    if (part != 3) {
      // I3: vc + i ∂y uc
      load_pair_m<LOG2N>(v, ri, g, F[6], 0, F[5], 0);
      fft_line<LOG2N, +1>(v, c.t, tws, line);
      double2 w[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        vc[s] = v[s].x;
        p7[s] = vt[s] * vc[s];
        p8[s] = vt[s] * v[s].y;
        w[s] = make_double2(ut[s] * zt[s], uc[s] * vc[s]);          // p2 + i p3
        v[s] = make_double2(vt[s] * zt[s], uc[s] * uc[s] - vc[s] * vc[s]);  // p1 + i p4
      }
      if (want(0)) {
        fft_line<LOG2N, -1>(w, c.t, tws, line);
        split_pair<LOG2N>(w, c.t, g, line, [&](int k, int s, double2 a, double2 b) {
          const double kw = k * g.mk;
          const int o = ri.ofwd(g, s);
          Mo[o] = cscale(csub(cmul_i(a, kw), cscale(b, kw * kw)), nRo);
          Mo[2 * MF + o] = cscale(b, nRo);
        });
        if constexpr (ALIAS)
          store_alias_with<LOG2N, ma_nfa(MODEL)>(w, c.t, g, line, yg, [&](long long o, int k, double2 a, double2 b) {
            const double kw = k * g.mk;
            Ma[o] = cscale(csub(cmul_i(a, kw), cscale(b, kw * kw)), nRo);
            Ma[2 * MA + o] = cscale(b, nRo);
          });
        fft_line<LOG2N, -1>(v, c.t, tws, line);
        split_pair<LOG2N>(v, c.t, g, line, [&](int k, int s, double2 a, double2 b) {
          const double kw = k * g.mk;
          Mo[MF + ri.ofwd(g, s)] = cscale(cadd(cmul_i(a, 1.0), cscale(b, kw)), nRo);
        });
        if constexpr (ALIAS)
          store_alias_with<LOG2N, ma_nfa(MODEL)>(v, c.t, g, line, yg, [&](long long o, int k, double2 a, double2 b) {
            Ma[MA + o] = cscale(cadd(cmul_i(a, 1.0), cscale(b, k * g.mk)), nRo);
          });
      }
    }
    if (part < 0 || part == 1 || part == 2) {
      // I4: ∂y ut + i ∂x vc
      load_pair_m<LOG2N>(v, ri, g, F[3], 0, F[6], 1);
      fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        p8[s] = p8[s] + vc[s] * v[s].x;
        p9[s] = ut[s] * v[s].y;
        v[s] = make_double2(p6[s], p8[s]);
      }
      if (want(1)) {
        fft_line<LOG2N, -1>(v, c.t, tws, line);
        split_pair<LOG2N>(v, c.t, g, line, [&](int k, int s, double2 a, double2 b) {
          Mo[3 * MF + ri.ofwd(g, s)] = cscale(cadd(cmul_i(a, k * g.mk), b), nRo);
        });
        if constexpr (ALIAS)
          store_alias_with<LOG2N, ma_nfa(MODEL)>(v, c.t, g, line, yg, [&](long long o, int k, double2 a, double2 b) {
            Ma[3 * MA + o] = cscale(cadd(cmul_i(a, k * g.mk), b), nRo);
          });
      }
    }
    if (part < 0 || part == 2 || part == 3) {
      // I5: ∂x vt + i ∂x pc
      load_pair_m<LOG2N>(v, ri, g, F[1], 2, F[7], 1);
      fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        p9[s] = p9[s] + uc[s] * v[s].x;
        p10[s] = ut[s] * v[s].y;
        v[s] = make_double2(p7[s], p9[s]);
      }
      if (want(2)) {
        fft_line<LOG2N, -1>(v, c.t, tws, line);
        split_pair<LOG2N>(v, c.t, g, line, [&](int k, int s, double2 a, double2 b) {
          const int o = ri.ofwd(g, s);
          Mo[4 * MF + o] = cscale(a, nRo);
          Mo[5 * MF + o] = cscale(b, nRo);
        });
        if constexpr (ALIAS)
          store_alias_with<LOG2N, ma_nfa(MODEL)>(v, c.t, g, line, yg, [&](long long o, int, double2 a, double2 b) {
            Ma[4 * MA + o] = cscale(a, nRo);
            Ma[5 * MA + o] = cscale(b, nRo);
          });
      }
    }
    if (want(3)) {
      // I6: ∂y pc
      load_pair_m<LOG2N>(v, ri, g, F[8], 0, nullptr, 0);
      fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = make_double2(p10[s] + vt[s] * v[s].x, 0.0);
      fft_line<LOG2N, -1>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int k = c.t + s * Bk::NT;
        if (RowIdx<LOG2N>::fwd_any(g, s) && k < g.kc) Mo[6 * MF + ri.ofwd(g, s)] = cscale(v[s], nRo);
        if constexpr (ALIAS)  // (a real line: its transform is the spectrum itself)
          if (k >= g.kc && k <= Bk::NT * 4) Ma[6 * MA + ma_off(g, ma_nfa(MODEL), k - g.kc, yg)] = cscale(v[s], nRo);
      }
    }
  } else {
    const double2 *Q1 = Mi, *Q2 = Mi + MF, *P1 = Mi + 2 * MF, *P2 = Mi + 3 * MF,
                  *Py1 = Mi + 4 * MF, *Py2 = Mi + 5 * MF;
    // the decimated transforms (roww): physical x in the DIF's order
    constexpr int W = roww<LOG2N>();
    // the lean row (row_fly) reads the wave-local stage twiddles per stage
    // and W_N^t at each transform: held in registers they spill (8-33 VGPRs
    // at 128); a 64-entry LDS table of the stage twiddles spilled 26 and read
    // 88-91 against 74.5-75 µs (round 3, interleaved A/B)
    constexpr bool FL = row_fly<MODEL, LOG2N>();
    Twiddles<9, FL> tq;
    double2 wt = zero2();
    if constexpr (W > 0) {
      tq.load(c.t & 63, tw, LOG2N - 9);
      if constexpr (!FL) wt = tw[c.t];
    }
    auto wnt = [&]() { return FL ? tw[c.t] : wt; };
    using V1 = double2(&)[1][8];
    constexpr bool PR = PRUNE && W > 0 && !ALIAS;  // (ALIAS reads the slots kc <= k <= N/2)
    auto inv = [&](double2(&x)[8]) {
      if constexpr (W > 0) fftw_dif<W, +1, 1, true, FL, false, PR>(reinterpret_cast<V1>(x), c.t, wnt(), tq, line, 0);
      else fft_line<LOG2N, +1>(x, c.t, tws, line);
    };
    auto fwd = [&](double2(&x)[8]) {
      if constexpr (W > 0) fftw_dit<W, -1, 1, FL, false, false, PR>(reinterpret_cast<V1>(x), c.t, wnt(), tq, line, 0);
      else fft_line<LOG2N, -1>(x, c.t, tws, line);
    };
    if constexpr (W > 0 && row_lds_lines<MODEL, LOG2N>() == 2 && !ALIAS && !SPLIT) {
      // (qg_row_pair) the same transforms, products and splits as below, in pairs
      constexpr int LS = FftPlan<LOG2N>::LDS;
      double2 w2[2][8], q[8];
      load_pair<LOG2N>(w2[0], ri, g, Q1, Q2, false);  // q1 + i q2
      load_pair<LOG2N>(w2[1], ri, g, P1, P2, true);   // ψx1 + i ψx2
      fftw_dif<W, +1, 2, false, false, false, PR>(w2, c.t, wt, tq, line, LS);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        q[s] = w2[0][s];
        w2[0][s] = make_double2(w2[1][s].x * q[s].x, w2[1][s].y * q[s].y);  // ψx q (swqg/TwoLayerQG.jl:169)
      }
      load_pair<LOG2N>(w2[1], ri, g, Py1, Py2, false);  // ψy1 + i ψy2
      fftw_dif<W, +1, 1, true, false, false, PR>(reinterpret_cast<V1>(w2[1]), c.t, wt, tq, line + LS, 0);
#pragma unroll
      for (int s = 0; s < 8; ++s) w2[1][s] = make_double2(w2[1][s].x * q[s].x, w2[1][s].y * q[s].y);  // ψy q (:177)
      fftw_dit<W, -1, 2, false, true, false, PR>(w2, c.t, wt, tq, line, LS);
      split_pairs<LOG2N, 2, PR>(w2, c.t, g, line, LS, [&](int cc, int, int s, double2 a, double2 b) {
        const int o = ri.ofwd(g, s);
        Mo[(2 * cc) * MF + o] = a;
        Mo[(2 * cc + 1) * MF + o] = b;
      });
      return;
    }
    double2 q[8];
    // q1 + i q2
    load_pair<LOG2N>(v, ri, g, Q1, Q2, false);
    inv(v);
#pragma unroll
    for (int s = 0; s < 8; ++s) q[s] = v[s];
    // fwd + store_pair (the split folded into the transform where it can be)
    auto fwd_store = [&](double2* A, double2* B) {
      if constexpr (W > 0 && SW_SPLIT_FOLD && !ALIAS) {
        fftw_dit_split<W, 1, FL>(reinterpret_cast<V1>(v), c.t, g.kc, wnt(), tq, line, 0,
                                 [&](int, int, int s, double2 a, double2 b) {
                                   const int o = ri.ofwd(g, s);
                                   A[o] = a;
                                   B[o] = b;
                                 });
      } else {
        fwd(v);
        store_pair<LOG2N, row_fly<MODEL, LOG2N>(), PR>(v, ri, g, line, A, B);
      }
    };
    const int part = SPLIT ? (int)blockIdx.y : -1;
    const long long MA = ma_field(g);  // aliased columns × rows per field
    if (part != 1) {
      // ψx1 + i ψx2;  ψx q per layer (swqg/TwoLayerQG.jl:169)
      load_pair<LOG2N>(v, ri, g, P1, P2, true);
      inv(v);
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = make_double2(v[s].x * q[s].x, v[s].y * q[s].y);
      fwd_store(Mo, Mo + MF);
      if constexpr (ALIAS) store_alias_pair<LOG2N, ma_nfa(MODEL)>(v, c.t, g, line, Ma, Ma + MA, y + g.y0);
    }
    if (part != 0) {
      // ψy q per layer (:177)
      load_pair<LOG2N>(v, ri, g, Py1, Py2, false);
      inv(v);
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = make_double2(v[s].x * q[s].x, v[s].y * q[s].y);
      fwd_store(Mo + 2 * MF, Mo + 3 * MF);
      if constexpr (ALIAS)
        store_alias_pair<LOG2N, ma_nfa(MODEL)>(v, c.t, g, line, Ma + 2 * MA, Ma + 3 * MA, y + g.y0);
    }
  }
}

// ===========================================================================
// 2LQG / MultiLayerQG row with half-length real transforms.  Each real line
// of N = nx points travels alone as one complex line of M = N/2 points,
// z[m] = x[2m] + i x[2m+1] (W = exp(-2πi/N), all transforms unnormalised):
//   c2r: Z[k] = (X[k] + conj X[M-k]) + i conj(W^k) (X[k] - conj X[M-k]),
//        k < M, then z = IDFT_M(Z)
//   r2c: Z = DFT_M(z), X[k] = E + W^k O, E = (Z[k] + conj Z[M-k]) / 2,
//        O = (Z[k] - conj Z[M-k]) / 2i
// Products of physical fields are products of the re and im parts.  A line
// buffer holds M points (64 KB at nx = 8192), so two rows, as two blocks of
// M/8 threads, share a CU where the full-length pair transform of k_row
// holds one 1024-thread block.  Same outputs as k_row
// (swqg/TwoLayerQG.jl:157-179): 0,1 ψx q per layer, 2,3 ψy q per layer.
// Thread t holds k = t + s·M/8; the mirrors M - k are loaded by the thread
// itself (the same row's lines, cache hits) rather than exchanged in LDS.
// ===========================================================================
template <int LOG2N>
struct RowH {
  static constexpr int N = 1 << LOG2N, M = N / 2, LM = LOG2N - 1, NTH = M / 8;
  // inverse-layout offset of wavenumber kk of local row y
  __device__ __forceinline__ static int inv(const Geom& g, int kk, int y) {
    if (SW_ROW_CLOSED && g.nslab == 1)
      return RowIdx<LOG2N>::row_inv(g, y) + 8 * (kk >> 1) + (g.tcm ? 4 : 1) * (kk & 1);
    return midx_i(g, kk, y);
  }
  __device__ __forceinline__ static int fwd(const Geom& g, int k, int y) {
    if (SW_ROW_CLOSED && g.nslab == 1) return RowIdx<LOG2N>::fwd0(g, k, y);
    return midx(g, k, y);
  }
  // W^(t + s M/8) = W^t · exp(-2πi s/16)
  __device__ __forceinline__ static double2 wk(double2 wt, int s) {
    constexpr double c1 = 0.92387953251128675613, s1 = 0.38268343236508977173, h = 0.70710678118654752440;
    const double cs[8] = {1.0, c1, h, s1, 0.0, -s1, -h, -c1};
    const double sn[8] = {0.0, s1, h, c1, 1.0, c1, h, s1};
    if (s == 0) return wt;
    return cmul(wt, make_double2(cs[s], -sn[s]));
  }
};

// Spectral sources of load_real_h: ld(o) issues the loads of mixed offset o,
// val(raw, kk) forms the x-spectral value at wavenumber kk.
struct SrcField {  // A, times ik when deriv
  const double2* A;
  bool deriv;
  using Raw = double2;
  __device__ __forceinline__ static Raw zero() { return zero2(); }
  __device__ __forceinline__ Raw ld(int o) const { return mix_ld_row(A + o); }
  __device__ __forceinline__ double2 val(const Raw& r, int kk, const Geom& g) const {
    return deriv ? cmul_i(r, kk * g.mk) : r;
  }
};
struct SrcZeta {  // RSW ζ̂ = ik V̂ − Ûy (x-spectral, per element)
  const double2 *V, *Uy;
  struct Raw {
    double2 v, uy;
  };
  __device__ __forceinline__ static Raw zero() { return Raw{zero2(), zero2()}; }
  __device__ __forceinline__ Raw ld(int o) const { return Raw{mix_ld_row(V + o), mix_ld_row(Uy + o)}; }
  __device__ __forceinline__ double2 val(const Raw& r, int kk, const Geom& g) const {
    return csub(cmul_i(r.v, kk * g.mk), r.uy);
  }
};

// The half rows' live band kc (KC > 0: known at compile time — the 2/3 rule
// on the full-length line, kc = N/3 — so every slot that is wholly live or
// wholly dead resolves at compile time and only the boundary slot selects per
// lane; round 6, SW_ROWH_KC; KC = 0: g.kc at run time)
template <int KC>
__device__ __forceinline__ int live_kc(const Geom& g) {
  return KC > 0 ? KC : g.kc;
}

// c2r input of one real field: v[s] = Z[t + s NTH].  Loads in two batches of
// four slots (eight loads per source array in flight)
template <int LOG2N, typename Src, int KC = 0>
__device__ __forceinline__ void load_real_h(double2 (&v)[8], const Geom& g, int t, int y, const Src& src,
                                            double2 wt) {
  using H = RowH<LOG2N>;
  const int kc = live_kc<KC>(g);
  // offsets and W^k formed per call, not kept across the row's calls
  asm volatile("" : "+v"(t), "+v"(wt.x), "+v"(wt.y));
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    typename Src::Raw a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * hb + j, k = t + s * H::NTH, km = H::M - k;
      a[j] = b[j] = Src::zero();
      // (all: every lane of the slot live — no clamp, no select)
      const bool alla = (s + 1) * H::NTH <= kc, allb = H::M - s * H::NTH < kc;
      if (s * H::NTH < kc) a[j] = src.ld(H::inv(g, (alla || k < kc) ? k : 0, y));
      if (H::M - (s + 1) * H::NTH < kc) b[j] = src.ld(H::inv(g, (allb || km < kc) ? km : 0, y));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * hb + j, k = t + s * H::NTH, km = H::M - k;
      const bool alla = (s + 1) * H::NTH <= kc, allb = H::M - s * H::NTH < kc;
      double2 x, xm;
      if constexpr (std::is_same<Src, SrcField>::value) {  // (the 2LQG row's register budget: this order)
        x = (alla || k < kc) ? a[j] : zero2();
        xm = (allb || km < kc) ? b[j] : zero2();
        if (s == 0 && k == 0) x.y = 0.0;
        if (src.deriv) {
          x = cmul_i(x, k * g.mk);
          xm = cmul_i(xm, km * g.mk);
        }
      } else {
        x = (alla || k < kc) ? src.val(a[j], k, g) : zero2();
        xm = (allb || km < kc) ? src.val(b[j], km, g) : zero2();
        if (s == 0 && k == 0) x.y = 0.0;  // numpy's c2r rule; X[M] is never live
      }
      const double2 S = cadd(x, cconj(xm)), D = csub(x, cconj(xm));
      const double2 T = cmul(D, cconj(H::wk(wt, s)));
      v[s] = make_double2(S.x - T.y, S.y + T.x);
    }
  }
}

// RSW half row: the c2r inputs of v and of ζ = ik V̂ − Ûy from ONE read of V
// (with Uy), the same arithmetic as load_real_h with SrcField{V} and
// SrcZeta{V, Uy} (bitwise)
template <int LOG2N, int KC = 0>
__device__ __forceinline__ void load_v_zeta_h(double2 (&v)[8], double2 (&z)[8], const Geom& g, int t, int y,
                                              const double2* __restrict__ V, const double2* __restrict__ Uy,
                                              double2 wt) {
  using H = RowH<LOG2N>;
  const int kc = live_kc<KC>(g);
  asm volatile("" : "+v"(t), "+v"(wt.x), "+v"(wt.y));
  const SrcZeta sz{V, Uy};
  auto comb = [&](double2 x, double2 xm, int s) {
    const double2 S = cadd(x, cconj(xm)), D = csub(x, cconj(xm));
    const double2 T = cmul(D, cconj(H::wk(wt, s)));
    return make_double2(S.x - T.y, S.y + T.x);
  };
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    SrcZeta::Raw a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * hb + j, k = t + s * H::NTH, km = H::M - k;
      a[j] = b[j] = SrcZeta::zero();
      const bool alla = (s + 1) * H::NTH <= kc, allb = H::M - s * H::NTH < kc;
      if (s * H::NTH < kc) a[j] = sz.ld(H::inv(g, (alla || k < kc) ? k : 0, y));
      if (H::M - (s + 1) * H::NTH < kc) b[j] = sz.ld(H::inv(g, (allb || km < kc) ? km : 0, y));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int s = 4 * hb + j, k = t + s * H::NTH, km = H::M - k;
      const bool la = (s + 1) * H::NTH <= kc || k < kc, lb = H::M - s * H::NTH < kc || km < kc;
      double2 x = la ? a[j].v : zero2(), xm = lb ? b[j].v : zero2();
      if (s == 0 && k == 0) x.y = 0.0;
      v[s] = comb(x, xm, s);
      x = la ? sz.val(a[j], k, g) : zero2();
      xm = lb ? sz.val(b[j], km, g) : zero2();
      if (s == 0 && k == 0) x.y = 0.0;
      z[s] = comb(x, xm, s);
    }
  }
}

// r2c output of one real field from v[s] = Z[t + s NTH]: emit(k, s, X[k]) for
// live k (one LDS round trip for the mirrors Z[M - k])
template <int LOG2N, int KC = 0, typename Emit>
__device__ __forceinline__ void split_real_h(const double2 (&v)[8], int t, const Geom& g, double2* line,
                                             double2 wt, Emit emit) {
  using H = RowH<LOG2N>;
  const int kc = live_kc<KC>(g);
  asm volatile("" : "+v"(t), "+v"(wt.x), "+v"(wt.y));
  lds_barrier();  // previous LDS readers are done
#pragma unroll
  for (int s = 0; s < 8; ++s) line[LP<H::LM>(t + s * H::NTH)] = v[s];
  lds_barrier();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = t + s * H::NTH;
    if (s * H::NTH < kc && ((s + 1) * H::NTH <= kc || k < kc)) {
      const double2 zk = v[s];
      const double2 zn = line[LP<H::LM>((H::M - k) & (H::M - 1))];
      const double2 E = make_double2(0.5 * (zk.x + zn.x), 0.5 * (zk.y - zn.y));
      const double2 O = make_double2(0.5 * (zk.y + zn.y), -0.5 * (zk.x - zn.x));
      emit(k, s, cadd(E, cmul(H::wk(wt, s), O)));
    }
  }
}

#ifndef SW_MINW_ROW_H
#define SW_MINW_ROW_H 4
#endif
#ifndef SW_ROW_H_FLY
#define SW_ROW_H_FLY true
#endif
// rows per block of the half-length rows (experiment knob; NB = 2: the two
// rows of a block write the two 32-B halves of each 64-B half-line of a 2×4
// forward tile in lockstep, and blocks b, b + 8 (one XCD) the tile's other
// two rows — row0_of_block)
#ifndef SW_ROWH_NB
#define SW_ROWH_NB 1
#endif
#ifndef SW_RSW_ROWH_NB
#define SW_RSW_ROWH_NB 1
#endif
template <int LOG2N, bool RSW = false>
__host__ __device__ constexpr int rowh_nb();
// local row of line ln of block b (NB rows per block)
template <int NB>
__device__ __forceinline__ int rowh_row(int b, int nb, int ln) {
  return NB == 1 ? col_of_block(b, nb) : row0_of_block<NB>(b, nb) + ln;
}
template <int LOG2N, int KC = 0>
static __global__ void __launch_bounds__(RowH<LOG2N>::NTH * rowh_nb<LOG2N>(), SW_MINW_ROW_H)
    k_row_qg_h(Geom g_in, Phys p, const double2* __restrict__ Mi, double2* __restrict__ Mo,
               const double2* __restrict__ tw, int yoff) {
  // (KC is launched only on one slab, but telling the half rows so — their
  // slab-division paths compiled out — measured slower: config 5 row
  // 1550-1595 → 1626-1632 µs, tools/ab/r6_slab1.sh)
  const Geom& g = g_in;
  using H = RowH<LOG2N>;
  constexpr int NB = rowh_nb<LOG2N>();
  extern __shared__ double2 smem_all[];
  const int ln = NB == 1 ? 0 : (int)threadIdx.x / H::NTH;
  const int t = threadIdx.x - ln * H::NTH;
  double2* smem = smem_all + ln * FftPlan<H::LM>::LDS;
  const int y = yoff + rowh_row<NB>(blockIdx.x, gridDim.x, ln);
  Twiddles<H::LM, SW_ROW_H_FLY> tws;  // stage twiddles read per stage: register room
  tws.load(t, tw, 1);                    // W_M^j = W_N^(2j)
  const double2 wt = tw[t];
  const long long MF = g.mfield;
  // the decimated transforms (roww) of the M-point lines
  constexpr int W = roww_h<H::LM>();
  Twiddles<9, SW_ROW_H_FLY> tq;
  double2 wm = zero2();
  if constexpr (W > 0) {
    tq.load(t & 63, tw, H::LM - 9 + 1);
    wm = tw[2 * t];  // W_M^t
  }
  using V1 = double2(&)[1][8];
  auto inv = [&](double2(&x)[8]) {
    if constexpr (W > 0) fftw_dif<W, +1, 1, true, SW_ROW_H_FLY>(reinterpret_cast<V1>(x), t, wm, tq, smem, 0);
    else fft_line<H::LM, +1>(x, t, tws, smem);
  };
  auto fwd = [&](double2(&x)[8]) {
    if constexpr (W > 0) fftw_dit<W, -1, 1, SW_ROW_H_FLY>(reinterpret_cast<V1>(x), t, wm, tq, smem, 0);
    else fft_line<H::LM, -1>(x, t, tws, smem);
  };
  double2 q[8], v[8];
#pragma unroll 1
  for (int l = 0; l < 2; ++l) {
    load_real_h<LOG2N, SrcField, KC>(q, g, t, y, SrcField{Mi + l * MF, false}, wt);
    inv(q);
#pragma unroll 1
    for (int d = 0; d < 2; ++d) {  // ψx q (:169), ψy q (:177)
      load_real_h<LOG2N, SrcField, KC>(v, g, t, y, SrcField{Mi + (d == 0 ? 2 + l : 4 + l) * MF, d == 0}, wt);
      inv(v);
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = make_double2(v[s].x * q[s].x, v[s].y * q[s].y);
      fwd(v);
      double2* O = Mo + (2 * d + l) * MF;
      split_real_h<LOG2N, KC>(v, t, g, smem, wt, [&](int k, int, double2 X) { O[H::fwd(g, k, y)] = X; });
    }
  }
}

// RSW row with half-length real transforms (the vorticity form of k_row,
// rsw/RotatingShallowWater.jl:140-230): 4 inverse + 5 forward real lines
// (k_row: 2 + 2 complex pairs and the real vη line as a full complex FFT).
// Live: u, v, η (then ζ in η's registers), one product line; K̂ is kept in
// u's registers (dead by then) for P = -ik K̂ + (ζv)^.
#ifndef SW_MINW_ROW_RSW_H
#define SW_MINW_ROW_RSW_H 2
#endif
// ζ's c2r input formed from the same read of V as v's and parked in a second
// line buffer of LDS until η's registers are free (0: V read twice)
#ifndef SW_RSW_ROWH_ZPARK
#define SW_RSW_ROWH_ZPARK 1
#endif
template <int LOG2N>
__host__ __device__ constexpr int rsw_rowh_lines() { return SW_RSW_ROWH_ZPARK ? 2 : 1; }
template <int LOG2N, bool RSW>
__host__ __device__ constexpr int rowh_nb() {
  if constexpr (RSW)
    return (SW_RSW_ROWH_NB == 2 && 2 * rsw_rowh_lines<LOG2N>() * FftPlan<LOG2N - 1>::LDS * 16 <= 160 * 1024) ? 2 : 1;
  else
    return SW_ROWH_NB;
}
template <int LOG2N, int KC = 0>
static __global__ void __launch_bounds__((RowH<LOG2N>::NTH * rowh_nb<LOG2N, true>()), SW_MINW_ROW_RSW_H)
    k_row_rsw_h(Geom g_in, Phys p, const double2* __restrict__ Mi, double2* __restrict__ Mo,
                const double2* __restrict__ tw, int yoff) {
  // (KC is launched only on one slab, but telling the half rows so — their
  // slab-division paths compiled out — measured slower: config 5 row
  // 1550-1595 → 1626-1632 µs, tools/ab/r6_slab1.sh)
  const Geom& g = g_in;
  using H = RowH<LOG2N>;
  constexpr int NB = rowh_nb<LOG2N, true>();
  extern __shared__ double2 smem_all[];
  const int ln = NB == 1 ? 0 : (int)threadIdx.x / H::NTH;
  const int t = threadIdx.x - ln * H::NTH;
  double2* smem = smem_all + ln * rsw_rowh_lines<LOG2N>() * FftPlan<H::LM>::LDS;
  double2* park = smem + FftPlan<H::LM>::LDS;  // ZPARK: ζ's c2r input, slots t + s NTH
  const int y = yoff + rowh_row<NB>(blockIdx.x, gridDim.x, ln);
  Twiddles<H::LM> tws;
  tws.load(t, tw, 1);  // W_M^j = W_N^(2j)
  const double2 wt = tw[t];
  // the decimated transforms (roww) of the M-point lines; PRE: a barrier
  // first (the previous split's mirror reads span every wave's region)
  constexpr int W = roww_h<H::LM, true>();
  Twiddles<9> tq;
  double2 wm = zero2();
  if constexpr (W > 0) {
    tq.load(t & 63, tw, H::LM - 9 + 1);
    wm = tw[2 * t];  // W_M^t
  }
  using V1 = double2(&)[1][8];
  auto inv = [&](double2(&x)[8]) {
    if constexpr (W > 0) fftw_dif<W, +1, 1, true, false>(reinterpret_cast<V1>(x), t, wm, tq, smem, 0);
    else fft_line<H::LM, +1>(x, t, tws, smem);
  };
  auto fwd = [&](double2(&x)[8], auto pre) {
    if constexpr (W > 0) fftw_dit<W, -1, 1, false, decltype(pre)::value>(reinterpret_cast<V1>(x), t, wm, tq, smem, 0);
    else fft_line<H::LM, -1>(x, t, tws, smem);
  };
  using Pre = std::true_type;
  using NoPre = std::false_type;
  const long long MF = g.mfield;
  const double2 *U = Mi, *V = Mi + MF, *Hh = Mi + 2 * MF, *Uy = Mi + 3 * MF;
  double2 u[8], v[8], e[8], w[8];
  load_real_h<LOG2N, SrcField, KC>(u, g, t, y, SrcField{U, false}, wt);
  inv(u);
  if constexpr (SW_RSW_ROWH_ZPARK) {
    load_v_zeta_h<LOG2N, KC>(v, e, g, t, y, V, Uy, wt);
#pragma unroll
    for (int s = 0; s < 8; ++s) park[t + s * H::NTH] = e[s];  // read back by this thread only
  } else {
    load_real_h<LOG2N, SrcField, KC>(v, g, t, y, SrcField{V, false}, wt);
  }
  inv(v);
  load_real_h<LOG2N, SrcField, KC>(e, g, t, y, SrcField{Hh, false}, wt);
  inv(e);
  auto prod = [&](const double2 (&a)[8], const double2 (&b)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) w[s] = make_double2(a[s].x * b[s].x, a[s].y * b[s].y);
  };
  // 4: (vη)^
  prod(v, e);
  fwd(w, NoPre{});
  split_real_h<LOG2N, KC>(w, t, g, smem, wt, [&](int k, int, double2 X) { Mo[4 * MF + H::fwd(g, k, y)] = X; });
  // 3: Q = -ik (uη)^
  prod(u, e);
  fwd(w, Pre{});
  split_real_h<LOG2N, KC>(w, t, g, smem, wt,
                      [&](int k, int, double2 X) { Mo[3 * MF + H::fwd(g, k, y)] = cmul_i(X, -(k * g.mk)); });
  // ζ = vx - uy in η's registers
  if constexpr (SW_RSW_ROWH_ZPARK) {
#pragma unroll
    for (int s = 0; s < 8; ++s) e[s] = park[t + s * H::NTH];
  } else {
    load_real_h<LOG2N, SrcZeta, KC>(e, g, t, y, SrcZeta{V, Uy}, wt);
  }
  inv(e);
  // 2: (ζu)^
  prod(e, u);
  fwd(w, NoPre{});
  split_real_h<LOG2N, KC>(w, t, g, smem, wt, [&](int k, int, double2 X) { Mo[2 * MF + H::fwd(g, k, y)] = X; });
  // 1: K̂, K = (u² + v²)/2; kept in u
#pragma unroll
  for (int s = 0; s < 8; ++s)
    w[s] = make_double2(0.5 * (u[s].x * u[s].x + v[s].x * v[s].x), 0.5 * (u[s].y * u[s].y + v[s].y * v[s].y));
  fwd(w, Pre{});
  split_real_h<LOG2N, KC>(w, t, g, smem, wt, [&](int k, int s, double2 X) {
    Mo[MF + H::fwd(g, k, y)] = X;
    u[s] = X;
  });
  // 0: P = -ik K̂ + (ζv)^
  prod(e, v);
  fwd(w, Pre{});
  split_real_h<LOG2N, KC>(w, t, g, smem, wt,
                      [&](int k, int s, double2 X) { Mo[H::fwd(g, k, y)] = cadd(cmul_i(u[s], -(k * g.mk)), X); });
}

#ifndef SW_RSW_ROW_HALF_MIN
#define SW_RSW_ROW_HALF_MIN 12
#endif
template <int LOG2N>
__host__ __device__ constexpr bool rsw_row_half() {
  return LOG2N >= SW_RSW_ROW_HALF_MIN && LOG2N >= 11;
}

// lengths whose 2LQG row runs k_row_qg_h (SW_QG_ROW_HALF_MIN: from this
// log2 nx up; measured in DESIGN.md §3e: 8192 -12 %, 4096 -3 %, 2048 neutral)
#ifndef SW_QG_ROW_HALF_MIN
#define SW_QG_ROW_HALF_MIN 12
#endif
template <int LOG2N>
__host__ __device__ constexpr bool qg_row_half() {
  return LOG2N >= SW_QG_ROW_HALF_MIN && LOG2N >= 10;
}

// ===========================================================================
// col_fwd: forward FFT along y of the row outputs, combine into N (live rows).
// N_f is the sum of at most two forward y-transforms of row outputs, each
// with a per-mode multiplier (nterms):
//   RSW (rsw/RotatingShallowWater.jl:174-226, vorticity form of k_row):
//     N_u = F(P),  N_v = -il F(K̂) - F((ζu)^),  N_η = F(Q) - il F((vη)^)
//   QG2 (swqg/TwoLayerQG.jl:171,179): N_l = -il F(A_l) + ik F(B_l)
// ===========================================================================
//   TY (thomasyamada/ThomasYamada.jl:166-262, k_row outputs):
//     N_ζ = F(0) + l F(1) + l² F(2),  N_uc = F(3),  N_vc = il F(4) + F(5),
//     N_pc = F(6);  plus the linear terms (:142-145) from the calcN input
enum { MUL_ONE = 0, MUL_NEG, MUL_NIK, MUL_NIL, MUL_PIK, MUL_PIL, MUL_L, MUL_L2 };
struct NTerms {
  int fa, ma, fb, mb, fc, mc;  // fb < 0: one term; fc < 0: at most two
};
template <int MODEL>
__device__ __forceinline__ NTerms nterms(int f) {
  if constexpr (MODEL == MODEL_RSW) {
    if (f == 0) return NTerms{0, MUL_ONE, -1, MUL_ONE, -1, MUL_ONE};
    if (f == 1) return NTerms{1, MUL_NIL, 2, MUL_NEG, -1, MUL_ONE};
    return NTerms{3, MUL_ONE, 4, MUL_NIL, -1, MUL_ONE};
  } else if constexpr (MODEL == MODEL_RSWA) {
    if (f == 0) return NTerms{0, MUL_NEG, -1, MUL_ONE, -1, MUL_ONE};
    if (f == 1) return NTerms{1, MUL_NEG, -1, MUL_ONE, -1, MUL_ONE};
    return NTerms{2, MUL_ONE, 3, MUL_NIL, -1, MUL_ONE};
  } else if constexpr (MODEL == MODEL_TY) {
    if (f == 0) return NTerms{0, MUL_ONE, 1, MUL_L, 2, MUL_L2};
    if (f == 1) return NTerms{3, MUL_ONE, -1, MUL_ONE, -1, MUL_ONE};
    if (f == 2) return NTerms{4, MUL_PIL, 5, MUL_ONE, -1, MUL_ONE};
    return NTerms{6, MUL_ONE, -1, MUL_ONE, -1, MUL_ONE};
  } else {
    return NTerms{f, MUL_NIL, 2 + f, MUL_PIK, -1, MUL_ONE};
  }
}
__device__ __forceinline__ double2 apply_mul(double2 a, int mul, double k, double l) {
  switch (mul) {
    case MUL_ONE: return a;
    case MUL_NEG: return make_double2(-a.x, -a.y);
    case MUL_NIK: return cmul_i(a, -k);
    case MUL_NIL: return cmul_i(a, -l);
    case MUL_PIK: return cmul_i(a, k);
    case MUL_PIL: return cmul_i(a, l);
    case MUL_L: return cscale(a, l);
    default: return cscale(a, l * l);
  }
}
template <int MODEL>
constexpr int model_nf() {
  return (MODEL == MODEL_RSW || MODEL == MODEL_RSWA) ? 3 : (MODEL == MODEL_TY ? 4 : 2);
}

// Thomas–Yamada calcN!'s linear terms (thomasyamada/ThomasYamada.jl:142-145)
// of field grp added to its nonlinear part r, from the dealiased calcN input
// X (ζ, uc, vc, pc) at mode i; one definition for k_col_fwd and the updates
// that assemble a split N (assemble_terms)
__device__ __forceinline__ double2 ty_linear_terms(const double2* __restrict__ X, long long cf, long long i, int grp,
                                                   double k, double l, double2 r) {
#pragma clang fp contract(off)
  if (grp == 1) return cadd(csub(X[2 * cf + i], cmul_i(X[3 * cf + i], k)), r);  // vc - ik pc
  if (grp == 2) {                                                                 // -uc - il pc
    const double2 u = X[cf + i];
    return cadd(csub(make_double2(-u.x, -u.y), cmul_i(X[3 * cf + i], l)), r);
  }
  if (grp == 3) return cadd(csub(cmul_i(X[cf + i], -k), cmul_i(X[2 * cf + i], l)), r);  // -ik uc - il vc
  return r;
}

// SPLIT (short columns, sw_api.cpp fsplit): grid (columns, 3 × fields), one
// term of N_f (nterms) per block — its transform and multiplier, no sum and
// no linear terms — into N (term 0), T1 or T2; the update that consumes N
// adds them in k_col_fwd's order (assemble_terms): bitwise the same N
template <int MODEL, int LOG2N, bool SPLIT = false, int BAND = 0>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW_M(MODEL, LOG2N))
    k_col_fwd(Geom g, Phys p, const double2* __restrict__ Mf, double2* __restrict__ N,
              const double2* __restrict__ X, const double2* __restrict__ tw, int gbase,
              double2* __restrict__ T1, double2* __restrict__ T2) {
  band_fix<LOG2N, BAND>(g);
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int krl = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
  const int grp = gbase + (SPLIT ? (int)blockIdx.y / 3 : (int)blockIdx.y);
  const int term = SPLIT ? (int)blockIdx.y % 3 : -1;
  if constexpr (SPLIT) {
    const NTerms nt0 = nterms<MODEL>(grp);
    if ((term == 1 && nt0.fb < 0) || (term == 2 && nt0.fc < 0)) return;
  }
  const bool live = krl < g.kcn;
  if (B::NB == 1 && !live) return;
  const int krA = krl < g.kcl ? krl : g.kcl - 1;  // in-bounds address
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  constexpr bool CD = col_dec<LOG2N, MODEL>();  // the family's stored-row order
  ColTw<LOG2N, CD> tws;
  tws.load(c.t, tw);
  const double k = (g.kr0 + krl) * g.mk;
  const long long MF = g.mfield;
  double2 v[8], acc[8];

  auto load_col = [&](const double2* Mfield) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double2 t = mix_ld_col(Mfield + midc(g, krA, cpos<LOG2N, CD>(c.t, s)));
      v[s] = live ? t : zero2();
    }
  };

  const NTerms nt = nterms<MODEL>(grp);
  if constexpr (SPLIT) {  // one term: its transform and multiplier
    const int src = term == 0 ? nt.fa : (term == 1 ? nt.fb : nt.fc);
    const int mul = term == 0 ? nt.ma : (term == 1 ? nt.mb : nt.mc);
    load_col(Mf + src * MF);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
    if (live) {
      double2* D = (term == 0 ? N : (term == 1 ? T1 : T2)) + (long long)grp * g.cfield + (long long)krl * g.LrP;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int j = compact_of(g, c.t + s * NT);
        if (j >= 0) D[j] = apply_mul(v[s], mul, k, lwav(g, c.t + s * NT));
      }
    }
    return;
  }
  // fft_line leaves F[m = t + s*NT] in v[s]; only live rows are written
  load_col(Mf + nt.fa * MF);
  col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
  for (int s = 0; s < 8; ++s) acc[s] = apply_mul(v[s], nt.ma, k, lwav(g, c.t + s * NT));
  if (nt.fb >= 0) {
    load_col(Mf + nt.fb * MF);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = cadd(acc[s], apply_mul(v[s], nt.mb, k, lwav(g, c.t + s * NT)));
  }
  if (MODEL == MODEL_TY && nt.fc >= 0) {
    load_col(Mf + nt.fc * MF);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = cadd(acc[s], apply_mul(v[s], nt.mc, k, lwav(g, c.t + s * NT)));
  }
  if (live) {
    double2* Nf = N + (long long)grp * g.cfield + (long long)krl * g.LrP;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = compact_of(g, c.t + s * NT);
      if (j >= 0) {
        double2 r = acc[s];
        if constexpr (MODEL == MODEL_QG2) {
          if (p.model == MODEL_MLQG) {
            const long long i = (long long)krl * g.LrP + j;
            r = mlqg_linear_terms(p, k, lwav(g, c.t + s * NT), X[i], X[g.cfield + i], grp, r);
          }
        }
        if constexpr (MODEL == MODEL_TY)  // linear terms, from the dealiased calcN input
          r = ty_linear_terms(X, g.cfield, (long long)krl * g.LrP + j, grp, k, lwav(g, c.t + s * NT), r);
        Nf[j] = r;
      }
    }
  }
}

// N at the aliased modes of region ga (aliased-state tracking, one slab;
// sw_api.cpp alias_geom) with k_col_fwd's y-transforms and multipliers
// (nterms): 2LQG N_l = -il F(A_l) + ik F(B_l) (swqg/TwoLayerQG.jl:171,179),
// RSW in the advective form (MODEL_RSWA, rsw/RotatingShallowWater.jl:140-230,
// exact on every mode).  Region 0 = the columns kr in [kc, nx/2] (row outputs
// from the row pass's aliased output Ma, [field][kr - kc][y]); region 1 = the
// rows l in the 2/3-rule band of the live columns (the forward mixed fields,
// as k_col_fwd reads them).  grid: (columns, output fields).
template <int MODEL, int LOG2N>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW_M(MODEL, LOG2N))
    k_col_fwd_alias(Geom g, Geom ga, int region, Phys p, const double2* __restrict__ Mf,
                    const double2* __restrict__ Ma, double2* __restrict__ N, const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int col = blockIdx.x * B::NB + c.ln;  // column of the region
  const int f = blockIdx.y;                   // output field
  const bool live = col < ga.kcn;
  const int colA = live ? col : 0;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  constexpr bool CD = col_dec<LOG2N, MODEL>();  // the family's stored-row order
  ColTw<LOG2N, CD> tws;
  tws.load(c.t, tw);
  const double k = (ga.kr0 + colA) * g.mk;
  const long long MA = ma_field(g);
  double2 v[8], acc[8];
  auto load_col = [&](int fi) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int m = cpos<LOG2N, CD>(c.t, s);  // stored row
      const double2 t = region == 0 ? Ma[fi * MA + ma_off(g, ma_nfa(MODEL), colA, m)] : Mf[fi * g.mfield + midc(g, colA, m)];
      v[s] = live ? t : zero2();
    }
  };
  const NTerms nt = nterms<MODEL>(f);
  load_col(nt.fa);
  col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
  for (int s = 0; s < 8; ++s) acc[s] = apply_mul(v[s], nt.ma, k, lwav(g, c.t + s * NT));
  if (nt.fb >= 0) {
    load_col(nt.fb);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = cadd(acc[s], apply_mul(v[s], nt.mb, k, lwav(g, c.t + s * NT)));
  }
  if (nt.fc >= 0) {  // Thomas–Yamada's N_ζ (the linear terms vanish here: calcN! dealiases its input)
    load_col(nt.fc);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = cadd(acc[s], apply_mul(v[s], nt.mc, k, lwav(g, c.t + s * NT)));
  }
  if (live) {
    double2* Nf = N + (long long)f * ga.cfield + (long long)col * ga.LrP;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = compact_of(ga, c.t + s * NT);
      if (j >= 0 && j < ga.Lr) Nf[j] = acc[s];
    }
  }
}

// ===========================================================================
// stepper updates: per-mode operations shared by the elementwise kernels and
// the fused column kernel (identical arithmetic on both paths)
// ===========================================================================
// compact index i -> global column kr, live row j; false for padding
__device__ __forceinline__ bool mode_of(const Geom& g, long long i, int& kr, int& j) {
  const int krl = (int)(i / g.LrP);
  j = (int)(i - (long long)krl * g.LrP);
  kr = g.kr0 + krl;
  return krl < g.kcn && j < g.Lr;
}

template <int NF>
__device__ __forceinline__ void model_L(const Phys& p, double k, double l, cplx L[NF][NF]) {
  if constexpr (NF == 3) {
    rsw_L(p, k, l, L);
  } else {
    if (p.model == MODEL_MLQG) {  // MultiLayerQG Equation: L = -ν K^(2nν) per layer
      const double D = -(p.nu * ipow(k * k + l * l, p.nnu));
      L[0][0] = cx(D);
      L[0][1] = cx(0.0);
      L[1][0] = cx(0.0);
      L[1][1] = cx(D);
    } else {
      qg2_L(p, k, l, L);
    }
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
__device__ __forceinline__ void store_vec(double2* __restrict__ X, long long cf, long long i,
                                          const cplx x[NF]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) X[f * cf + i] = make_double2(x[f].re, x[f].im);
}

// the same for data used once per step (state_ld / state_st policy)
template <int NF, bool NT>
__device__ __forceinline__ void load_vec_once(const double2* __restrict__ X, long long cf, long long i,
                                              cplx x[NF]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const double2 t = state_ld<NT>(X + f * cf + i);
    x[f] = cx(t.x, t.y);
  }
}
template <int NF, bool NT>
__device__ __forceinline__ void store_vec_once(double2* __restrict__ X, long long cf, long long i,
                                               const cplx x[NF]) {
#pragma unroll
  for (int f = 0; f < NF; ++f) state_st<NT>(X + f * cf + i, make_double2(x[f].re, x[f].im));
}

template <int NF>
__device__ __forceinline__ void matvec(const cplx M[NF][NF], const cplx x[NF], cplx y[NF]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int r = 0; r < NF; ++r) {
    cplx s = cx(0.0);
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) s = s + M[r][cc] * x[cc];
    y[r] = s;
  }
}

// StepPtrs (sw_internal.hpp): h0 receives this step's history entry
// (FAB3: RHS, IFMAB3: N, RK4: the running combination acc).

// FF FilteredAB3 for field F of one mode:
//   RHS_F = N_F + (L·sol)_F;  x_F = sol_F + dt·(Euler | AB3);  x_F *= filter.
// Reads the old state (all fields, for L·sol) from a.sol and writes the new
// field to a.sol_out (a separate buffer, so fields can be updated one by one).
// The update proper, on operands already in registers: the old state s (all
// fields) and field F's RHS₋₁, RHS₋₂ (r1, r2; unused on Euler steps).
// Returns the new field F (x) and its RHS (history entry).  Branch-free
// (Euler/AB3 by select), so a kernel can issue several modes' loads at once.
// (L·s)_F of the RSW operator (rsw_L) without its zero parts: the same
// values as the complex matrix-vector product Σ_c L[F][c]·s_c (products by
// exact zeros and additions of them dropped; at most a zero's sign differs)
template <int F>
__device__ __forceinline__ cplx rsw_Ls(const Phys& p, double k, double l, const cplx (&s)[3]) {
#pragma clang fp contract(off)
  const double D = -(p.nu * ipow(k * k + l * l, p.nnu));
  if constexpr (F == 0) {  // [D, f, −i k Cg²]
    const double c = -k * p.Cg2;
    return cx((D * s[0].re + p.f * s[1].re) - c * s[2].im, (D * s[0].im + p.f * s[1].im) + c * s[2].re);
  } else if constexpr (F == 1) {  // [−f, D, −i l Cg²]
    const double c = -l * p.Cg2, mf = -p.f;
    return cx((mf * s[0].re + D * s[1].re) - c * s[2].im, (mf * s[0].im + D * s[1].im) + c * s[2].re);
  } else {  // [−i k, −i l, D]
    const double mk = -k, ml = -l;
    return cx((-(mk * s[0].im) - ml * s[1].im) + D * s[2].re, (mk * s[0].re + ml * s[1].re) + D * s[2].im);
  }
}

template <int NF, int F>
__device__ __forceinline__ void fab3_compute(const Geom& g, const Phys& p, int euler, double k, double l, cplx n,
                                             const cplx (&s)[NF], double2 r1, double2 r2, cplx& x, cplx& rhs) {
#pragma clang fp contract(off)
  const double filt = filter_value(g, p, k, l);
  const double dt = p.dt;
  cplx Ls = cx(0.0);
  if constexpr (NF == 3) {
    Ls = rsw_Ls<F>(p, k, l, s);
  } else {
    cplx L[NF][NF];
    model_L<NF>(p, k, l, L);
#pragma unroll
    for (int cc = 0; cc < NF; ++cc) Ls = Ls + L[F][cc] * s[cc];
  }
  rhs = cx(n.re + Ls.re, n.im + Ls.im);
  const cplx xe = s[F] + dt * rhs;
  const cplx xa = s[F] + dt * cx(23.0 / 12 * rhs.re - 16.0 / 12 * r1.x + 5.0 / 12 * r2.x,
                                 23.0 / 12 * rhs.im - 16.0 / 12 * r1.y + 5.0 / 12 * r2.y);
  const cplx xx = euler ? xe : xa;
  x = cx(xx.re * filt, xx.im * filt);
}

template <int NF, int F, bool NT>
__device__ __forceinline__ cplx op_fab3_field(const Geom& g, const Phys& p, const StepPtrs& a,
                                              long long i, double k, double l, cplx n) {
  const long long cf = g.cfield;
  cplx s[NF];
  load_vec_once<NF, NT>(a.sol, cf, i, s);
  // read even on Euler steps (in bounds); history is used once per step
  const double2 r1 = state_ld<NT>(a.h1 + F * cf + i), r2 = state_ld<NT>(a.h2 + F * cf + i);
  cplx x, rhs;
  fab3_compute<NF, F>(g, p, a.euler, k, l, n, s, r1, r2, x, rhs);
  state_st<NT>(a.h0 + F * cf + i, make_double2(rhs.re, rhs.im));
  a.sol_out[F * cf + i] = make_double2(x.re, x.im);  // the next col_inv reads it
  note_nonfinite(a.nan, nonfinite(x));
  return x;
}

template <int NF, bool NT>
__device__ __forceinline__ void op_fab3(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                        double k, double l, const cplx n[NF], cplx x[NF]) {
  x[0] = op_fab3_field<NF, 0, NT>(g, p, a, i, k, l, n[0]);
  x[1] = op_fab3_field<NF, 1, NT>(g, p, a, i, k, l, n[1]);
  if constexpr (NF == 3) x[2] = op_fab3_field<NF, 2, NT>(g, p, a, i, k, l, n[2]);
}

// utils/IFMAB3.jl:129-160: Euler for step < 3, else AB3 with E N₋₁, E2 N₋₂;
// then sol = E·(…); filter.  N becomes history.  E = exp(dt L), E2 =
// exp(2 dt L) evaluated per mode in closed form (sw_internal.hpp ExpOf).
// the new state x at mode i without stores (op_ifmab3; k_step_elem when N
// already sits in the history slot the op would store it to)
template <int NF, bool NT>
__device__ __forceinline__ void ifmab3_x(const Geom& g, const Phys& p, const StepPtrs& a, long long i, double k,
                                         double l, const cplx n[NF], cplx x[NF]) {
#pragma clang fp contract(off)
  const long long cf = g.cfield;
  cplx s[NF], y[NF];
  load_vec_once<NF, NT>(a.sol, cf, i, s);
  const double dt = p.dt;
  const auto E = ExpOf<NF>::make(p, k, l, dt);
  if (a.euler) {
#pragma unroll
    for (int f = 0; f < NF; ++f) y[f] = s[f] + dt * n[f];
  } else {
    cplx r1[NF], r2[NF], e1[NF], e2[NF];
    load_vec_once<NF, NT>(a.h1, cf, i, r1);
    load_vec_once<NF, NT>(a.h2, cf, i, r2);
    exp_apply(p, E, r1, e1);
    exp_apply(p, exp_double(p, E, dt), r2, e2);
#pragma unroll
    for (int f = 0; f < NF; ++f)
      y[f] = s[f] + dt * cx(23.0 / 12 * n[f].re - 16.0 / 12 * e1[f].re + 5.0 / 12 * e2[f].re,
                            23.0 / 12 * n[f].im - 16.0 / 12 * e1[f].im + 5.0 / 12 * e2[f].im);
  }
  exp_apply(p, E, y, x);
  if (p.use_filter) {
    const double filt = filter_value(g, p, k, l);
#pragma unroll
    for (int f = 0; f < NF; ++f) x[f] = cx(x[f].re * filt, x[f].im * filt);
  }
}
template <int NF, bool NT>
__device__ __forceinline__ void op_ifmab3(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                          double k, double l, const cplx n[NF], cplx x[NF]) {
  ifmab3_x<NF, NT>(g, p, a, i, k, l, n, x);
  store_vec_once<NF, NT>(a.h0, g.cfield, i, n);
  store_vec<NF>(a.sol_out, g.cfield, i, x);  // the next col_inv reads it
  note_state<NF>(a, x);
}

// Lawson IF-RK4, one calcN result per stage, H = exp(dt L / 2)
// in closed form, E = exp(dt L) from it (exp_double):
//   1: k1 -> acc = E k1;          x = H (u + dt/2 k1)
//   2: k2 -> acc += 2 H k2;       x = H u + dt/2 k2
//   3: k3 -> acc += 2 H k3;       x = E u + dt H k3
//   4: k4 -> u = E u + dt/6 (acc + k4), filtered;  x = u
template <int NF>
__device__ __forceinline__ void op_rk4(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                       double k, double l, const cplx n[NF], cplx x[NF]) {
#pragma clang fp contract(off)
  const long long cf = g.cfield;
  const double dt = p.dt;
  cplx u[NF], t[NF], acc[NF];
  load_vec<NF>(a.sol, cf, i, u);
  const auto H = ExpOf<NF>::make(p, k, l, 0.5 * dt);
  if (a.stage == 1) {
    exp_apply(p, exp_double(p, H, 0.5 * dt), n, acc);
#pragma unroll
    for (int f = 0; f < NF; ++f) t[f] = u[f] + (0.5 * dt) * n[f];
    exp_apply(p, H, t, x);
    store_vec<NF>(a.h0, cf, i, acc);
  } else if (a.stage == 2 || a.stage == 3) {
    cplx hk[NF];
    load_vec<NF>(a.h0, cf, i, acc);
    exp_apply(p, H, n, hk);
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[f] = acc[f] + 2.0 * hk[f];
    if (a.stage == 2) {
      exp_apply(p, H, u, t);
#pragma unroll
      for (int f = 0; f < NF; ++f) x[f] = t[f] + (0.5 * dt) * n[f];
    } else {
      exp_apply(p, exp_double(p, H, 0.5 * dt), u, t);
#pragma unroll
      for (int f = 0; f < NF; ++f) x[f] = t[f] + dt * hk[f];
    }
    store_vec<NF>(a.h0, cf, i, acc);
  } else {
    load_vec<NF>(a.h0, cf, i, acc);
    exp_apply(p, exp_double(p, H, 0.5 * dt), u, t);
    double filt = 1.0;
    if (p.use_filter) filt = filter_value(g, p, k, l);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const cplx r = t[f] + (dt / 6) * (acc[f] + n[f]);
      x[f] = cx(r.re * filt, r.im * filt);
    }
    store_vec<NF>(a.sol_out, cf, i, x);
    note_state<NF>(a, x);
  }
}

// FF ETDRK4TimeStepper (ETDRK4substeps!/ETDRK4update!) for a real diagonal
// L shared by every field; coefficients per mode from the table a.etd
// (k_etd_coeffs).  One calcN result per stage:
//   1: N1 -> n1 = N1; acc = E u + α N1;           x = s1 = E2 u + ζ N1
//   2: N2 -> n2 = N2;                             x = s2 = E2 u + ζ N2
//   3: N3 -> acc = acc + 2β (n2 + N3);            x = s2 = E2 s1 + ζ (2 N3 - n1)
//   4: N4 -> u = acc + Γ N4
// acc accumulates FF's left-to-right sum E u + α N1 + 2β (N2 + N3) + Γ N4
// term by term, so the rounding sequence is FF's.
template <int NF>
__device__ __forceinline__ void op_etdrk4(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                          const cplx n[NF], cplx x[NF]) {
#pragma clang fp contract(off)
  const long long cf = g.cfield;
  const double* T = a.etd + i;
  if (a.stage == 1) {
    const double E = T[ETD_E * cf], E2 = T[ETD_E2 * cf], z = T[ETD_ZETA * cf], al = T[ETD_ALPHA * cf];
    cplx u[NF], acc[NF];
    load_vec<NF>(a.sol, cf, i, u);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      acc[f] = E * u[f] + al * n[f];
      x[f] = E2 * u[f] + z * n[f];
    }
    store_vec<NF>(a.n1, cf, i, n);
    store_vec<NF>(a.h0, cf, i, acc);
    store_vec<NF>(a.xs, cf, i, x);
  } else if (a.stage == 2) {
    const double E2 = T[ETD_E2 * cf], z = T[ETD_ZETA * cf];
    cplx u[NF];
    load_vec<NF>(a.sol, cf, i, u);
#pragma unroll
    for (int f = 0; f < NF; ++f) x[f] = E2 * u[f] + z * n[f];
    store_vec<NF>(a.n2, cf, i, n);
    store_vec<NF>(a.xs2, cf, i, x);
  } else if (a.stage == 3) {
    const double E2 = T[ETD_E2 * cf], z = T[ETD_ZETA * cf], b2 = 2.0 * T[ETD_BETA * cf];
    cplx s1[NF], acc[NF], N1[NF], N2[NF];
    load_vec<NF>(a.xs, cf, i, s1);
    load_vec<NF>(a.h0, cf, i, acc);
    load_vec<NF>(a.n1, cf, i, N1);
    load_vec<NF>(a.n2, cf, i, N2);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      acc[f] = acc[f] + b2 * (N2[f] + n[f]);
      x[f] = E2 * s1[f] + z * (2.0 * n[f] - N1[f]);
    }
    store_vec<NF>(a.h0, cf, i, acc);
    store_vec<NF>(a.xs2, cf, i, x);
  } else {
    const double G = T[ETD_GAMMA * cf];
    cplx acc[NF];
    load_vec<NF>(a.h0, cf, i, acc);
#pragma unroll
    for (int f = 0; f < NF; ++f) x[f] = acc[f] + G * n[f];
    store_vec<NF>(a.sol_out, cf, i, x);
    note_state<NF>(a, x);
  }
}

// FF FilteredRK4 (simulation/Parameters.jl:25; RK4substeps!/RK4update!):
// RHS_s = N(X_s) + L·X_s for the stage input X_s (a.sol at stage 1, a.xs
// after), then
//   1: acc = RHS/6;        x = sol + dt/2 RHS
//   2: acc = acc + RHS/3;  x = sol + dt/2 RHS
//   3: acc = acc + RHS/3;  x = sol + dt RHS
//   4: sol = (sol + dt (acc + RHS/6)) · filter
// acc follows FF's left-to-right sum RHS₁/6 + RHS₂/3 + RHS₃/3 + RHS₄/6.
template <int NF>
__device__ __forceinline__ void op_frk4(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                        double k, double l, const cplx n[NF], cplx x[NF]) {
#pragma clang fp contract(off)
  const long long cf = g.cfield;
  const double dt = p.dt;
  cplx L[NF][NF], X[NF], u[NF], rhs[NF], acc[NF];
  model_L<NF>(p, k, l, L);
  load_vec<NF>(a.stage == 1 ? a.sol : a.xs, cf, i, X);
  if (a.stage == 1) {
#pragma unroll
    for (int f = 0; f < NF; ++f) u[f] = X[f];
  } else {
    load_vec<NF>(a.sol, cf, i, u);
  }
  matvec<NF>(L, X, rhs);
#pragma unroll
  for (int f = 0; f < NF; ++f) rhs[f] = n[f] + rhs[f];
  if (a.stage > 1) load_vec<NF>(a.h0, cf, i, acc);
  if (a.stage < 4) {
    const double h = a.stage == 3 ? dt : dt / 2;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const cplx r = a.stage == 1 ? cx(rhs[f].re / 6, rhs[f].im / 6) : cx(rhs[f].re / 3, rhs[f].im / 3);
      acc[f] = a.stage == 1 ? r : acc[f] + r;
      x[f] = u[f] + h * rhs[f];
    }
    store_vec<NF>(a.h0, cf, i, acc);
    store_vec<NF>(a.xs, cf, i, x);
  } else {
    const double filt = filter_value(g, p, k, l);
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const cplx r = u[f] + dt * (acc[f] + cx(rhs[f].re / 6, rhs[f].im / 6));
      x[f] = cx(r.re * filt, r.im * filt);
    }
    store_vec<NF>(a.sol_out, cf, i, x);
    note_state<NF>(a, x);
  }
}

// a split N (k_col_fwd SPLIT: term 0 in N, terms 1-2 in a.nt1 / a.nt2, no
// linear terms) completed at mode i in k_col_fwd's order: the terms summed
// left to right, then MultiLayerQG's / Thomas–Yamada's linear terms from the
// calcN input a.xin
template <int NF>
__device__ __forceinline__ void assemble_terms(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                               double k, double l, cplx (&n)[NF]) {
  constexpr int MODEL = NF == 3 ? MODEL_RSW : (NF == 4 ? MODEL_TY : MODEL_QG2);
  const long long cf = g.cfield;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const NTerms nt = nterms<MODEL>(f);
    double2 r = make_double2(n[f].re, n[f].im);
    if (nt.fb >= 0) r = cadd(r, a.nt1[f * cf + i]);
    if (nt.fc >= 0) r = cadd(r, a.nt2[f * cf + i]);
    if constexpr (MODEL == MODEL_QG2)
      if (p.model == MODEL_MLQG) r = mlqg_linear_terms(p, k, l, a.xin[i], a.xin[cf + i], f, r);
    if constexpr (MODEL == MODEL_TY) r = ty_linear_terms(a.xin, cf, i, f, k, l, r);
    n[f] = cx(r.x, r.y);
  }
}

template <int NF, int OP, bool NT = false>
__device__ __forceinline__ void step_op(const Geom& g, const Phys& p, const StepPtrs& a, long long i,
                                        double k, double l, const cplx n[NF], cplx x[NF]) {
  if constexpr (OP == OP_FAB3) op_fab3<NF, NT>(g, p, a, i, k, l, n, x);
  else if constexpr (OP == OP_IFMAB3) op_ifmab3<NF, NT>(g, p, a, i, k, l, n, x);
  else if constexpr (OP == OP_ETDRK4) op_etdrk4<NF>(g, p, a, i, n, x);
  else if constexpr (OP == OP_FRK4) op_frk4<NF>(g, p, a, i, k, l, n, x);
  else op_rk4<NF>(g, p, a, i, k, l, n, x);
}

// FF getetdcoeffs(dt, L; ncirc = 32, rcirc = 1) per live mode for the real
// diagonal L = -ν K^(2nν) (thomasyamada/ThomasYamada.jl:265-277): the mean
// over 32 points z = dt L + e^{2πi (j + 1/2)/32} of the Cox–Matthews
// functions, times dt, real part; plus e^{dt L}, e^{dt L / 2}.
__device__ __forceinline__ cplx cexp_d(cplx z) {
  const double e = exp(z.re);
  return cplx{e * cos(z.im), e * sin(z.im)};
}
static __global__ void __launch_bounds__(256) k_etd_coeffs(Geom g, Phys p, double* __restrict__ etd) {
#pragma clang fp contract(off)
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.cfield) return;
  int kr, j;
  const long long cf = g.cfield;
  if (!mode_of(g, i, kr, j)) {
    for (int c = 0; c < ETD_N; ++c) etd[c * cf + i] = 0.0;
    return;
  }
  const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
  const double L = -(p.nu * ipow(k * k + l * l, p.nnu));
  const double dt = p.dt;
  const double zr = dt * L;
  cplx sz = cx(0.0), sa = cx(0.0), sb = cx(0.0), sg = cx(0.0);
  for (int m = 0; m < 32; ++m) {
    const double th = 2.0 * 3.14159265358979323846 / 32.0 * (m + 0.5);
    const cplx z = cx(zr + cos(th), sin(th));
    const cplx ez = cexp_d(z), ez2 = cexp_d(0.5 * z);
    const cplx z2 = z * z, z3 = z2 * z;
    sz = sz + cdiv(ez2 - cx(1.0), z);
    sa = sa + cdiv(cx(-4.0) - z + ez * (cx(4.0) - 3.0 * z + z2), z3);
    sb = sb + cdiv(cx(2.0) + z + ez * (cx(-2.0) + z), z3);
    sg = sg + cdiv(cx(-4.0) - 3.0 * z - z2 + ez * (cx(4.0) - z), z3);
  }
  etd[ETD_E * cf + i] = exp(dt * L);
  etd[ETD_E2 * cf + i] = exp(dt * L / 2);
  etd[ETD_ZETA * cf + i] = dt * (sz.re / 32.0);
  etd[ETD_ALPHA * cf + i] = dt * (sa.re / 32.0);
  etd[ETD_BETA * cf + i] = dt * (sb.re / 32.0);
  etd[ETD_GAMMA * cf + i] = dt * (sg.re / 32.0);
}

// Elementwise (unfused) stepper kernel: N from memory; the stage input x is
// written to xs (RK4 stages 1-3) for a separate col_inv.
template <int NF, int OP, bool NT>
static __global__ void __launch_bounds__(256) k_step_elem(Geom g, Phys p, StepPtrs a, const double2* __restrict__ N,
                            double2* __restrict__ xs) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
  cplx n[NF], x[NF];
  load_vec_once<NF, NT>(N, g.cfield, i, n);  // last use of this calcN output
  if (a.nt1) assemble_terms<NF>(g, p, a, i, k, l, n);
  if constexpr (OP == OP_IFMAB3) {
    // N already sits in the history slot op_ifmab3 stores it to (calcN wrote
    // it there: sw_api.cpp run_stage): only the new state is written — unless
    // it was completed here from split terms
    if (N == a.h0 && !a.nt1) {
      ifmab3_x<NF, NT>(g, p, a, i, k, l, n, x);
      store_vec<NF>(a.sol_out, g.cfield, i, x);
      note_state<NF>(a, x);
      return;
    }
  }
  step_op<NF, OP, NT>(g, p, a, i, k, l, n, x);
  if (OP == OP_RK4 && a.stage < 4) store_vec<NF>(a.xs, g.cfield, i, x);
}

// ===========================================================================
// col_step: the fused column pass of one stepper stage.  For column kr:
//   forward y-FFTs of the row outputs -> N (registers, never in HBM)
//   -> stepper op per live mode (state/history read and written once)
//   -> the next calcN's inverse y-FFTs straight from registers -> mixed space.
// Replaces col_fwd + update + col_inv of the next step.
// ===========================================================================
// keep the state/history loads of at most SW_SLOT_GROUP slots in flight
#ifndef SW_SLOT_GROUP
#define SW_SLOT_GROUP 2
#endif
#define SW_SLOT_FENCE(s) \
  if (((s) + 1) % SW_SLOT_GROUP == 0) __builtin_amdgcn_sched_barrier(0)

// INV = false: forward + update only (k_col_fwd + k_step_elem in one pass, N
// never in HBM); the next calcN's k_col_inv runs separately.  STREAM: the
// state/history cache policy of k_step_elem (StepPtrs::stream).
template <int MODEL, int LOG2N, int OP, bool INV = true, bool STREAM = false, int BAND = 0>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_col_step(Geom g, Phys p, StepPtrs a, const double2* __restrict__ Mf,
               double2* __restrict__ Minv, const double2* __restrict__ tw) {
  band_fix<LOG2N, BAND>(g);
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  constexpr int NF = MODEL == MODEL_RSW ? 3 : 2;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int krl = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
  const bool live = krl < g.kcn;
  if (B::NB == 1 && !live) return;
  const int krA = krl < g.kcl ? krl : g.kcl - 1;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  constexpr bool CD = col_dec<LOG2N, MODEL>();  // the family's stored-row order
  ColTw<LOG2N, CD> tws;
  tws.load(c.t, tw);
  const double k = (g.kr0 + krl) * g.mk;
  const long long MF = g.mfield;
  double2 v[8];

  auto load_col = [&](const double2* Mfield) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double2 t = mix_ld_col(Mfield + midc(g, krA, cpos<LOG2N, CD>(c.t, s)));
      v[s] = live ? t : zero2();
    }
  };

  // N_f (nterms): forward y-FFTs of row outputs with per-mode multipliers
  auto compute_N = [&](double2 (&n)[8], int f) {
    const NTerms nt = nterms<MODEL>(f);
    load_col(Mf + nt.fa * MF);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) n[s] = apply_mul(v[s], nt.ma, k, lwav(g, c.t + s * NT));
    if (nt.fb >= 0) {
      load_col(Mf + nt.fb * MF);
      col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) n[s] = cadd(n[s], apply_mul(v[s], nt.mb, k, lwav(g, c.t + s * NT)));
    }
  };

  if constexpr (OP == OP_FAB3) {
    // FilteredAB3 updates field f from N_f alone: no N array is kept
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      double2 n[8];
      compute_N(n, f);
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int m = c.t + s * NT;
        const int j = compact_of(g, m);
        if (live && j >= 0) {
          const long long i = (long long)krl * g.LrP + j;
          const cplx nf = cx(n[s].x, n[s].y);
          if (f == 0) op_fab3_field<NF, 0, STREAM>(g, p, a, i, k, lwav(g, m), nf);
          else if (f == 1) op_fab3_field<NF, 1, STREAM>(g, p, a, i, k, lwav(g, m), nf);
          else op_fab3_field<NF, (NF == 3 ? 2 : 1), STREAM>(g, p, a, i, k, lwav(g, m), nf);
        }
        SW_SLOT_FENCE(s);
      }
    }
  } else {
    double2 X[NF][8];
#pragma unroll
    for (int f = 0; f < NF; ++f) compute_N(X[f], f);
    // stepper op on the live modes of this column; it stores the next calcN
    // input (new state, or the RK4 stage input in xs), which the inverse phase
    // reads back (same thread, same addresses, L2-hot)
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int m = c.t + s * NT;
      const int j = compact_of(g, m);
      if (live && j >= 0) {
        cplx n[NF], x[NF];
        const long long i = (long long)krl * g.LrP + j;
        if constexpr (MODEL == MODEL_QG2 && OP == OP_FRK4) {
          if (p.model == MODEL_MLQG) {  // (k_col_fwd's terms, from this stage's calcN input)
            const double2* Xin = a.stage == 1 ? a.sol : a.xs;
            const double2 q1 = Xin[i], q2 = Xin[g.cfield + i];
#pragma unroll
            for (int f = 0; f < NF; ++f) X[f][s] = mlqg_linear_terms(p, k, lwav(g, m), q1, q2, f, X[f][s]);
          }
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) n[f] = cx(X[f][s].x, X[f][s].y);
        step_op<NF, OP, STREAM>(g, p, a, i, k, lwav(g, m), n, x);
        if (OP == OP_RK4 && a.stage < 4) store_vec<NF>(a.xs, g.cfield, i, x);
      }
      SW_SLOT_FENCE(s);
    }
  }
  if constexpr (!INV) return;
  const double2* Xs = (OP == OP_RK4 && a.stage < 4) ? a.xs : a.sol_out;
  const double2* Xc = Xs + (long long)(live ? krl : 0) * g.LrP;
  auto load_x = [&](int f, double2 (&x)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = compact_of(g, c.t + s * NT);
      const double2 t = Xc[f * g.cfield + (j >= 0 ? j : 0)];
      x[s] = (live && j >= 0) ? t : zero2();
    }
  };

  // ---- inverse for the next calcN (same outputs as k_col_inv)
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  auto store = [&](int o) {
    if (live) {
      double2* Mo = Minv + (long long)o * MF;
      store_col_p<LOG2N, CD>(g, krl, c.t, [&](int s, int o) { Mo[o] = v[s]; });
    }
  };
  if constexpr (MODEL == MODEL_RSW) {
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      double2 x[8];
      load_x(f, x);
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cscale(x[s], scale);
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(f);
      if (f == 0) {  // Uy
#pragma unroll
        for (int s = 0; s < 8; ++s) v[s] = cmul_i(x[s], lwav(g, c.t + s * NT) * scale);
        col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
        store(3);
      }
    }
  } else {
    double2 q1[8], q2[8];
    load_x(0, q1);
    load_x(1, q2);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cscale(f ? q2[s] : q1[s], scale);
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(f);
      double2 psi[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {  // streamfunctionfrompv! (swqg/TwoLayerQG.jl:101-111)
        const double l = lwav(g, c.t + s * NT);
        const double K2 = k * k + l * l;
        qg_psi(p, K2, q1[s].x, q1[s].y, q2[s].x, q2[s].y, f, psi[s].x, psi[s].y);
        v[s] = cscale(psi[s], scale);
      }
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(2 + f);
#pragma unroll
      for (int s = 0; s < 8; ++s) v[s] = cmul_i(psi[s], lwav(g, c.t + s * NT) * scale);
      col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
      store(4 + f);
    }
  }
}

// ===========================================================================
// col_fwd_step_lds: k_col_fwd + k_step_elem for the coupled updates with each
// field's N parked in LDS (live rows only, own slots: no barrier) as soon as
// its forward transforms are done, so that no N array is live in registers
// beside the per-mode update, which runs as a rolled loop over the slots.
// Dynamic LDS: NB * (FftPlan::LDS + NF * Lr) double2 (fwd_step_lds_bytes).
// ===========================================================================
#ifndef SW_FS_UNROLL
#define SW_FS_UNROLL 1  // slots per update-loop iteration (experiments)
#endif
#define SW_PRAGMA_(x) _Pragma(#x)
#define SW_PRAGMA(x) SW_PRAGMA_(x)
template <int MODEL, int LOG2N, int OP, bool STREAM>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_col_fwd_step_lds(Geom g, Phys p, StepPtrs a, const double2* __restrict__ Mf,
                       const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  constexpr int NF = MODEL == MODEL_RSW ? 3 : 2;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int krl = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
  const bool live = krl < g.kcn;
  if (B::NB == 1 && !live) return;
  const int krA = krl < g.kcl ? krl : g.kcl - 1;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  double2* park = smem + B::NB * FftPlan<LOG2N>::LDS + (long long)c.ln * NF * g.Lr;
  constexpr bool CD = col_dec<LOG2N, MODEL>();  // the family's stored-row order
  ColTw<LOG2N, CD> tws;
  tws.load(c.t, tw);
  const double k = (g.kr0 + krl) * g.mk;
  const long long MF = g.mfield;
  double2 v[8], n[8];
  auto load_col = [&](const double2* Mfield) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double2 t = mix_ld_col(Mfield + midc(g, krA, cpos<LOG2N, CD>(c.t, s)));
      v[s] = live ? t : zero2();
    }
  };
  // N_f (nterms), the same arithmetic as k_col_fwd
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const NTerms nt = nterms<MODEL>(f);
    load_col(Mf + nt.fa * MF);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) n[s] = apply_mul(v[s], nt.ma, k, lwav(g, c.t + s * NT));
    if (nt.fb >= 0) {
      load_col(Mf + nt.fb * MF);
      col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
      for (int s = 0; s < 8; ++s) n[s] = cadd(n[s], apply_mul(v[s], nt.mb, k, lwav(g, c.t + s * NT)));
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int j = compact_of(g, c.t + s * NT);
      if (j >= 0) park[f * g.Lr + j] = n[s];
    }
  }
  if (!live) return;
  SW_PRAGMA(unroll SW_FS_UNROLL)
  for (int s = 0; s < 8; ++s) {
    const int m = c.t + s * NT;
    const int j = compact_of(g, m);
    if (j >= 0) {
      cplx nn[NF], x[NF];
      const long long i = (long long)krl * g.LrP + j;
      double2 q1 = zero2(), q2 = zero2();
      if constexpr (MODEL == MODEL_QG2 && OP == OP_FRK4) {
        if (p.model == MODEL_MLQG) {
          const double2* Xin = a.stage == 1 ? a.sol : a.xs;
          q1 = Xin[i];
          q2 = Xin[g.cfield + i];
        }
      }
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        double2 t = park[f * g.Lr + j];
        if constexpr (MODEL == MODEL_QG2 && OP == OP_FRK4)
          if (p.model == MODEL_MLQG) t = mlqg_linear_terms(p, k, lwav(g, m), q1, q2, f, t);
        nn[f] = cx(t.x, t.y);
      }
      step_op<NF, OP, STREAM>(g, p, a, i, k, lwav(g, m), nn, x);
      if (OP == OP_RK4 && a.stage < 4) store_vec<NF>(a.xs, g.cfield, i, x);
    }
  }
}

// ===========================================================================
// col_step_fab3 (RSW FilteredAB3): one block per (column, field f).  The
// FilteredAB3 update of field f needs N_f alone (plus the old state for L·sol),
// and the next calcN's inverse transforms of field f need only the new field f:
//   f=0: N_u = F(P)                   -> u -> U, Uy
//   f=1: N_v = -il F(K̂) - F((ζu)^)    -> v -> V
//   f=2: N_η = F(Q) - il F((vη)^)     -> η -> H
// three y-FFTs per block, N never in HBM, old/new state in separate buffers.
// ===========================================================================
#ifndef SW_CS_GROUP
#define SW_CS_GROUP 2  // slots per load group of the fused FilteredAB3 update
#endif
// 3 waves/SIMD (<= 168 VGPRs) where 256-thread blocks hold the line: the
// kernel lands at 160-170 VGPRs and 2 against 3 waves costs ~6 % (87.5 vs 93 µs
// at 2048²), so the register budget is pinned rather than left to chance
#ifndef SW_MINW_CS
#define SW_MINW_CS 2
#endif
template <int LOG2N, bool STREAM, int BAND = 0>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, (Blk<LOG2N>::THREADS >= 512 ? 4 : SW_MINW_CS))
    k_col_step_fab3_rsw(Geom g, Phys p, StepPtrs a, const double2* __restrict__ Mf,
                        double2* __restrict__ Minv, const double2* __restrict__ tw, int fbase) {
  band_fix<LOG2N, BAND>(g);
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  int krl, f;
  if (fbase < 0) {
    // all fields, 1-D grid of 3*kcl blocks (NB == 1, kcl a multiple of 64).  The 3 fields of the 8
    // columns that share each 128-B chunk of the mixed layout (24 blocks) sit
    // on one XCD label (b % 8) within 192 consecutive block ids: they meet in
    // one L2, where the other fields' reads of the old state and the chunk
    // writes coalesce (speed only; any placement is correct).
    const int b = blockIdx.x, q = b / 192, r = b - q * 192, x = r & 7, jj = r >> 3;
    f = jj % 3;
    krl = q * 64 + x * 8 + jj / 3;
  } else {
    krl = blockIdx.x * B::NB + c.ln;
    f = fbase + blockIdx.y;
  }
  const bool live = krl < g.kcn;
  if (B::NB == 1 && !live) return;
  const int krA = krl < g.kcl ? krl : g.kcl - 1;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  constexpr bool CD = col_dec<LOG2N, MODEL_RSW>();  // the family's stored-row order
  ColTw<LOG2N, CD> tws;
  tws.load(c.t, tw);
  const double k = (g.kr0 + krl) * g.mk;
  const long long MF = g.mfield;
  double2 v[8], n[8];

  auto load_col = [&](double2 (&dst)[8], const double2* Mfield) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#ifdef SW_EXP_CS_NOMIX  // experiment: mixed-field loads from one line (wrong results)
      const double2 t = Mfield[c.t & 7];
#else
      const double2 t = mix_ld_col(Mfield + midc(g, krA, cpos<LOG2N, CD>(c.t, s)));
#endif
      dst[s] = live ? t : zero2();
    }
  };
  const NTerms nt = nterms<MODEL_RSW>(f);
  // ---- N_f (rsw/RotatingShallowWater.jl:174-226; nterms)
  load_col(v, Mf + nt.fa * MF);
  col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
  for (int s = 0; s < 8; ++s) n[s] = apply_mul(v[s], nt.ma, k, lwav(g, c.t + s * NT));
  if (nt.fb >= 0) {
    load_col(v, Mf + nt.fb * MF);
    col_fft<LOG2N, -1, CD>(v, c.t, tws, line);
#pragma unroll
    for (int s = 0; s < 8; ++s) n[s] = cadd(n[s], apply_mul(v[s], nt.mb, k, lwav(g, c.t + s * NT)));
  }
  // ---- FilteredAB3 update of field f on the live modes; x = new field f.
  // Slots in groups of SW_CS_GROUP: all loads of a group are issued before
  // the first is used (in-bounds clamped addresses, branch-free arithmetic;
  // dead modes are computed and dropped), one memory round trip per group
  // instead of two per slot.
  double2 x[8];
  bool bad = false;  // (note_nonfinite)
  {
    const long long cf = g.cfield;
    // compact fields hold the kcn live columns only: padding lines of a
    // multi-line block (krl in [kcn, kcl)) read column 0 and store nothing
    const long long cb = (long long)(live ? krl : 0) * g.LrP;
    const double2* S = a.sol + cb;
    const double2* H1 = a.h1 + f * cf + cb;
    const double2* H2 = a.h2 + f * cf + cb;
    // slots in the order 0 1 2 5 6 7 3 4: under the 2/3 rule the slots 3, 4
    // (m in [3N/8, 5N/8)) are dead on every thread, and a group of them is
    // skipped (uniform branch)
    constexpr int G = SW_CS_GROUP;
    constexpr int ord[8] = {0, 1, 2, 5, 6, 7, 3, 4};
    auto slot_live = [&](int s) { return s * NT < g.lc || (s + 1) * NT > g.lr2; };
#pragma unroll
    for (int s0 = 0; s0 < 8; s0 += G) {
      bool any = false;
#pragma unroll
      for (int q = 0; q < G; ++q) any = any || slot_live(ord[s0 + q]);
      if (!any) {
#pragma unroll
        for (int q = 0; q < G; ++q) x[ord[s0 + q]] = zero2();
        continue;
      }
      cplx st[G][3];
      double2 r1[G], r2[G];
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int j = compact_of(g, c.t + ord[s0 + q] * NT);
        const int jc = j >= 0 ? j : 0;
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
#ifdef SW_SOL_NT
          const double2 t = state_ld<STREAM>(S + cc * cf + jc);
#else
          // temporal: the three field blocks of a column read it (one L2)
          const double2 t = S[cc * cf + jc];
#endif
          st[q][cc] = cx(t.x, t.y);
        }
        r1[q] = state_ld<STREAM>(H1 + jc);
        r2[q] = state_ld<STREAM>(H2 + jc);
      }
#pragma unroll
      for (int q = 0; q < G; ++q) {
        const int s = ord[s0 + q];
        const int m = c.t + s * NT;
        const int j = compact_of(g, m);
        const double l = lwav(g, m);
        const cplx nf = cx(n[s].x, n[s].y);
        cplx r, rhs;
        if (f == 0) fab3_compute<3, 0>(g, p, a.euler, k, l, nf, st[q], r1[q], r2[q], r, rhs);
        else if (f == 1) fab3_compute<3, 1>(g, p, a.euler, k, l, nf, st[q], r1[q], r2[q], r, rhs);
        else fab3_compute<3, 2>(g, p, a.euler, k, l, nf, st[q], r1[q], r2[q], r, rhs);
#ifdef SW_EXP_CS_NOUPD  // experiment: no stepper update (no state traffic; wrong results)
        r = nf;
#endif
        const bool ok = live && j >= 0;
        x[s] = ok ? make_double2(r.re, r.im) : zero2();
        if (ok) {
          const long long i = cb + j;
          state_st<STREAM>(a.h0 + f * cf + i, make_double2(rhs.re, rhs.im));
          state_st<STREAM>(a.sol_out + f * cf + i, make_double2(r.re, r.im));
        }
        bad |= ok & nonfinite(r);
      }
    }
  }
  note_nonfinite(a.nan, bad);
  // ---- inverse transforms of field f for the next calcN (as k_col_inv)
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  auto store = [&](int o) {
    if (live) {
      double2* Mo = Minv + (long long)o * MF;
      store_col_p<LOG2N, CD>(g, krl, c.t, [&](int s, int o) { Mo[o] = v[s]; });
    }
  };
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = cscale(x[s], scale);
  col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
  store(f);
  if (f == 0) {  // ∂y u: Uy
#pragma unroll
    for (int s = 0; s < 8; ++s) v[s] = cmul_i(x[s], lwav(g, c.t + s * NT) * scale);
    col_fft<LOG2N, +1, CD>(v, c.t, tws, line);
    store(3);
  }
}

// ===========================================================================
// state I/O: Julia column-major (nkr, nl, nf) <-> compact live columns
// ===========================================================================
// this slab's live columns [kr0, kr0 + kcn) of the full array
static __global__ void k_gather(Geom g, int nf, const double2* __restrict__ full, double2* __restrict__ cmp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)g.kcn * g.Lr;
  if (i >= per * nf) return;
  const int f = (int)(i / per);
  const long long r = i - f * per;
  const int j = (int)(r / g.kcn), krl = (int)(r - (long long)j * g.kcn);
  const int m = lrow_of(g, j);
  cmp[f * g.cfield + (long long)krl * g.LrP + j] = full[((long long)f * g.nl + m) * g.nkr + g.kr0 + krl];
}

// columns [lo, hi) of the full array from this slab (zero outside live modes)
static __global__ void k_scatter(Geom g, int nf, int lo, int hi, const double2* __restrict__ cmp,
                          double2* __restrict__ full) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int w = hi - lo;
  const long long per = (long long)w * g.nl;
  if (i >= per * nf) return;
  const int f = (int)(i / per);
  const long long r = i - f * per;
  const int m = (int)(r / w), kr = lo + (int)(r - (long long)m * w);
  const int j = compact_of(g, m), krl = kr - g.kr0;
  double2 v = zero2();
  if (krl >= 0 && krl < g.kcn && j >= 0) v = cmp[f * g.cfield + (long long)krl * g.LrP + j];
  full[((long long)f * g.nl + m) * g.nkr + kr] = v;
}

// the compact modes of ga only (aliased regions; the other modes untouched)
static __global__ void k_scatter_modes(Geom ga, int nf, const double2* __restrict__ cmp, double2* __restrict__ full) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= ga.cfield || !mode_of(ga, i, kr, j)) return;
  const int m = lrow_of(ga, j);
  for (int f = 0; f < nf; ++f) full[((long long)f * ga.nl + m) * ga.nkr + kr] = cmp[f * ga.cfield + i];
}
static __global__ void k_gather_modes(Geom ga, int nf, const double2* __restrict__ full, double2* __restrict__ cmp) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= ga.cfield || !mode_of(ga, i, kr, j)) return;
  const int m = lrow_of(ga, j);
  for (int f = 0; f < nf; ++f) cmp[f * ga.cfield + i] = full[((long long)f * ga.nl + m) * ga.nkr + kr];
}

static __global__ void k_nan_check(Geom g, int nf, const double2* __restrict__ cmp, int* flag) {
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
static __global__ void k_make_spec(Geom g, Phys p, int model, int fid, const double2* __restrict__ sol,
                            double2* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  const long long cf = g.cfield;
  const double k = kr * g.mk, l = lwav(g, lrow_of(g, j));
  double2 r = zero2();
  if (model == MODEL_TY) {
    // thomasyamada/ThomasYamada.jl:67-92: 0 uc, 1 vc, 2 pc, 3 ζt, 4 qc =
    // ik vc - il uc - pc, 5 ψt = -ζt/K², 8 ut = -il ψt, 9 vt = ik ψt
    const double K2 = k * k + l * l;
    const double iK2 = K2 == 0.0 ? 0.0 : 1.0 / K2;
    const double2 z = sol[i];
    const double2 ps = make_double2(-z.x * iK2, -z.y * iK2);
    if (fid <= 2) r = sol[(fid + 1) * cf + i];
    else if (fid == 3) r = z;
    else if (fid == 4) r = csub(csub(cmul_i(sol[2 * cf + i], k), cmul_i(sol[cf + i], l)), sol[3 * cf + i]);
    else if (fid == 5) r = ps;
    else if (fid == 8) r = cmul_i(ps, -l);
    else if (fid == 9) r = cmul_i(ps, k);
  } else if (model == MODEL_RSW) {
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
      double2 ps;
      qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, layer, ps.x, ps.y);
      if (id == 5) r = ps;
      else if (id == 3) r = make_double2(-K2 * ps.x, -K2 * ps.y);
      else if (id == 0) r = cmul_i(ps, -l);
      else if (id == 1) r = cmul_i(ps, k);
    }
  }
  out[i] = r;
}

template <int LOG2N>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_col_inv1(Geom g, const double2* __restrict__ X, double2* __restrict__ M,
               const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int krl = blockIdx.x * B::NB + c.ln;
  const bool live = krl < g.kcn;
  if (B::NB == 1 && !live) return;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  const double scale = 1.0 / ((double)g.nx * (double)g.ny);
  const double2* Xf = X + (long long)(live ? krl : 0) * g.LrP;
  double2 v[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int j = compact_of(g, c.t + s * NT);
    const double2 t = Xf[j >= 0 ? j : 0];
    v[s] = (live && j >= 0) ? cscale(t, scale) : zero2();
  }
  fft_line<LOG2N, +1>(v, c.t, tws, line);
  if (live) {
    store_col_i<NT>(g, krl, c.t, [&](int s, int o) { M[o] = v[s]; });
  }
}

template <int LOG2N>
static __global__ void __launch_bounds__(Blk<LOG2N>::THREADS, SW_MINW(LOG2N))
    k_row_c2r1(Geom g, const double2* __restrict__ M, double* __restrict__ out,
               const double2* __restrict__ tw) {
  using B = Blk<LOG2N>;
  constexpr int NT = B::NT;
  extern __shared__ double2 smem[];
  const LineCtx c = line_ctx<LOG2N>();
  const int y = (B::NB == 1) ? col_of_block(blockIdx.x, gridDim.x) : blockIdx.x * B::NB + c.ln;
  double2* line = smem + c.ln * FftPlan<LOG2N>::LDS;
  Twiddles<LOG2N> tws;
  tws.load(c.t, tw);
  double2 v[8];
  RowIdx<LOG2N> ri;
  ri.init(g, c.t, y);
  load_pair<LOG2N>(v, ri, g, M, nullptr, false);
  fft_line<LOG2N, +1>(v, c.t, tws, line);
#pragma unroll
  for (int s = 0; s < 8; ++s) out[(long long)(g.y0 + y) * g.nx + c.t + s * NT] = v[s].x;
}

// Energies by Parseval over live modes (FF parsevalsum2 / parsevalsum:
// weight 2 for 0 < kr < nx/2, 1 for kr = 0).  SW_NSUM sums per state:
//   RSW: 0 |u|²+|v|², 1 |η|², 2.. unused
//   QG2/MLQG: 0 K²|ψ1|², 1 K²|ψ2|², 2 |ψ1-ψ2|², 3.. unused
//   TY: 0 |K⁻¹ζ|², 1 |u_c|²+|v_c|², 2 |p_c|², then the wave/balanced split
//       (ty_split): 3 |W_u|²+|W_v|², 4 |W_p|², 5 |G_u|²+|G_v|², 6 |G_p|²
// Deterministic and independent of the slab decomposition: one block per
// column reduces that column in a fixed order (k_energy_cols, padding
// columns give 0), then the column sums are added in global column order
// (k_energy_final).  No atomics: results repeat bitwise for any P.
// thomasyamada/TYUtils.jl:10-51 (decompose_balanced_wave) at one mode (k, l):
// G = (b·Φ₀*)Φ₀, W = (b·Φ₊*)Φ₊ + (b·Φ₋*)Φ₋ of b = (u_c, v_c, p_c), with
// ω = √(1+K²), Φ₀ = (il, −ik, −1)/ω, Φ± = (±ωk + il, ±ωl − ik, ω²−1)·s,
// s = √(1/(2K²))/ω; at K = 0, Φ₀ = (0, 0, 1) and Φ± = (i, ±1, 0)/√2.
// Adds w·(|W_u|²+|W_v|², |W_p|², |G_u|²+|G_v|², |G_p|²) to a[0..3].
__device__ __forceinline__ double2 cdotc(double2 u, double2 v, double2 q, double2 P0, double2 P1, double2 P2) {
  return cadd(cadd(cmul(u, cconj(P0)), cmul(v, cconj(P1))), cmul(q, cconj(P2)));
}
__device__ void ty_split(double k, double l, double2 u, double2 v, double2 q, double w, double* a) {
  double2 Z[3], Pp[3], Pm[3];
  const double K2 = k * k + l * l;
  if (K2 == 0.0) {
    const double r = sqrt(0.5);
    Z[0] = make_double2(0.0, 0.0), Z[1] = make_double2(0.0, 0.0), Z[2] = make_double2(1.0, 0.0);
    Pp[0] = make_double2(0.0, r), Pp[1] = make_double2(r, 0.0), Pp[2] = make_double2(0.0, 0.0);
    Pm[0] = make_double2(0.0, r), Pm[1] = make_double2(-r, 0.0), Pm[2] = make_double2(0.0, 0.0);
  } else {
    const double om = sqrt(1.0 + K2), io = 1.0 / om;
    const double sc = sqrt(1.0 / K2 / 2.0) / om;
    Z[0] = make_double2(0.0, l * io), Z[1] = make_double2(0.0, -k * io), Z[2] = make_double2(-io, 0.0);
    Pp[0] = make_double2(om * k * sc, l * sc), Pp[1] = make_double2(om * l * sc, -k * sc);
    Pm[0] = make_double2(-om * k * sc, l * sc), Pm[1] = make_double2(-om * l * sc, -k * sc);
    Pp[2] = Pm[2] = make_double2((om * om - 1.0) * sc, 0.0);
  }
  const double2 c0 = cdotc(u, v, q, Z[0], Z[1], Z[2]);
  const double2 cp = cdotc(u, v, q, Pp[0], Pp[1], Pp[2]);
  const double2 cm = cdotc(u, v, q, Pm[0], Pm[1], Pm[2]);
  double2 W[3], G[3];
  for (int j = 0; j < 3; ++j) {
    W[j] = cadd(cmul(cp, Pp[j]), cmul(cm, Pm[j]));
    G[j] = cmul(c0, Z[j]);
  }
  auto n2 = [](double2 z) { return z.x * z.x + z.y * z.y; };
  a[0] += w * (n2(W[0]) + n2(W[1]));
  a[1] += w * n2(W[2]);
  a[2] += w * (n2(G[0]) + n2(G[1]));
  a[3] += w * n2(G[2]);
}

__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += sh[i];
  return r;
}

static __global__ void __launch_bounds__(256) k_energy_cols(Geom g, Phys p, int model,
                                                     const double2* __restrict__ sol,
                                                     double* __restrict__ cols) {
  __shared__ double sh[4];
  const int krl = blockIdx.x;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, ws[4] = {0.0, 0.0, 0.0, 0.0};
  if (krl < g.kcn) {
    const long long cf = g.cfield;
    const int kr = g.kr0 + krl;
    const double w = (kr == 0 || 2 * kr == g.nx) ? 1.0 : 2.0, k = kr * g.mk;  // FF parsevalsum
    for (int j = threadIdx.x; j < g.Lr; j += blockDim.x) {
      const long long i = (long long)krl * g.LrP + j;
      if (model == MODEL_RSW) {
        const double2 u = sol[i], v = sol[cf + i], e = sol[2 * cf + i];
        a0 += w * (u.x * u.x + u.y * u.y + v.x * v.x + v.y * v.y);
        a1 += w * (e.x * e.x + e.y * e.y);
      } else if (model == MODEL_TY) {
        // barotropic |K⁻¹ ζ|², baroclinic |uc|² + |vc|², |pc|²
        const double l = lwav(g, lrow_of(g, j));
        const double K2 = k * k + l * l;
        const double r = sqrt(K2 == 0.0 ? 0.0 : 1.0 / K2);
        const double2 z = sol[i], u = sol[cf + i], v = sol[2 * cf + i], q = sol[3 * cf + i];
        const double zx = r * z.x, zy = r * z.y;
        a0 += w * (zx * zx + zy * zy);
        a1 += w * (u.x * u.x + u.y * u.y + v.x * v.x + v.y * v.y);
        a2 += w * (q.x * q.x + q.y * q.y);
        ty_split(k, l, u, v, q, w, ws);
      } else {
        const double l = lwav(g, lrow_of(g, j));
        const double K2 = k * k + l * l;
        const double2 q1 = sol[i], q2 = sol[cf + i];
        double2 p1, p2;
        qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, 0, p1.x, p1.y);
        qg_psi(p, K2, q1.x, q1.y, q2.x, q2.y, 1, p2.x, p2.y);
        a0 += w * K2 * (p1.x * p1.x + p1.y * p1.y);
        a1 += w * K2 * (p2.x * p2.x + p2.y * p2.y);
        const double dx_ = p1.x - p2.x, dy_ = p1.y - p2.y;
        a2 += w * (dx_ * dx_ + dy_ * dy_);
      }
    }
  }
  a0 = block_sum(a0, sh);
  a1 = block_sum(a1, sh);
  a2 = block_sum(a2, sh);
  if (model == MODEL_TY)
    for (int i = 0; i < 4; ++i) ws[i] = block_sum(ws[i], sh);
  if (threadIdx.x == 0) {
    double* o = cols + SW_NSUM * krl;
    o[0] = a0, o[1] = a1, o[2] = a2;
    for (int i = 0; i < 4; ++i) o[3 + i] = ws[i];
  }
}

static __global__ void k_energy_final(const double* __restrict__ cols, int ncols, double* __restrict__ out) {
  if (threadIdx.x < SW_NSUM) {
    double r = 0.0;
    for (int b = 0; b < ncols; ++b) r += cols[SW_NSUM * b + threadIdx.x];
    out[threadIdx.x] = r;
  }
}

// max |f| (sgn = 0) or max f (sgn = 1) over this slab's physical rows, as an
// order-preserving integer key (dkey) so that an integer atomicMax is exact
// and order-free; the host decodes it (key_double in sw_api.cpp)
__device__ __forceinline__ unsigned long long dkey(double d) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
static __global__ void k_absmax(const double* __restrict__ f, long long n, unsigned long long* out, int sgn) {
  double m = sgn ? -INFINITY : 0.0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    m = fmax(m, sgn ? f[i] : fabs(f[i]));
  for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_down(m, off, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, dkey(m));
}

// ===========================================================================
// launchers
// ===========================================================================
// host-side: dispatch the LOG2N instantiation (N = 32 … 8192)
#ifdef SW_ONLY_LOG2  // register/spill experiments: instantiate one length only
#define SW_LOG2_CASES(X) X(SW_ONLY_LOG2)
#else
#define SW_LOG2_CASES(X) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13)
#endif

// Split build (juliaraytracingsw_amd/build.py): the length-templated kernels
// of one transform length per translation unit (-DSW_PART=L, L = 5 … 13), the
// rest and the dispatch in SW_PART=0; without SW_PART one TU holds all.
#if !defined(SW_PART) || SW_PART > 0
// the column kernels' band (band_fix): 1 the 2/3 rule, 2 aliased_fraction = 0
template <int L>
static int band_of(const Geom& g) {
  constexpr int N = 1 << L;
  if (!SW_COL_BAND) return 0;
  if (g.lc == N / 3 && g.lr2 == N - N / 3) return 1;
  if (g.lc == N / 2 && g.lr2 == N / 2 + 1) return 2;
  return 0;
}
// SW_LAUNCH of a kernel template expression naming SWB, the band, for the
// band BV (one instantiation per band)
#define SW_LAUNCH_BAND(BV, KEXPR, ...)                     \
  do {                                                     \
    if ((BV) == 1) {                                       \
      constexpr int SWB = 1;                               \
      SW_LAUNCH(KEXPR, __VA_ARGS__);                       \
    } else if ((BV) == 2) {                                \
      constexpr int SWB = 2;                               \
      SW_LAUNCH(KEXPR, __VA_ARGS__);                       \
    } else {                                               \
      constexpr int SWB = 0;                               \
      SW_LAUNCH(KEXPR, __VA_ARGS__);                       \
    }                                                      \
  } while (0)

template <int L>
static int col_blocks(const Geom& g) {
  return (g.kcl + Blk<L>::NB - 1) / Blk<L>::NB;
}
template <int L>
static int row_blocks(const Geom& g) {
  return g.nyl / Blk<L>::NB;
}
template <int L>
static size_t lds_bytes() {
  return (size_t)Blk<L>::NB * FftPlan<L>::LDS * sizeof(double2);
}

// 2LQG col_inv with the two layer blocks of a column paired on one XCD
// (k_col_inv, gbase < 0), measured (tools/ab/qg_inv_pair_ab.sh): 8192-point
// columns 949.7 -> 881.3 µs (config 5 61.2 -> 61.9 steps/s); 2048-point
// columns 47-48 -> 48-50 µs (not used there).  1: on 8192-point lines,
// 2: every length, 0: never (experiments).
#ifndef SW_QG_INV_PAIR
#define SW_QG_INV_PAIR 1
#endif
template <int L>
void LenOps<L>::col_inv(int model, const Geom& g, const Phys& p, const double2* X, double2* M, const double2* tw,
                        hipStream_t s, int g0, int ng) {
  const int bnd = band_of<L>(g);
  const dim3 grid(col_blocks<L>(g), ng);
  const dim3 grid2(col_blocks<L>(g), 2 * ng);
  if (model == MODEL_RSW && g.isplit)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_RSW, L, true, SWB>), grid2, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M,
                       tw, g0);
  else if (model == MODEL_RSW)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_RSW, L, false, SWB>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M, tw, g0);
  else if (model == MODEL_RSWA && g.isplit)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_RSWA, L, true, SWB>), grid2, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M,
                       tw, g0);
  else if (model == MODEL_RSWA)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_RSWA, L, false, SWB>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M, tw, g0);
  else if (model == MODEL_TY && g.isplit)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_TY, L, true, SWB>), dim3(col_blocks<L>(g), 2 * ng), dim3(Blk<L>::THREADS),
                       lds_bytes<L>(), s, g, p, X, M, tw, g0);
  else if (model == MODEL_TY)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_TY, L, false, SWB>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M, tw, g0);
  else if (g0 == 0 && ng == 2 && Blk<L>::NB == 1 && g.kcl % 64 == 0 &&
           (SW_QG_INV_PAIR == 2 || (SW_QG_INV_PAIR == 1 && L >= 13)))
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_QG2, L, false, SWB>), dim3(2 * g.kcl), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X,
                       M, tw, -1);
  else if (g.isplit)
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_QG2, L, true, SWB>), dim3(col_blocks<L>(g), 3 * ng), dim3(Blk<L>::THREADS),
                       lds_bytes<L>(), s, g, p, X, M, tw, g0);
  else
    SW_LAUNCH_BAND(bnd, (k_col_inv<MODEL_QG2, L, false, SWB>), grid, dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, p, X, M, tw, g0);
}

// ===========================================================================
// row_rsw_sp: the decimated RSW row (1024-4096-point lines)
// over two blocks per row with ONE line buffer each and the transforms one
// after the other.  Part 0 forms ζu + iζv and K (outputs 0-2), part 1 uη + ivη
// (outputs 3-4); each transforms u + iv and the half of η + iζ it needs (part
// 0 reads no H, part 1 no Uy).  7 line transforms per row instead of 5, for a
// quarter of the LDS per block (32 KB at 2048) and half the live lines: up to
// SW_MINW_ROW_SP waves per SIMD instead of 2.  The same arithmetic on the
// same pairs as k_row: bitwise the same outputs.  1-D grid of 2 × rows: the
// two parts of 8 consecutive rows on one XCD label (the rows of a 2×4 tile
// meet in one L2).  SW_ROW_SP=1 selects it (sw_api.cpp, Geom::rsp).
// ===========================================================================
#ifndef SW_MINW_ROW_SP
#define SW_MINW_ROW_SP 4
#endif
#ifndef SW_ROW_SP_LEAN
#define SW_ROW_SP_LEAN false  // true: offsets per use (RowIdx LEAN)
#endif
#ifndef SW_ROW_SP_FLY
#define SW_ROW_SP_FLY false  // true: the wave-local stage twiddles read per stage
#endif
__device__ __forceinline__ void row_part_of_block(int b, int nb, int& y, int& part) {
  if ((nb & 127) == 0) {
    const int q = b >> 7, j = (b >> 3) & 15, x = b & 7;
    y = (q << 6) + (x << 3) + (j >> 1);
    part = j & 1;
  } else {
    y = b >> 1;
    part = b & 1;
  }
}
template <int LOG2N, bool PRUNE>
static __global__ void __launch_bounds__((BlkRow<MODEL_RSW, LOG2N>::THREADS), SW_MINW_ROW_SP)
    k_row_rsw_sp(Geom g, Phys p, const double2* __restrict__ Mi, double2* __restrict__ Mo,
                 const double2* __restrict__ tw, int yoff) {
  using Bk = BlkRow<MODEL_RSW, LOG2N>;
  static_assert(Bk::NB == 1 && roww<LOG2N>() > 0, "one decimated row per block");
  constexpr int W = roww<LOG2N>();
  extern __shared__ double2 smem[];
  double2* line = smem;
  const LineCtx c = line_ctx<LOG2N>();
  int yl, part;
  row_part_of_block(blockIdx.x, gridDim.x, yl, part);
  const int y = yoff + yl;
  RowIdx<LOG2N, SW_ROW_SP_LEAN> ri;
  ri.init(g, c.t, y);
  Twiddles<9, SW_ROW_SP_FLY> tq;
  tq.load(c.t & 63, tw, LOG2N - 9);
  const double2 wt = tw[c.t];
  const long long MF = g.mfield;
  const double2 *U = Mi, *V = Mi + MF, *H = Mi + 2 * MF, *Uy = Mi + 3 * MF;
  using R = RowIdx<LOG2N, SW_ROW_SP_LEAN>;
  double2 w[2][8];
  {  // u + i v, and η (part 1) or i ζ (part 0): one read of each field a part needs
    double2 u[8], vv[8], x[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      u[s] = vv[s] = x[s] = zero2();
      if (R::inv_any(g, s)) {
        const int o = ri.oinv(g, s);
        u[s] = mix_ld_row(U + o);
        vv[s] = mix_ld_row(V + o);
        x[s] = mix_ld_row((part ? H : Uy) + o);
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int kk = R::kk(ri.t, s);
      const bool mir = s >= 4 && kk != (R::N >> 1), live = kk < g.kc;
      w[0][s] = pair_z(u[s], vv[s], kk, mir, live);
      w[1][s] = part ? pair_z(x[s], zero2(), kk, mir, live)
                     : pair_z(zero2(), csub(cmul_i(vv[s], kk * g.mk), x[s]), kk, mir, live);
    }
  }
  fftw_dif<W, +1, 1, false, SW_ROW_SP_FLY, false, PRUNE>(reinterpret_cast<double2(&)[1][8]>(w[0]), c.t, wt, tq, line, 0);
  fftw_dif<W, +1, 1, true, SW_ROW_SP_FLY, false, PRUNE>(reinterpret_cast<double2(&)[1][8]>(w[1]), c.t, wt, tq, line, 0);
  if (part) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const double u = w[0][s].x, vv = w[0][s].y, eta = w[1][s].x;
      w[0][s] = make_double2(u * eta, vv * eta);  // uη + i vη
    }
    fftw_dit<W, -1, 1, SW_ROW_SP_FLY, true, false, PRUNE>(reinterpret_cast<double2(&)[1][8]>(w[0]), c.t, wt, tq, line, 0);
    split_pairs<LOG2N, 1, PRUNE>(reinterpret_cast<const double2(&)[1][8]>(w[0]), c.t, g, line, 0,
                                 [&](int, int k, int s, double2 a, double2 b) {
                                   const int o = ri.ofwd(g, s);
                                   Mo[3 * MF + o] = cmul_i(a, -(k * g.mk));
                                   Mo[4 * MF + o] = b;
                                 });
    return;
  }
  double kk[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const double u = w[0][s].x, vv = w[0][s].y, zeta = w[1][s].y;
    kk[s] = 0.5 * (u * u + vv * vv);
    w[0][s] = make_double2(zeta * u, zeta * vv);  // ζu + i ζv
  }
  fftw_dit<W, -1, 1, SW_ROW_SP_FLY, true, false, PRUNE>(reinterpret_cast<double2(&)[1][8]>(w[0]), c.t, wt, tq, line, 0);
  double2 zv[8];  // (ζv)^ of the live slots
#pragma unroll
  for (int s = 0; s < 8; ++s) zv[s] = zero2();
  split_pairs<LOG2N, 1, PRUNE>(reinterpret_cast<const double2(&)[1][8]>(w[0]), c.t, g, line, 0,
                               [&](int, int, int s, double2 a, double2 b) {
                                 Mo[2 * MF + ri.ofwd(g, s)] = a;
                                 zv[s] = b;
                               });
#pragma unroll
  for (int s = 0; s < 8; ++s) w[1][s] = make_double2(kk[s], 0.0);
  lds_barrier();  // split_pairs' mirror reads are done
  fftw_dit<W, -1, 1, SW_ROW_SP_FLY, false, false, PRUNE>(reinterpret_cast<double2(&)[1][8]>(w[1]), c.t, wt, tq, line, 0);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int k = c.t + s * Bk::NT;
    if (R::fwd_any(g, s) && k < g.kc) {
      const int o = ri.ofwd(g, s);
      Mo[o] = cadd(cmul_i(w[1][s], -(k * g.mk)), zv[s]);
      Mo[MF + o] = w[1][s];
    }
  }
}

// the pruned row transforms (k_row PRUNE) where they apply: the decimated
// transforms (roww) and a live band kc <= 3N/8 (every 2/3-rule grid;
// MultiLayerQG's aliased_fraction = 0 keeps the full ones).  SW_ROW_PRUNE=0:
// never (A/B builds)
#ifndef SW_ROW_PRUNE
#define SW_ROW_PRUNE 1
#endif
template <int L>
static bool row_prunable(const Geom& g) {
  return SW_ROW_PRUNE && roww<L>() > 0 && 8 * g.kc <= 3 * g.nx;
}

// the half rows with the live band at compile time (live_kc): the 2/3 rule's
// kc = nx/3 (SW_ROWH_KC=0: never, A/B).  Static VALU −20..−22 %, v_cndmask
// 355 → 166 (2LQG 8192) / 613 → 326 (RSW 4096); measured (tools/ab/r6_rowkc.sh,
// three interleaved rounds, bitwise equal): config 5 row 1598-1603 → 1545-1578
// µs (70.9 → 71.4-72.1 steps/s), config 4 row 360-362 → 356-357 µs
// (1349 → 1355)
#ifndef SW_ROWH_KC
#define SW_ROWH_KC 1
#endif
template <int L>
static bool rowh_kc(const Geom& g) {
  return SW_ROWH_KC && g.nslab == 1 && g.kc == (1 << L) / 3;
}
// the same for the full-length decimated rows (k_row<…, KC>; SW_ROW_KC=0:
// never).  Measured (tools/ab/r6_rowkc2.sh, three interleaved rounds, bitwise
// equal): RSW 2048 row static VALU 3362 → 2536, row 66.6-67.8 → 66.1-66.7 µs
// (6650-6684 → 6679-6691 steps/s), 1024² neutral — kept for RSW; the 2LQG
// row (4315 → 3574) ran slower, 69.9-72.1 → 71.5-73.5 µs; with the slab
// paths compiled out as well (k_row's KC variants since) it runs level to
// slightly faster, 71.7-73.3 → 71.1-72.3 µs, config 3 5795-5858 → 5829-5876
// (tools/ab/r6_qgkc.sh, bitwise equal): on (SW_ROW_KC_QG)
#ifndef SW_ROW_KC
#define SW_ROW_KC 1
#endif
#ifndef SW_ROW_KC_QG
#define SW_ROW_KC_QG 1
#endif
// short (split) rows of the drivers' 512² grids, RSW and Thomas–Yamada
// (SW_ROW_KC_SHORT).  Measured (tools/ab/r6_rowkc9.sh, three rounds, bitwise
// equal): TYdriver 512² ETDRK4 6289-6336 → 6656-6725 steps/s (row 18.0 →
// 16.0-16.7 µs), RSWDriver 512² IFMAB3 32210-32871 → 32848-33620
#ifndef SW_ROW_KC_SHORT
#define SW_ROW_KC_SHORT 1
#endif
// MultiLayerQG's short rows (aliased_fraction = 0: kc = nx/2; SW_ROW_KC_MLQG).
// Measured (tools/ab/r6_rowkc_mlqg.sh, bitwise equal): TwoLayerSimulation 512²
// FilteredRK4 7188-7251 → 7508-7607 steps/s (row 11.0-11.4 → 9.6-9.9 µs)
#ifndef SW_ROW_KC_MLQG
#define SW_ROW_KC_MLQG 1
#endif
template <int L>
static bool row_kc(const Geom& g, bool qg = false, bool shortrow = false) {
  return SW_ROW_KC && g.nslab == 1 && (!qg || SW_ROW_KC_QG) && (!shortrow || SW_ROW_KC_SHORT) && g.kc == (1 << L) / 3;
}

template <int L>
void LenOps<L>::row(int model, const Geom& g, const Phys& p, const double2* Mi, double2* Mo, const double2* tw,
                    hipStream_t s, int y0, int nrows, double2* Ma) {
  if (nrows < 0) nrows = g.nyl - y0;
  using BR = BlkRow<MODEL_RSW, L>;
  using BQ = BlkRow<MODEL_QG2, L>;
  using BT = BlkRow<MODEL_TY, L>;
  constexpr size_t sh_rsw = row_lds_lines<MODEL_RSW, L>() * FftPlan<L>::LDS * BR::NB * sizeof(double2);
  constexpr size_t sh_qg2 = row_lds_lines<MODEL_QG2, L>() * FftPlan<L>::LDS * BQ::NB * sizeof(double2);
  constexpr size_t sh_ty = FftPlan<L>::LDS * BT::NB * sizeof(double2);
  if (model == MODEL_RSW) {
    constexpr int nbr = rowh_nb<L, true>();
    if constexpr (rsw_row_half<L>()) {
      if (rowh_kc<L>(g))
        SW_LAUNCH((k_row_rsw_h<L, (1 << L) / 3>), dim3(nrows / nbr), dim3(RowH<L>::NTH * nbr),
                           nbr * rsw_rowh_lines<L>() * FftPlan<L - 1>::LDS * sizeof(double2), s, g, p, Mi, Mo,
                           tw, y0);
      else
        SW_LAUNCH((k_row_rsw_h<L>), dim3(nrows / nbr), dim3(RowH<L>::NTH * nbr),
                           nbr * rsw_rowh_lines<L>() * FftPlan<L - 1>::LDS * sizeof(double2), s, g, p, Mi, Mo,
                           tw, y0);
      return;
    }
    if constexpr (roww<L>() > 0 && BR::NB == 1) {
      if (g.rsp) {  // (Geom::rsp: the row over two blocks, k_row_rsw_sp)
        if (row_prunable<L>(g))
          SW_LAUNCH((k_row_rsw_sp<L, true>), dim3(2 * nrows), dim3(BR::THREADS),
                             FftPlan<L>::LDS * sizeof(double2), s, g, p, Mi, Mo, tw, y0);
        else
          SW_LAUNCH((k_row_rsw_sp<L, false>), dim3(2 * nrows), dim3(BR::THREADS),
                             FftPlan<L>::LDS * sizeof(double2), s, g, p, Mi, Mo, tw, y0);
        return;
      }
    }
    if (row_prunable<L>(g) && row_kc<L>(g))
      SW_LAUNCH((k_row<MODEL_RSW, L, false, true, false, (1 << L) / 3>), dim3(nrows / BR::NB), dim3(BR::THREADS),
                         sh_rsw, s, g, p, Mi, Mo, tw, y0, nullptr);
    else if (row_prunable<L>(g))
      SW_LAUNCH((k_row<MODEL_RSW, L, false, true>), dim3(nrows / BR::NB), dim3(BR::THREADS), sh_rsw, s, g,
                         p, Mi, Mo, tw, y0, nullptr);
    else if (g.rsplit && row_lds_lines<MODEL_RSW, L>() == 2 && roww<L>() == 0 && row_kc<L>(g, false, true))
      SW_LAUNCH((k_row<MODEL_RSW, L, false, false, true, (1 << L) / 3>), dim3(nrows / BR::NB, 2),
                         dim3(BR::THREADS), sh_rsw, s, g, p, Mi, Mo, tw, y0, nullptr);
    else if (g.rsplit && row_lds_lines<MODEL_RSW, L>() == 2 && roww<L>() == 0)
      SW_LAUNCH((k_row<MODEL_RSW, L, false, false, true>), dim3(nrows / BR::NB, 2), dim3(BR::THREADS),
                         sh_rsw, s, g, p, Mi, Mo, tw, y0, nullptr);
    else
      SW_LAUNCH((k_row<MODEL_RSW, L>), dim3(nrows / BR::NB), dim3(BR::THREADS), sh_rsw, s, g, p, Mi, Mo,
                         tw, y0, nullptr);
  } else if (model == MODEL_TY) {
    if (Ma)
      SW_LAUNCH((k_row<MODEL_TY, L, true>), dim3(nrows / BT::NB), dim3(BT::THREADS), sh_ty, s, g, p, Mi,
                         Mo, tw, y0, Ma);
    else if (g.rsplit && row_kc<L>(g, false, true))
      SW_LAUNCH((k_row<MODEL_TY, L, false, false, true, (1 << L) / 3>), dim3(nrows / BT::NB, 4),
                         dim3(BT::THREADS), sh_ty, s, g, p, Mi, Mo, tw, y0, nullptr);
    else if (g.rsplit)
      SW_LAUNCH((k_row<MODEL_TY, L, false, false, true>), dim3(nrows / BT::NB, 4), dim3(BT::THREADS), sh_ty,
                         s, g, p, Mi, Mo, tw, y0, nullptr);
    else
      SW_LAUNCH((k_row<MODEL_TY, L>), dim3(nrows / BT::NB), dim3(BT::THREADS), sh_ty, s, g, p, Mi, Mo, tw,
                         y0, nullptr);
  } else if (model == MODEL_RSWA) {
    using BA = BlkRow<MODEL_RSWA, L>;
    if (Ma)
      SW_LAUNCH((k_row<MODEL_RSWA, L, true>), dim3(nrows / BA::NB), dim3(BA::THREADS),
                         FftPlan<L>::LDS * BA::NB * sizeof(double2), s, g, p, Mi, Mo, tw, y0, Ma);
    else
      SW_LAUNCH((k_row<MODEL_RSWA, L>), dim3(nrows / BA::NB), dim3(BA::THREADS),
                         FftPlan<L>::LDS * BA::NB * sizeof(double2), s, g, p, Mi, Mo, tw, y0, nullptr);
  }
  else if (Ma) {  // aliased-state tracking: the full-length row (it writes the aliased x-spectra)
    SW_LAUNCH((k_row<MODEL_QG2, L, true>), dim3(nrows / BQ::NB), dim3(BQ::THREADS), sh_qg2, s, g, p, Mi,
                       Mo, tw, y0, Ma);
  } else if constexpr (qg_row_half<L>()) {
    if (rowh_kc<L>(g))
      SW_LAUNCH((k_row_qg_h<L, (1 << L) / 3>), dim3(nrows / rowh_nb<L>()), dim3(RowH<L>::NTH * rowh_nb<L>()),
                         rowh_nb<L>() * FftPlan<L - 1>::LDS * sizeof(double2), s, g, p, Mi, Mo, tw, y0);
    else
      SW_LAUNCH((k_row_qg_h<L>), dim3(nrows / rowh_nb<L>()), dim3(RowH<L>::NTH * rowh_nb<L>()),
                         rowh_nb<L>() * FftPlan<L - 1>::LDS * sizeof(double2), s, g, p, Mi, Mo, tw, y0);
  } else if (row_prunable<L>(g) && row_kc<L>(g, true)) {
    SW_LAUNCH((k_row<MODEL_QG2, L, false, true, false, (1 << L) / 3>), dim3(nrows / BQ::NB), dim3(BQ::THREADS),
                       sh_qg2, s, g, p, Mi, Mo, tw, y0, nullptr);
  } else if (row_prunable<L>(g)) {
    SW_LAUNCH((k_row<MODEL_QG2, L, false, true>), dim3(nrows / BQ::NB), dim3(BQ::THREADS), sh_qg2, s, g, p,
                       Mi, Mo, tw, y0, nullptr);
  } else if (g.rsplit && SW_ROW_KC_MLQG && g.nslab == 1 && g.kc == (1 << L) / 2) {
    // (aliased_fraction = 0, TwoLayerSimulation's MultiLayerQG: kc = nx/2)
    SW_LAUNCH((k_row<MODEL_QG2, L, false, false, true, (1 << L) / 2>), dim3(nrows / BQ::NB, 2),
                       dim3(BQ::THREADS), sh_qg2, s, g, p, Mi, Mo, tw, y0, nullptr);
  } else if (g.rsplit) {
    SW_LAUNCH((k_row<MODEL_QG2, L, false, false, true>), dim3(nrows / BQ::NB, 2), dim3(BQ::THREADS), sh_qg2,
                       s, g, p, Mi, Mo, tw, y0, nullptr);
  } else {
    SW_LAUNCH((k_row<MODEL_QG2, L>), dim3(nrows / BQ::NB), dim3(BQ::THREADS), sh_qg2, s, g, p, Mi, Mo, tw,
                       y0, nullptr);
  }
}

template <int L>
void LenOps<L>::col_fwd_alias(int model, const Geom& g, const Geom& ga, int region, const Phys& p,
                              const double2* Mf, const double2* Ma, double2* N, const double2* tw, hipStream_t s) {
  const int nb = (ga.kcn + Blk<L>::NB - 1) / Blk<L>::NB;
  if (model == MODEL_RSWA)
    SW_LAUNCH((k_col_fwd_alias<MODEL_RSWA, L>), dim3(nb, 3), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g,
                       ga, region, p, Mf, Ma, N, tw);
  else if (model == MODEL_TY)
    SW_LAUNCH((k_col_fwd_alias<MODEL_TY, L>), dim3(nb, 4), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g,
                       ga, region, p, Mf, Ma, N, tw);
  else
    SW_LAUNCH((k_col_fwd_alias<MODEL_QG2, L>), dim3(nb, 2), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g,
                       ga, region, p, Mf, Ma, N, tw);
}

template <int L>
void LenOps<L>::col_fwd(int model, const Geom& g, const Phys& p, const double2* Mf, double2* N, const double2* X,
                        const double2* tw, hipStream_t s, int f0, int nfl, double2* T1, double2* T2) {
  const dim3 grid(col_blocks<L>(g), nfl), grid3(col_blocks<L>(g), 3 * nfl), blk(Blk<L>::THREADS);
  const size_t sh = lds_bytes<L>();
  const int bnd = band_of<L>(g);
  const bool split = T1 != nullptr;  // (RSW, 2LQG / MultiLayerQG, Thomas–Yamada)
  if (model == MODEL_RSW && split)
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_RSW, L, true, SWB>), grid3, blk, sh, s, g, p, Mf, N, X, tw, f0, T1, T2);
  else if (model == MODEL_RSW)
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_RSW, L, false, SWB>), grid, blk, sh, s, g, p, Mf, N, X, tw, f0, nullptr, nullptr);
  else if (model == MODEL_RSWA)
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_RSWA, L, false, SWB>), grid, blk, sh, s, g, p, Mf, N, X, tw, f0, nullptr, nullptr);
  else if (model == MODEL_TY && split)
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_TY, L, true, SWB>), grid3, blk, sh, s, g, p, Mf, N, X, tw, f0, T1, T2);
  else if (model == MODEL_TY)
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_TY, L, false, SWB>), grid, blk, sh, s, g, p, Mf, N, X, tw, f0, nullptr, nullptr);
  else if (split)
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_QG2, L, true, SWB>), grid3, blk, sh, s, g, p, Mf, N, X, tw, f0, T1, T2);
  else
    SW_LAUNCH_BAND(bnd, (k_col_fwd<MODEL_QG2, L, false, SWB>), grid, blk, sh, s, g, p, Mf, N, X, tw, f0, nullptr, nullptr);
}

template <int L>
void LenOps<L>::col_inv1(const Geom& g, const double2* X, double2* M, const double2* tw, hipStream_t s) {
  SW_LAUNCH((k_col_inv1<L>), dim3(col_blocks<L>(g)), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, X, M, tw);
}

template <int L>
void LenOps<L>::row_c2r1(const Geom& g, const double2* M, double* out, const double2* tw, hipStream_t s) {
  SW_LAUNCH((k_row_c2r1<L>), dim3(row_blocks<L>(g)), dim3(Blk<L>::THREADS), lds_bytes<L>(), s, g, M, out, tw);
}

template <int L>
void LenOps<L>::col_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a, const double2* Mf,
                         double2* Minv, const double2* tw, hipStream_t s, int f0, int nfl) {
  const dim3 grid(col_blocks<L>(g)), blk(Blk<L>::THREADS);
  const size_t sh = lds_bytes<L>();
#define SW_CS(M, O) SW_LAUNCH((k_col_step<M, L, O>), grid, blk, sh, s, g, p, a, Mf, Minv, tw)
  if (model == MODEL_RSW) {
    // all three fields: the XCD-interleaved 1-D grid where it applies; a
    // field range (pipelined slab exchange): one grid row per field
    const bool all = f0 == 0 && nfl == 3;
    if (op == OP_FAB3) {
      const bool one = all && Blk<L>::NB == 1 && g.kcl % 64 == 0;
      const dim3 gr = one ? dim3(3 * g.kcl) : dim3(col_blocks<L>(g), nfl);
      if (a.stream)
        SW_LAUNCH_BAND(band_of<L>(g), (k_col_step_fab3_rsw<L, true, SWB>), gr, blk, sh, s, g, p, a, Mf, Minv, tw,
                       one ? -1 : f0);
      else
        SW_LAUNCH_BAND(band_of<L>(g), (k_col_step_fab3_rsw<L, false, SWB>), gr, blk, sh, s, g, p, a, Mf, Minv, tw,
                       one ? -1 : f0);
    } else if (op == OP_IFMAB3) SW_CS(MODEL_RSW, OP_IFMAB3);
    else SW_CS(MODEL_RSW, OP_RK4);
  } else {
    if (op == OP_FAB3) SW_CS(MODEL_QG2, OP_FAB3);
    else if (op == OP_IFMAB3) SW_CS(MODEL_QG2, OP_IFMAB3);
    else SW_CS(MODEL_QG2, OP_RK4);
  }
#undef SW_CS
}

template <int L>
size_t LenOps<L>::fwd_step_lds_bytes(int model, const Geom& g) {
  return (size_t)Blk<L>::NB * (FftPlan<L>::LDS + (size_t)(model == MODEL_RSW ? 3 : 2) * g.Lr) * sizeof(double2);
}

template <int L>
void LenOps<L>::col_fwd_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a, const double2* Mf,
                             const double2* tw, hipStream_t s, bool lds) {
  const dim3 grid(col_blocks<L>(g)), blk(Blk<L>::THREADS);
  const size_t sh = lds ? fwd_step_lds_bytes(model, g) : lds_bytes<L>();
#define SW_FS(M, O)                                                                                         \
  do {                                                                                                      \
    if (lds) {                                                                                              \
      if (a.stream) SW_LAUNCH((k_col_fwd_step_lds<M, L, O, true>), grid, blk, sh, s, g, p, a, Mf, tw); \
      else SW_LAUNCH((k_col_fwd_step_lds<M, L, O, false>), grid, blk, sh, s, g, p, a, Mf, tw);        \
    } else if (a.stream) SW_LAUNCH((k_col_step<M, L, O, false, true>), grid, blk, sh, s, g, p, a, Mf, nullptr, tw); \
    else SW_LAUNCH((k_col_step<M, L, O, false, false>), grid, blk, sh, s, g, p, a, Mf, nullptr, tw);        \
  } while (0)
  if (model == MODEL_RSW) {
    if (op == OP_IFMAB3) SW_FS(MODEL_RSW, OP_IFMAB3);
    else SW_FS(MODEL_RSW, OP_RK4);
  } else {
    if (op == OP_FAB3) SW_FS(MODEL_QG2, OP_FAB3);
    else if (op == OP_IFMAB3) SW_FS(MODEL_QG2, OP_IFMAB3);
    else if (op == OP_FRK4) SW_FS(MODEL_QG2, OP_FRK4);
    else SW_FS(MODEL_QG2, OP_RK4);
  }
#undef SW_FS
}

#ifdef SW_PART
template struct LenOps<SW_PART>;
#endif
#endif  // length-templated launchers

#if !defined(SW_PART) || SW_PART == 0
// host-side: dispatch the LOG2N instantiation (N = 32 … 8192)
template <typename F>
static void by_len(int log2n, F&& f) {
  switch (log2n) {
#define SW_CASE(L)                          \
  case L:                                   \
    f(std::integral_constant<int, L>{});    \
    break;
    SW_LOG2_CASES(SW_CASE)
#undef SW_CASE
    default:
      break;
  }
}

bool length_built(int log2n) {
  bool ok = false;
  by_len(log2n, [&](auto) { ok = true; });
  return ok;
}

// number of column-pass groups per launch unit: col_inv groups, col_fwd fields
int col_inv_groups(int model) { return (model == MODEL_RSW || model == MODEL_RSWA) ? 3 : (model == MODEL_TY ? 5 : 2); }
int col_fields(int model) { return (model == MODEL_RSW || model == MODEL_RSWA) ? 3 : (model == MODEL_TY ? 4 : 2); }

void launch_col_inv(int model, const Geom& g, const Phys& p, const double2* X, double2* Minv,
                    const double2* tw_y, hipStream_t s, int g0, int ng) {
  if (ng < 0) ng = col_inv_groups(model) - g0;
  by_len(g.log2ny, [&](auto L) { LenOps<decltype(L)::value>::col_inv(model, g, p, X, Minv, tw_y, s, g0, ng); });
}
void launch_row(int model, const Geom& g, const Phys& p, const double2* Minv, double2* Mfwd,
                const double2* tw_x, hipStream_t s, int y0, int nrows, double2* Ma) {
  by_len(g.log2nx, [&](auto L) { LenOps<decltype(L)::value>::row(model, g, p, Minv, Mfwd, tw_x, s, y0, nrows, Ma); });
}
bool row_alias_built(int model, int log2nx) {
  bool ok = false;
  by_len(log2nx, [&](auto L) {
    ok = model == MODEL_RSWA || model == MODEL_QG2 || model == MODEL_TY;
  });
  return ok;
}
void launch_col_fwd_alias(int model, const Geom& g, const Geom& ga, int region, const Phys& p, const double2* Mfwd,
                          const double2* Ma, double2* N, const double2* tw_y, hipStream_t s) {
  if (ga.kcn <= 0) return;
  by_len(g.log2ny, [&](auto L) {
    LenOps<decltype(L)::value>::col_fwd_alias(model, g, ga, region, p, Mfwd, Ma, N, tw_y, s);
  });
}
void launch_scatter_modes(int nf, const Geom& ga, const double2* cmp, double2* full, hipStream_t s) {
  if (ga.cfield <= 0 || ga.kcn <= 0) return;
  SW_LAUNCH(k_scatter_modes, dim3((unsigned)((ga.cfield + 255) / 256)), dim3(256), 0, s, ga, nf, cmp, full);
}
void launch_gather_modes(int nf, const Geom& ga, const double2* full, double2* cmp, hipStream_t s) {
  if (ga.cfield <= 0 || ga.kcn <= 0) return;
  SW_LAUNCH(k_gather_modes, dim3((unsigned)((ga.cfield + 255) / 256)), dim3(256), 0, s, ga, nf, full, cmp);
}
int row_lines_per_block(int model, int log2nx) {
  int nb = 1;
  by_len(log2nx, [&](auto L) {
    constexpr int l = decltype(L)::value;
    nb = model == MODEL_RSWA ? BlkRow<MODEL_RSWA, l>::NB
       : model == MODEL_RSW ? (rsw_row_half<l>() ? rowh_nb<l, true>() : BlkRow<MODEL_RSW, l>::NB)
                            : (model == MODEL_TY ? BlkRow<MODEL_TY, l>::NB
                                                 : (qg_row_half<l>() ? rowh_nb<l>() : BlkRow<MODEL_QG2, l>::NB));
  });
  return nb;
}
void launch_col_fwd(int model, const Geom& g, const Phys& p, const double2* Mfwd, double2* N,
                    const double2* X, const double2* tw_y, hipStream_t s, int f0, int nfl, double2* T1,
                    double2* T2) {
  if (nfl < 0) nfl = col_fields(model) - f0;
  by_len(g.log2ny,
         [&](auto L) { LenOps<decltype(L)::value>::col_fwd(model, g, p, Mfwd, N, X, tw_y, s, f0, nfl, T1, T2); });
}

static inline dim3 mode_grid(const Geom& g) { return dim3((unsigned)((g.cfield + 255) / 256)); }

void launch_col_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                     const double2* Mf, double2* Minv, const double2* tw_y, hipStream_t s, int f0, int nfl) {
  if (nfl < 0) nfl = col_fields(model) - f0;
  by_len(g.log2ny, [&](auto L) { LenOps<decltype(L)::value>::col_step(model, op, g, p, a, Mf, Minv, tw_y, s, f0, nfl); });
}

void launch_col_fwd_step(int model, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                         const double2* Mf, const double2* tw_y, hipStream_t s, bool lds) {
  by_len(g.log2ny, [&](auto L) { LenOps<decltype(L)::value>::col_fwd_step(model, op, g, p, a, Mf, tw_y, s, lds); });
}
size_t fwd_step_lds_bytes(int model, const Geom& g) {
  size_t b = 0;
  by_len(g.log2ny, [&](auto L) { b = LenOps<decltype(L)::value>::fwd_step_lds_bytes(model, g); });
  return b;
}

void launch_step_elem(int nf, int op, const Geom& g, const Phys& p, const StepPtrs& a,
                      const double2* N, double2* xs, hipStream_t s) {
#define SW_SE(F, O)                                                                                \
  do {                                                                                             \
    if (a.stream) SW_LAUNCH((k_step_elem<F, O, true>), mode_grid(g), dim3(256), 0, s, g, p, a, N, xs); \
    else SW_LAUNCH((k_step_elem<F, O, false>), mode_grid(g), dim3(256), 0, s, g, p, a, N, xs);       \
  } while (0)
  if (nf == 4) {
    SW_SE(4, OP_ETDRK4);
  } else if (nf == 3) {
    if (op == OP_FRK4) SW_SE(3, OP_FRK4);
    else if (op == OP_FAB3) SW_SE(3, OP_FAB3);
    else if (op == OP_IFMAB3) SW_SE(3, OP_IFMAB3);
    else SW_SE(3, OP_RK4);
  } else {
    if (op == OP_FRK4) SW_SE(2, OP_FRK4);
    else if (op == OP_FAB3) SW_SE(2, OP_FAB3);
    else if (op == OP_IFMAB3) SW_SE(2, OP_IFMAB3);
    else SW_SE(2, OP_RK4);
  }
#undef SW_SE
}

// a split N completed in place (sw_calcN: the caller reads N itself)
template <int NF>
static __global__ void __launch_bounds__(256) k_assemble(Geom g, Phys p, StepPtrs a, double2* __restrict__ N) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  int kr, j;
  if (i >= g.cfield || !mode_of(g, i, kr, j)) return;
  cplx n[NF];
  load_vec<NF>(N, g.cfield, i, n);
  assemble_terms<NF>(g, p, a, i, kr * g.mk, lwav(g, lrow_of(g, j)), n);
  store_vec<NF>(N, g.cfield, i, n);
}
void launch_assemble_terms(int nf, const Geom& g, const Phys& p, const StepPtrs& a, double2* N, hipStream_t s) {
  if (nf == 4) SW_LAUNCH((k_assemble<4>), mode_grid(g), dim3(256), 0, s, g, p, a, N);
  else if (nf == 3) SW_LAUNCH((k_assemble<3>), mode_grid(g), dim3(256), 0, s, g, p, a, N);
  else SW_LAUNCH((k_assemble<2>), mode_grid(g), dim3(256), 0, s, g, p, a, N);
}

void launch_gather(int nf, const Geom& g, const double2* full, double2* cmp, hipStream_t s) {
  const long long n = (long long)g.kcn * g.Lr * nf;
  if (n == 0) return;
  SW_LAUNCH(k_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, nf, full, cmp);
}

void launch_scatter(int nf, const Geom& g, int lo, int hi, const double2* cmp, double2* full, hipStream_t s) {
  const long long n = (long long)(hi - lo) * g.nl * nf;
  if (n <= 0) return;
  SW_LAUNCH(k_scatter, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, nf, lo, hi, cmp, full);
}

void launch_nan_check(int nf, const Geom& g, const double2* cmp, int* flag, hipStream_t s) {
  SW_LAUNCH(k_nan_check, mode_grid(g), dim3(256), 0, s, g, nf, cmp, flag);
}

void launch_make_spec(int model, int fid, const Geom& g, const Phys& p, const double2* sol,
                      double2* out, hipStream_t s) {
  SW_LAUNCH(k_make_spec, mode_grid(g), dim3(256), 0, s, g, p, model, fid, sol, out);
}

void launch_col_inv1(const Geom& g, const double2* X, double2* M, const double2* tw_y, hipStream_t s) {
  by_len(g.log2ny, [&](auto L) { LenOps<decltype(L)::value>::col_inv1(g, X, M, tw_y, s); });
}

void launch_row_c2r1(const Geom& g, const double2* M, double* out, const double2* tw_x, hipStream_t s) {
  by_len(g.log2nx, [&](auto L) { LenOps<decltype(L)::value>::row_c2r1(g, M, out, tw_x, s); });
}

void launch_energy_cols(int model, const Geom& g, const Phys& p, const double2* sol, double* cols,
                        hipStream_t s) {
  SW_LAUNCH(k_energy_cols, dim3(g.kcl), dim3(256), 0, s, g, p, model, sol, cols);
}

void launch_energy_final(const double* cols, int ncols, double* out, hipStream_t s) {
  SW_LAUNCH(k_energy_final, dim3(1), dim3(64), 0, s, cols, ncols, out);
}

void launch_absmax(const double* f, long long n, unsigned long long* out, int sgn, hipStream_t s) {
  SW_LAUNCH(k_absmax, dim3(1024), dim3(256), 0, s, f, n, out, sgn);
}

// caller-buffer precision (sw_config.precision = SW_PREC_F32): one rounding
// on the way out, exact widening on the way in
static __global__ void k_widen(const float* __restrict__ in, double* __restrict__ out, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (double)in[i];
}
static __global__ void k_narrow(const double* __restrict__ in, float* __restrict__ out, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}
void launch_widen(const float* in, double* out, long long n, hipStream_t s) {
  SW_LAUNCH(k_widen, dim3(2048), dim3(256), 0, s, in, out, n);
}
void launch_narrow(const double* in, float* out, long long n, hipStream_t s) {
  SW_LAUNCH(k_narrow, dim3(2048), dim3(256), 0, s, in, out, n);
}

void launch_etd_coeffs(const Geom& g, const Phys& p, double* etd, hipStream_t s) {
  SW_LAUNCH(k_etd_coeffs, mode_grid(g), dim3(256), 0, s, g, p, etd);
}

#endif  // SW_PART == 0

}  // namespace sw
