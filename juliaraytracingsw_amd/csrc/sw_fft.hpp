// Device-side fp64 FFT primitive for gfx950: one power-of-two transform of
// length N = 2^LOG2N per "line", NT = N/8 threads per line, 8 complex points
// per thread, Stockham autosort stages (one leading radix-2/4 stage when
// LOG2N is not a multiple of 3, then radix-8 stages) exchanged through LDS.
// The length is a template parameter, so every stage unrolls with constant
// LDS offsets and no per-stage index arithmetic.
//
// Register convention: on entry thread t of a line holds v[s] = x[t + s*NT];
// on exit it holds v[s] = X[t + s*NT] (natural order).  The last radix-8
// stage already leaves its outputs at t + r*NT, so no final LDS round trip
// is made; callers that write LDS after fft_line must lds_barrier() first.
// DIR = -1: forward exp(-2πi jk/N); DIR = +1: inverse, unnormalised.
// Twiddles: the first power W^k of every twiddled stage is loaded once per
// kernel (Twiddles::load); the other six powers are formed by complex
// multiplication (≤ 3 roundings deep).  These transforms replace FF's
// rfftplan (CUFFT/FFTW) calls, SURVEY A2.
#pragma once
#include <hip/hip_runtime.h>

// No implicit FMA contraction anywhere in libsw's device code: every kernel
// that evaluates the same formula rounds it the same way (the fused column
// pass is bitwise identical to the separate kernels).  Complex products use
// explicit fma below.
#pragma clang fp contract(off)

namespace sw {

// LDS index of line element i (16-B complex units).  Swizzle: no
// padding, bits 0-2 XOR bits 3-5 — conflict-free for every access of the
// transforms (MI355X_MICROARCH.md §LDS: ds_write_b128 serves lanes in groups
// of 8 over 128 B, ds_read_b128 in groups of 16 over 256 B): the consecutive
// loads and split stores (aligned 4-blocks stay in place), the radix-4 first
// stage's stores 4j + r (bank bits = r ^ (j bits 1,2), j bit 0) and the Ns = 4
// stage's stores 32(t/4) + t%4 + 4r (bank bit 2 = bit 5).  Padding: one
// pad element every 8 (LP(i) = i + i/8): conflict-free stores, but 2-way
// conflicts in the 16-lane read groups (24 % of LDS cycles, round-2 PMC).
// Per transform length: lines of at least 2^SW_LDS_SWZ_LOG2 points swizzle,
// shorter ones pad (measured: the RSW 2048² row 77.9 → 77.0 µs with the
// swizzle; the Thomas–Yamada 512² row 26.8 → 27.6 with it: its extra index
// arithmetic spills there).
#ifndef SW_LDS_SWZ_LOG2
#define SW_LDS_SWZ_LOG2 11
#endif
template <int LOG2N>
__host__ __device__ constexpr bool lds_swz() { return LOG2N >= SW_LDS_SWZ_LOG2; }
template <int LOG2N>
__host__ __device__ constexpr int LP(int i) { return lds_swz<LOG2N>() ? (i ^ ((i >> 3) & 7)) : i + (i >> 3); }
template <int LOG2N>
__host__ __device__ constexpr int lds_line_elems() { return lds_swz<LOG2N>() ? (1 << LOG2N) : (1 << LOG2N) + (1 << LOG2N) / 8; }

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x));
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
__device__ __forceinline__ void dft8(double2 (&v)[8]) {
  const double c = 0.70710678118654752440084436210485;
  double2 a0 = cadd(v[0], v[4]), a1 = cadd(v[1], v[5]), a2 = cadd(v[2], v[6]), a3 = cadd(v[3], v[7]);
  double2 b0 = csub(v[0], v[4]), b1 = csub(v[1], v[5]), b2 = csub(v[2], v[6]), b3 = csub(v[3], v[7]);
  // b_r *= W8^r, W8 = c(1 + DIR i)
  b1 = make_double2(c * (b1.x - DIR * b1.y), c * (b1.y + DIR * b1.x));
  b2 = (DIR < 0) ? make_double2(b2.y, -b2.x) : make_double2(-b2.y, b2.x);
  b3 = make_double2(c * (-b3.x - DIR * b3.y), c * (-b3.y + DIR * b3.x));
  dft4<DIR>(a0, a1, a2, a3);
  dft4<DIR>(b0, b1, b2, b3);
  v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
  v[1] = b0; v[3] = b1; v[5] = b2; v[7] = b3;
}

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for
// every outstanding global load/store (vmcnt(0)), which would stall each FFT
// stage behind in-flight HBM traffic; the LDS exchange needs only
// lgkmcnt(0) before the barrier.
__device__ __forceinline__ void lds_barrier() {
#ifdef SW_SCHED_FENCE
  __builtin_amdgcn_sched_barrier(0);
#endif
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifndef SW_EXP_NOBAR  // experiment: no workgroup barrier (wrong results: the cost of the syncs)
  __builtin_amdgcn_s_barrier();
#endif
  asm volatile("" ::: "memory");
#ifdef SW_SCHED_FENCE
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// Opaque thread index on lines of at least 2^SW_OPAQUE_LOG2 points (512 or
// 1024 threads, 128 VGPRs): the addresses a helper derives from t (LDS offsets of
// every FFT stage, mirror indices, tile offsets) are recomputed per call (a
// few integer ops) instead of being shared across the kernel's many calls and
// spilled for its whole life.  8192²: RSW row 2892 → 2278 µs (spills 67 →
// 23), 2LQG row 2308 → 2158 µs (20 → 0); shorter lines measured neutral to
// slower (TY 512² col_inv +23 %), so they keep the shared addresses.  Round 3:
// 4096-point lines too, with the per-stage twiddles below and 4 waves per
// SIMD for their 512-thread blocks (two blocks per CU instead of one): RSW
// 4096² col_step 405 -> 382 µs, 2LQG 4096² row 533 -> 440, col_fwd 140 -> 126
// (tools/ab_lean.sh).
#ifndef SW_OPAQUE_LOG2
#define SW_OPAQUE_LOG2 12
#endif
#define SW_OPAQUE_T(t)                                                  \
  do {                                                                  \
    if constexpr (LOG2N >= SW_OPAQUE_LOG2) asm volatile("" : "+v"(t)); \
  } while (0)

template <int LOG2N>
struct FftPlan {
  static constexpr int N = 1 << LOG2N;
  static constexpr int NT = N / 8;
  static constexpr int REM = LOG2N % 3;
  static constexpr int FIRST8 = REM ? REM : 3;               // lNs of the first twiddled stage
  static constexpr int NTW = (LOG2N - FIRST8) / 3;            // twiddled radix-8 stages
  static constexpr int LDS = lds_line_elems<LOG2N>();          // complex per line buffer
};

// W^(k_i << (LOG2N - lNs_i - 3)) for every twiddled stage i (forward sign).
// Lines of 8192 points run 1024 threads per block, which caps a thread at
// 128 VGPRs, and 4096-point lines 512 threads at 4 waves per SIMD (two
// blocks per CU), the same cap: there the stage twiddles are read from the
// (L1-resident) table at each stage instead of being held in registers for
// the whole kernel.
#ifndef SW_TWFLY_LOG2
#define SW_TWFLY_LOG2 12  // lines of at least 2^this read their stage twiddles per stage
#endif
// lines of at least 2^this form the seven powers of a radix-8 stage's
// twiddle as a chain (two live at a time) instead of all at once
#ifndef SW_TW_CHAIN_LOG2
#define SW_TW_CHAIN_LOG2 12
#endif
// FLY: read per stage whatever the length (a kernel with little register room)
template <int LOG2N, bool FLY = (LOG2N >= SW_TWFLY_LOG2)>
struct Twiddles {
  static constexpr bool kPreload = !FLY;
  double2 w[(kPreload && FftPlan<LOG2N>::NTW > 0) ? FftPlan<LOG2N>::NTW : 1];
  const double2* tab = nullptr;
  int t0 = 0, sh = 0;
  // tw: W_L^m of a table of length L = N << tsh (tsh > 0: a longer line's
  // table, W_N^j = W_L^(j << tsh))
  __device__ __forceinline__ void load(int t, const double2* __restrict__ tw, int tsh = 0) {
    using P = FftPlan<LOG2N>;
    if constexpr (kPreload) {
#pragma unroll
      for (int i = 0; i < P::NTW; ++i) w[i] = tw[index(t, i) << tsh];
    } else {
      tab = tw;
      t0 = t;
      sh = tsh;
    }
  }
  __device__ __forceinline__ static int index(int t, int i) {
    using P = FftPlan<LOG2N>;
    const int lNs = P::FIRST8 + 3 * i;
    const int k = t & ((1 << lNs) - 1);
    return k << (LOG2N - lNs - 3);
  }
  // W^k of twiddled stage i for this thread
  __device__ __forceinline__ double2 get(int i) const {
    if constexpr (kPreload) return w[i];
    else return tab[index(t0, i) << sh];
  }
};

template <int LOG2N>
__device__ __forceinline__ void load_line(double2 (&v)[8], int t, const double2* __restrict__ line) {
  constexpr int NT = FftPlan<LOG2N>::NT;
  // padding: NT a multiple of 8 (N >= 64) gives LP(t + s*NT) = LP(t) + s*(NT + NT/8);
  // swizzle: NT a multiple of 64 (N >= 512) gives LP(t + s*NT) = LP(t) + s*NT
  constexpr bool swz = lds_swz<LOG2N>();
  constexpr bool lin = swz ? (NT % 64 == 0) : (NT % 8 == 0);
  constexpr int step = swz ? NT : NT + NT / 8;
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = line[lin ? LP<LOG2N>(t) + s * step : LP<LOG2N>(t + s * NT)];
}

// C independent transforms of one line each, sharing every barrier (C LDS
// line buffers, `stride` complex apart).  v[c] holds x[t + s*NT] on entry and
// X[t + s*NT] on exit.  All threads of the block must call this (barriers).
template <int LOG2N, int DIR, int C, bool FLY = (LOG2N >= SW_TWFLY_LOG2)>
__device__ __forceinline__ void fft_lines(double2 (&v)[C][8], int t, const Twiddles<LOG2N, FLY>& tws,
                                          double2* __restrict__ line, int stride) {
  using P = FftPlan<LOG2N>;
  constexpr int NT = P::NT;
  // opaque t on the long lines and in kernels with little register room (FLY)
  if constexpr (LOG2N >= SW_OPAQUE_LOG2 || FLY) asm volatile("" : "+v"(t));
  // Opaque copy of the stage twiddles: keeps the compiler from sharing the
  // derived powers w2..w7 across the several transforms of one kernel, which
  // would pin 28 VGPRs per stage for the kernel's whole lifetime.
  double2 tw1[P::NTW > 0 ? P::NTW : 1];
  constexpr bool kPre = Twiddles<LOG2N, FLY>::kPreload;
  if constexpr (kPre) {
#pragma unroll
    for (int i = 0; i < P::NTW; ++i) {
      tw1[i] = tws.w[i];
      asm volatile("" : "+v"(tw1[i].x), "+v"(tw1[i].y));
    }
  }
  if constexpr (P::REM == 2) {  // radix-4, Ns = 1: butterflies j = t, t + NT
#pragma unroll
    for (int c = 0; c < C; ++c) {
      dft4<DIR>(v[c][0], v[c][2], v[c][4], v[c][6]);
      dft4<DIR>(v[c][1], v[c][3], v[c][5], v[c][7]);
    }
    lds_barrier();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = t + h * NT;
#pragma unroll
        for (int r = 0; r < 4; ++r) line[c * stride + LP<LOG2N>(4 * j + r)] = v[c][h + 2 * r];
      }
    lds_barrier();
#pragma unroll
    for (int c = 0; c < C; ++c) load_line<LOG2N>(v[c], t, line + c * stride);
  } else if constexpr (P::REM == 1) {  // radix-2, Ns = 1: butterflies j = t + h*NT, h < 4
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < 4; ++h) dft2<DIR>(v[c][h], v[c][h + 4]);
    lds_barrier();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int j = t + h * NT;
        line[c * stride + LP<LOG2N>(2 * j)] = v[c][h];
        line[c * stride + LP<LOG2N>(2 * j + 1)] = v[c][h + 4];
      }
    lds_barrier();
#pragma unroll
    for (int c = 0; c < C; ++c) load_line<LOG2N>(v[c], t, line + c * stride);
  }
  // radix-8 stages
  constexpr int S0 = P::REM ? P::REM : 0;
#pragma unroll
  for (int lNs = S0, ti = (P::REM ? 0 : -1); lNs + 3 <= LOG2N; lNs += 3, ++ti) {
    const int Ns = 1 << lNs;
    const int k = t & (Ns - 1);
#ifdef SW_EXP_NOTW  // experiment: no twiddle multiplications (wrong results)
    if (false) {
#else
    if (lNs > 0) {
#endif
      const double2 wt = kPre ? tw1[ti] : tws.get(ti);
      const double2 w1 = DIR < 0 ? wt : cconj(wt);
      if constexpr (kPre && LOG2N < SW_TW_CHAIN_LOG2) {
        const double2 w2 = cmul(w1, w1), w3 = cmul(w2, w1), w4 = cmul(w2, w2);
        const double2 w5 = cmul(w4, w1), w6 = cmul(w3, w3), w7 = cmul(w4, w3);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          v[c][1] = cmul(v[c][1], w1);
          v[c][2] = cmul(v[c][2], w2);
          v[c][3] = cmul(v[c][3], w3);
          v[c][4] = cmul(v[c][4], w4);
          v[c][5] = cmul(v[c][5], w5);
          v[c][6] = cmul(v[c][6], w6);
          v[c][7] = cmul(v[c][7], w7);
        }
      } else {
        // register budget (8192; SW_TW_CHAIN_LOG2): powers formed as a chain, two live at a time
        double2 wp = w1;
#pragma unroll
        for (int r = 1; r < 8; ++r) {
#pragma unroll
          for (int c = 0; c < C; ++c) v[c][r] = cmul(v[c][r], wp);
          if (r < 7) wp = cmul(wp, w1);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c) dft8<DIR>(v[c]);
    if (lNs + 3 >= LOG2N) break;  // last stage: outputs already at t + r*NT
#ifdef SW_EXP_NOLDS  // experiment: no LDS exchange in the radix-8 stages (wrong results)
    continue;
#endif
    lds_barrier();                // in-place LDS: everyone has loaded this stage's inputs
    const int idxD = ((t >> lNs) << (lNs + 3)) + k;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (lds_swz<LOG2N>() ? lNs >= 6 : lNs >= 3) {  // r * Ns moves no bit the index function mixes
        const int base = LP<LOG2N>(idxD);
#pragma unroll
        for (int r = 0; r < 8; ++r) line[c * stride + base + r * (lds_swz<LOG2N>() ? Ns : Ns + Ns / 8)] = v[c][r];
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) line[c * stride + LP<LOG2N>(idxD + r * Ns)] = v[c][r];
      }
    }
    lds_barrier();
#pragma unroll
    for (int c = 0; c < C; ++c) load_line<LOG2N>(v[c], t, line + c * stride);
  }
}

// Full transform.  v holds x[t + s*NT] on entry and X[t + s*NT] on exit.
// All threads of the block must call this (it contains barriers).
template <int LOG2N, int DIR, bool FLY = (LOG2N >= SW_TWFLY_LOG2)>
__device__ __forceinline__ void fft_line(double2 (&v)[8], int t, const Twiddles<LOG2N, FLY>& tws,
                                         double2* __restrict__ line) {
  fft_lines<LOG2N, DIR, 1, FLY>(reinterpret_cast<double2(&)[1][8]>(v), t, tws, line, 0);
}

}  // namespace sw
