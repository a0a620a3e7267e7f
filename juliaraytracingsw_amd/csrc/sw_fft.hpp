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
// (tools/ab/ab_lean.sh).
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
#ifndef SW_TW_AHEAD
#define SW_TW_AHEAD 0
#endif
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

// LDS index with the layout chosen explicitly (SWZ: the swizzle; else the
// padding).  Wave-local transforms (WL below) always swizzle: their regions
// tile a longer line buffer without padding.
template <bool SWZ>
__host__ __device__ constexpr int LPs(int i) { return SWZ ? (i ^ ((i >> 3) & 7)) : i + (i >> 3); }

template <int LOG2N, bool SWZ = lds_swz<LOG2N>()>
__device__ __forceinline__ void load_line(double2 (&v)[8], int t, const double2* __restrict__ line) {
  constexpr int NT = FftPlan<LOG2N>::NT;
  // padding: NT a multiple of 8 (N >= 64) gives LP(t + s*NT) = LP(t) + s*(NT + NT/8);
  // swizzle: NT a multiple of 64 (N >= 512) gives LP(t + s*NT) = LP(t) + s*NT
  constexpr bool lin = SWZ ? (NT % 64 == 0) : (NT % 8 == 0);
  constexpr int step = SWZ ? NT : NT + NT / 8;
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = line[lin ? LPs<SWZ>(t) + s * step : LPs<SWZ>(t + s * NT)];
}

// LDS ordering inside one wave (wave-local transforms): a wave's LDS
// instructions execute in order, so its own exchange needs no workgroup
// barrier; the wait keeps the compiler and the counters honest.
__device__ __forceinline__ void wave_lds_fence() {
  // (without the wait, in-order LDS alone would order it: measured slower,
  // row 75.6 vs 74.9 µs)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
template <bool WL>
__device__ __forceinline__ void stage_sync() {
  if constexpr (WL) wave_lds_fence();
  else lds_barrier();
}

// Two wave-local 512-point transforms software-pipelined (SW_WL_PIPE, round
// 6): a wave's LDS instructions execute in order, so line c's exchange (its
// stage writes, then the next stage's reads of the same region) is issued
// without waiting, and the other line's butterflies run while it is in flight;
// the compiler's own lgkmcnt waits hold each line's reads until it uses them.
// The same butterflies, twiddles and exchanges as fft_lines<9, DIR, 2, FLY,
// true, SHARE> in another order: bitwise the same results (state hashes at
// 1024² and 2048²).  Measured (tools/ab/r6_wlpipe.sh, three interleaved
// rounds): RSW 2048 row 66.6-67.6 → 65.3-66.6 µs, 222 → 176 VGPRs (still two
// waves per SIMD: the two line buffers cap a CU at two blocks), 6604-6638 →
// 6647-6680 steps/s; 1024² neutral.  Used where two wave-local lines are
// transformed together (the RSW rows' pairs).
#ifndef SW_WL_PIPE
#define SW_WL_PIPE 1
#endif
template <int DIR, bool FLY, bool SHARE>
__device__ __forceinline__ void fft512_wl2_pipe(double2 (&v)[2][8], int t, const Twiddles<9, FLY>& tws,
                                                double2* __restrict__ line, int stride) {
  using P = FftPlan<9>;
  static_assert(P::NTW == 2 && P::REM == 0, "512 = 8·8·8");
  if constexpr (FLY) asm volatile("" : "+v"(t));
  constexpr bool kPre = Twiddles<9, FLY>::kPreload;
  double2 tw1[2];
  if constexpr (kPre) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      tw1[i] = tws.w[i];
      if constexpr (!SHARE) asm volatile("" : "+v"(tw1[i].x), "+v"(tw1[i].y));
    }
  }
  // stage lNs's outputs to the line's region, then the next stage's inputs
  auto exch = [&](int c, int lNs) {
    const int Ns = 1 << lNs, k = t & (Ns - 1);
    const int idxD = ((t >> lNs) << (lNs + 3)) + k;
    double2* ln = line + c * stride;
    if (lNs >= 6) {
      const int base = LPs<true>(idxD);
#pragma unroll
      for (int r = 0; r < 8; ++r) ln[base + r * Ns] = v[c][r];
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) ln[LPs<true>(idxD + r * Ns)] = v[c][r];
    }
    asm volatile("" ::: "memory");  // (compiler order only: the reads stay after the writes)
    load_line<9, true>(v[c], t, ln);
  };
  // stage ti's twiddle powers (fft_lines' forms: all at once when preloaded,
  // a chain when read per stage), applied to line c, then its DFT-8
  double2 wq[8];
  auto powers = [&](int ti) {
    const double2 wt = kPre ? tw1[ti] : tws.get(ti);
    wq[1] = DIR < 0 ? wt : cconj(wt);
    if constexpr (kPre) {
      wq[2] = cmul(wq[1], wq[1]);
      wq[3] = cmul(wq[2], wq[1]);
      wq[4] = cmul(wq[2], wq[2]);
      wq[5] = cmul(wq[4], wq[1]);
      wq[6] = cmul(wq[3], wq[3]);
      wq[7] = cmul(wq[4], wq[3]);
    } else {
#pragma unroll
      for (int r = 2; r < 8; ++r) wq[r] = cmul(wq[r - 1], wq[1]);
    }
  };
  auto twdft = [&](int c) {
#pragma unroll
    for (int r = 1; r < 8; ++r) v[c][r] = cmul(v[c][r], wq[r]);
    dft8<DIR>(v[c]);
  };
  dft8<DIR>(v[0]);
  exch(0, 0);
  dft8<DIR>(v[1]);
  exch(1, 0);
  powers(0);
  twdft(0);
  exch(0, 3);
  twdft(1);
  exch(1, 3);
  powers(1);
  twdft(0);
  twdft(1);
}

// C independent transforms of one line each, sharing every barrier (C LDS
// line buffers, `stride` complex apart).  v[c] holds x[t + s*NT] on entry and
// X[t + s*NT] on exit.  All threads of the block must call this (barriers).
// WL: wave-local — the line's NT threads are one wave (NT = 64, N = 512) and
// `line` is that wave's own region: exchanges are ordered by wave_lds_fence,
// not by workgroup barriers, and the layout is the swizzle.
// SHARE: no opaque copy of the stage twiddles — the compiler may keep their
// powers for every transform of the kernel (registers for VALU; for kernels
// whose occupancy is set by LDS, not registers)
template <int LOG2N, int DIR, int C, bool FLY = (LOG2N >= SW_TWFLY_LOG2), bool WL = false, bool SHARE = false>
__device__ __forceinline__ void fft_lines(double2 (&v)[C][8], int t, const Twiddles<LOG2N, FLY>& tws,
                                          double2* __restrict__ line, int stride) {
  using P = FftPlan<LOG2N>;
  constexpr int NT = P::NT;
  constexpr bool SWZ = WL || lds_swz<LOG2N>();
  static_assert(!WL || NT == 64, "a wave-local transform is one wave's line");
  if constexpr (WL && C == 2 && SW_WL_PIPE) {
    fft512_wl2_pipe<DIR, FLY, SHARE>(v, t, tws, line, stride);
    return;
  }
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
      if constexpr (!SHARE) asm volatile("" : "+v"(tw1[i].x), "+v"(tw1[i].y));
    }
  }
  // read per stage (FLY): SW_TW_AHEAD=1 issues each stage's table read one
  // stage ahead (the first at entry), so a transform exposes one memory wait
  // instead of one per stage.  Measured neutral (round 3, config 5: col_fwd
  // 550 -> 537, row 1822 -> 1813, col_inv 876 -> 895 µs; config 4 ±0.3 %):
  // the other waves of the CU cover those waits, so off
  double2 twn = make_double2(1.0, 0.0);
  if constexpr (!kPre && P::NTW > 0 && SW_TW_AHEAD) twn = tws.get(0);
  if constexpr (P::REM == 2) {  // radix-4, Ns = 1: butterflies j = t, t + NT
#pragma unroll
    for (int c = 0; c < C; ++c) {
      dft4<DIR>(v[c][0], v[c][2], v[c][4], v[c][6]);
      dft4<DIR>(v[c][1], v[c][3], v[c][5], v[c][7]);
    }
    stage_sync<WL>();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = t + h * NT;
#pragma unroll
        for (int r = 0; r < 4; ++r) line[c * stride + LPs<SWZ>(4 * j + r)] = v[c][h + 2 * r];
      }
    stage_sync<WL>();
#pragma unroll
    for (int c = 0; c < C; ++c) load_line<LOG2N, SWZ>(v[c], t, line + c * stride);
  } else if constexpr (P::REM == 1) {  // radix-2, Ns = 1: butterflies j = t + h*NT, h < 4
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < 4; ++h) dft2<DIR>(v[c][h], v[c][h + 4]);
    stage_sync<WL>();
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int j = t + h * NT;
        line[c * stride + LPs<SWZ>(2 * j)] = v[c][h];
        line[c * stride + LPs<SWZ>(2 * j + 1)] = v[c][h + 4];
      }
    stage_sync<WL>();
#pragma unroll
    for (int c = 0; c < C; ++c) load_line<LOG2N, SWZ>(v[c], t, line + c * stride);
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
      double2 wt;
      if constexpr (kPre) {
        wt = tw1[ti];
      } else if constexpr (SW_TW_AHEAD) {
        wt = twn;
        if (ti + 1 < P::NTW) twn = tws.get(ti + 1);
      } else {
        wt = tws.get(ti);
      }
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
    stage_sync<WL>();                // in-place LDS: everyone has loaded this stage's inputs
    const int idxD = ((t >> lNs) << (lNs + 3)) + k;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (SWZ ? lNs >= 6 : lNs >= 3) {  // r * Ns moves no bit the index function mixes
        const int base = LPs<SWZ>(idxD);
#pragma unroll
        for (int r = 0; r < 8; ++r) line[c * stride + base + r * (SWZ ? Ns : Ns + Ns / 8)] = v[c][r];
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) line[c * stride + LPs<SWZ>(idxD + r * Ns)] = v[c][r];
      }
    }
    stage_sync<WL>();
#pragma unroll
    for (int c = 0; c < C; ++c) load_line<LOG2N, SWZ>(v[c], t, line + c * stride);
  }
}

// Full transform.  v holds x[t + s*NT] on entry and X[t + s*NT] on exit.
// All threads of the block must call this (it contains barriers).
template <int LOG2N, int DIR, bool FLY = (LOG2N >= SW_TWFLY_LOG2)>
__device__ __forceinline__ void fft_line(double2 (&v)[8], int t, const Twiddles<LOG2N, FLY>& tws,
                                         double2* __restrict__ line) {
  fft_lines<LOG2N, DIR, 1, FLY>(reinterpret_cast<double2(&)[1][8]>(v), t, tws, line, 0);
}

// ---------------------------------------------------------------------------
// Transforms of N = 512·W points over the W waves (NT = 64 W threads) of a
// line, decimated by W across the waves (Q = 512 = one wave × 8 points): one
// workgroup-wide LDS exchange per transform, the other two inside each wave
// (wave_lds_fence, no s_barrier) in that wave's region R_w = line + w Q of
// the line buffer.  W = 2, 4, 8: 1024-, 2048-, 4096-point lines.  With
// ω = exp(DIR 2πi/N), thread t holding x[t + NT s]:
//   DIF (fftw_dif, natural in → decimated out):
//     X[W m + c] = Σ_n ω_Q^(nm) · ω^(nc) Σ_q x[n + Qq] ω_W^(qc)
//     the radix-W over q and the twiddle ω^(nc) in the registers of thread
//     t (n = t + NT h, h < 8/W: x[n + Qq] is v[h + (8/W) q]), y_c[n] to R_c,
//     then wave c runs the Q-point transform: on exit lane j of wave c
//     holds X[W (j + 64 r) + c] in v[r].
//   DIT (fftw_dit, that decimated order in → natural out):
//     X[k + Qp] = Σ_c ω_W^(cp) · ω^(ck) Y_c[k],  Y_c = DFT_Q(x[W m + c])
//     wave c's Q-point transform, Y_c to R_c, then thread t reads Y_c[t +
//     NT h] of every c: on exit v[s] = X[t + NT s].
// ω^(ck) for k = t + NT h is ω^(ct) ω_8^(hc).  Physical-space work between
// the two (pointwise products) is order-blind.  wt = W_N^t with the forward
// sign, read once per kernel (a read here would put a memory wait, which
// also drains the stores in flight, in every transform); tq: the Q-point
// stage twiddles of lane t & 63 (Twiddles<9, FLY>::load(t & 63, tab,
// log2(N_tab / 512)) for a forward-sign table of length N_tab).  PRE: a
// workgroup barrier before the DIF's exchange writes (some thread may still
// be reading the line buffer) or before the DIT's first writes, which go to
// the wave's own region (needed when another wave may still read it).
// ---------------------------------------------------------------------------
// a · ω_8^k, ω_8 = exp(DIR 2πi/8), k in 0..3 (a constant once the callers'
// loops are unrolled)
template <int DIR>
__device__ __forceinline__ double2 w8_mul(double2 a, int k) {
  const double c = 0.70710678118654752440084436210485;
  if (k == 0) return a;
  if (k == 1) return make_double2(c * (a.x - DIR * a.y), c * (a.y + DIR * a.x));
  if (k == 2) return (DIR < 0) ? make_double2(a.y, -a.x) : make_double2(-a.y, a.x);
  return make_double2(c * (-a.x - DIR * a.y), c * (-a.y + DIR * a.x));
}

// in-place DFT-W (natural order) of a[0..W)
template <int W, int DIR>
__device__ __forceinline__ void dft_w(double2 (&a)[W]) {
  if constexpr (W == 2) dft2<DIR>(a[0], a[1]);
  else if constexpr (W == 4) dft4<DIR>(a[0], a[1], a[2], a[3]);
  else dft8<DIR>(a);
}

// Pruned radix-W butterflies of the decimated transforms (PRUNE): the
// row transforms' inputs are zero, and their outputs unused, at the natural
// positions [3N/8, 5N/8) — slots s = 3 and 4 of every thread — whenever the
// live band kc <= 3N/8 (the 2/3 rule: kc = N/3): the inverse inputs there are
// the dealiased modes kc <= k <= N - kc, the forward outputs k there are
// neither live (k < kc) nor a live mirror (N - k < kc).  ZM: bit q set ->
// a[q] is zero (inputs, DIF) or not needed (outputs, DIT).
__host__ __device__ constexpr bool prune_slot(int s) { return s == 3 || s == 4; }
template <int W, int HN, int H>
__host__ __device__ constexpr unsigned prune_mask() {
  unsigned m = 0;
  for (int q = 0; q < W; ++q)
    if (prune_slot(H + HN * q)) m |= 1u << q;
  return m;
}
__device__ __forceinline__ double2 cneg(double2 a) { return make_double2(-a.x, -a.y); }
// a + b, a - b with compile-time zeros (no rounding of x ± 0: the sign of a
// zero result may differ from the unpruned form, the values do not)
template <bool ZA, bool ZB>
__device__ __forceinline__ double2 zadd(double2 a, double2 b) {
  if constexpr (ZA && ZB) return make_double2(0.0, 0.0);
  else if constexpr (ZA) return b;
  else if constexpr (ZB) return a;
  else return cadd(a, b);
}
template <bool ZA, bool ZB>
__device__ __forceinline__ double2 zsub(double2 a, double2 b) {
  if constexpr (ZA && ZB) return make_double2(0.0, 0.0);
  else if constexpr (ZA) return cneg(b);
  else if constexpr (ZB) return a;
  else return csub(a, b);
}
// dft_w with the inputs of ZM known zero (DIF)
template <int W, int DIR, unsigned ZM>
__device__ __forceinline__ void dft_w_zin(double2 (&a)[W]) {
  if constexpr (ZM == 0) {
    dft_w<W, DIR>(a);
  } else if constexpr (W == 2) {
    const double2 x0 = a[0], x1 = a[1];
    a[0] = zadd<(ZM & 1) != 0, (ZM & 2) != 0>(x0, x1);
    a[1] = zsub<(ZM & 1) != 0, (ZM & 2) != 0>(x0, x1);
  } else if constexpr (W == 4) {
    constexpr bool z0 = ZM & 1, z1 = ZM & 2, z2 = ZM & 4, z3 = ZM & 8;
    const double2 s0 = zadd<z0, z2>(a[0], a[2]), s1 = zsub<z0, z2>(a[0], a[2]);
    const double2 s2 = zadd<z1, z3>(a[1], a[3]), d = zsub<z1, z3>(a[1], a[3]);
    const double2 s3 = (DIR < 0) ? make_double2(d.y, -d.x) : make_double2(-d.y, d.x);
    a[0] = cadd(s0, s2);
    a[2] = csub(s0, s2);
    a[1] = cadd(s1, s3);
    a[3] = csub(s1, s3);
  } else {
    dft_w<W, DIR>(a);  // W = 8 (4096-point lines): unpruned
  }
}

// the radix-8 decimations (4096-point lines: the 128-VGPR half rows) form
// the powers of ω^t as a chain, two live at a time (for_twiddles)
template <int W>
__host__ __device__ constexpr bool tw_chain() { return W == 8; }

// pw[c] = ω^(c t), c < W (pw[0] unused; tw_chain: pw[1] only).  tw_chain:
// ω^t made opaque per call, so that its powers (formed per transform) are not
// hoisted out of the caller's loops and kept for the kernel's life (the 2LQG
// half row at 8192 spilled 54 VGPRs on them)
template <int W, int DIR>
__device__ __forceinline__ void tw_powers(double2 wt, double2 (&pw)[W]) {
  if constexpr (tw_chain<W>()) asm volatile("" : "+v"(wt.x), "+v"(wt.y));
  pw[0] = make_double2(1.0, 0.0);
  if constexpr (W > 1) pw[1] = DIR < 0 ? wt : cconj(wt);
  if constexpr (tw_chain<W>()) return;
  if constexpr (W > 2) {
    pw[2] = cmul(pw[1], pw[1]);
    pw[3] = cmul(pw[2], pw[1]);
  }
  if constexpr (W > 4) {
    pw[4] = cmul(pw[2], pw[2]);
    pw[5] = cmul(pw[4], pw[1]);
    pw[6] = cmul(pw[3], pw[3]);
    pw[7] = cmul(pw[4], pw[3]);
  }
}

// ω^(q t) for q = 1 … W−1: the table pw, or (CHAIN: the 4096-point lines
// of the 128-VGPR half rows) a chain from pw[1], two powers live at a time
template <int W, int DIR, bool CHAIN, typename F>
__device__ __forceinline__ void for_twiddles(const double2 (&pw)[W], F f) {
  if constexpr (CHAIN) {
    double2 wq = pw[1];
#pragma unroll
    for (int q = 1; q < W; ++q) {
      f(q, wq);
      if (q + 1 < W) wq = cmul(wq, pw[1]);
    }
  } else {
#pragma unroll
    for (int q = 1; q < W; ++q) f(q, pw[q]);
  }
}
// the DIF's radix-W over q for h = H (then H + 1 …): pruned inputs per H
template <int W, int DIR, int C, bool PRUNE, int H>
__device__ __forceinline__ void dif_radix(double2 (&v)[C][8], const double2 (&pw)[W]) {
  constexpr int HN = 8 / W;
  if constexpr (H < HN) {
    constexpr unsigned ZM = PRUNE ? prune_mask<W, HN, H>() : 0u;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double2 a[W];
#pragma unroll
      for (int q = 0; q < W; ++q) a[q] = v[c][H + HN * q];
      dft_w_zin<W, DIR, ZM>(a);
      v[c][H] = a[0];
      for_twiddles<W, DIR, tw_chain<W>()>(pw, [&](int q, double2 wq) {
        v[c][H + HN * q] = w8_mul<DIR>(cmul(a[q], wq), H * q);
      });
    }
    dif_radix<W, DIR, C, PRUNE, H + 1>(v, pw);
  }
}

// PRUNE: slots 3 and 4 hold zeros (prune_slot: a live band kc <= 3N/8)
template <int W, int DIR, int C, bool PRE = true, bool FLY = false, bool SHARE = false, bool PRUNE = false>
__device__ __forceinline__ void fftw_dif(double2 (&v)[C][8], int t, double2 wt,
                                         const Twiddles<9, FLY>& tq, double2* __restrict__ line, int stride) {
  constexpr int Q = 512, NT = 64 * W, HN = 8 / W;
  static_assert(W == 2 || W == 4 || W == 8, "1024-, 2048- or 4096-point lines");
  double2 pw[W];
  tw_powers<W, DIR>(wt, pw);
  dif_radix<W, DIR, C, PRUNE && W != 8, 0>(v, pw);
  if constexpr (PRE) lds_barrier();
  const int b = LPs<true>(t);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int q = 0; q < W; ++q)
#pragma unroll
      for (int h = 0; h < HN; ++h) line[c * stride + q * Q + b + NT * h] = v[c][h + HN * q];
  lds_barrier();
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), j = t & 63;
  double2* reg = line + w * Q;
#pragma unroll
  for (int c = 0; c < C; ++c) load_line<9, true>(v[c], j, reg + c * stride);
  fft_lines<9, DIR, C, FLY, true, SHARE>(v, j, tq, reg, stride);
}

// PRUNE: slots 3 and 4 of the result are not needed (left zero)
template <int W, int DIR, int C, bool FLY = false, bool PRE = false, bool SHARE = false, bool PRUNE = false>
__device__ __forceinline__ void fftw_dit(double2 (&v)[C][8], int t, double2 wt,
                                         const Twiddles<9, FLY>& tq, double2* __restrict__ line, int stride) {
  constexpr int Q = 512, NT = 64 * W, HN = 8 / W;
  static_assert(W == 2 || W == 4 || W == 8, "1024-, 2048- or 4096-point lines");
  if constexpr (PRE) lds_barrier();
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), j = t & 63;
  double2* reg = line + w * Q;
  fft_lines<9, DIR, C, FLY, true, SHARE>(v, j, tq, reg, stride);  // Y_w[j + 64 r] in v[r]
  const int bj = LPs<true>(j);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int r = 0; r < 8; ++r) reg[c * stride + bj + 64 * r] = v[c][r];
  lds_barrier();
  double2 pw[W];
  tw_powers<W, DIR>(wt, pw);
  const int b = LPs<true>(t);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int h = 0; h < HN; ++h) {
      double2 a[W];
#pragma unroll
      for (int q = 0; q < W; ++q) a[q] = line[c * stride + q * Q + b + NT * h];
      for_twiddles<W, DIR, tw_chain<W>()>(pw, [&](int q, double2 wq) { a[q] = w8_mul<DIR>(cmul(a[q], wq), h * q); });
      dft_w<W, DIR>(a);
#pragma unroll
      for (int p = 0; p < W; ++p)  // (an unused output's arithmetic is dead code)
        v[c][h + HN * p] = (PRUNE && prune_slot(h + HN * p)) ? make_double2(0.0, 0.0) : a[p];
    }
}

// fftw_dit (DIR = -1) of z = a + i b, two real signals in the DIF's order,
// with the pair split of the natural-order spectrum (split_pairs) folded
// into the exchange: each wave's sub-spectrum Y_w is split into the two real
// signals' sub-spectra before the radix-W combination,
//   A_w[k] = (Y_w[k] + conj Y_w[Q - k]) / 2,  B_w[k] = (Y_w[k] - conj Y_w[Q - k]) / 2i
//   Â[k + Qp] = Σ_w ω_W^(wp) ω^(wk) A_w[k]   (likewise B̂)
// (conj Z[N - K] is the same combination of conj Y_w[Q - k]), so the split
// costs reads of the mirrored sub-spectra instead of a second exchange.
// emit(c, K, s, Â[K], B̂[K]) for the live K = t + NT s < kc.  v is left
// undefined.  Entry rule as fftw_dit; the line buffer is read on exit.
template <int W, int C, bool FLY = false, bool PRE = false, typename Emit>
__device__ __forceinline__ void fftw_dit_split(double2 (&v)[C][8], int t, int kc, double2 wt,
                                               const Twiddles<9, FLY>& tq, double2* __restrict__ line, int stride,
                                               Emit emit) {
  constexpr int Q = 512, NT = 64 * W, HN = 8 / W, DIR = -1;
  static_assert(W == 2 || W == 4 || W == 8, "1024-, 2048- or 4096-point lines");
  if constexpr (PRE) lds_barrier();
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), j = t & 63;
  double2* reg = line + w * Q;
  fft_lines<9, DIR, C, FLY, true>(v, j, tq, reg, stride);  // Y_w[j + 64 r] in v[r]
  const int bj = LPs<true>(j);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int r = 0; r < 8; ++r) reg[c * stride + bj + 64 * r] = v[c][r];
  lds_barrier();
  double2 pw[W];
  tw_powers<W, DIR>(wt, pw);
#pragma unroll
  for (int h = 0; h < HN; ++h) {
    if (NT * h >= kc) continue;  // no live output K = t + NT h + Q p (uniform)
    const int k = t + NT * h, km = (Q - k) & (Q - 1);
    const int bk = LPs<true>(k), bm = LPs<true>(km);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      double2 A[W], B[W];
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const double2 y = line[c * stride + q * Q + bk], ym = line[c * stride + q * Q + bm];
        A[q] = make_double2(0.5 * (y.x + ym.x), 0.5 * (y.y - ym.y));
        B[q] = make_double2(0.5 * (y.y + ym.y), -0.5 * (y.x - ym.x));
      }
      for_twiddles<W, DIR, tw_chain<W>()>(pw, [&](int q, double2 wq) {
        A[q] = w8_mul<DIR>(cmul(A[q], wq), h * q);
        B[q] = w8_mul<DIR>(cmul(B[q], wq), h * q);
      });
      dft_w<W, DIR>(A);
      dft_w<W, DIR>(B);
#pragma unroll
      for (int p = 0; p < W; ++p)
        if (k + Q * p < kc) emit(c, k + Q * p, h + HN * p, A[p], B[p]);
    }
  }
}

// ---------------------------------------------------------------------------
// 8192-point lines over 1024 threads (16 waves) decimated by 16 across the
// waves, as fftw_dif/fftw_dit above (Q = 512, one wave per sub-transform):
// the radix-16 split as a radix-8 in each thread's registers (spacing 1024)
// and a radix-2 on the way out of the one workgroup-wide exchange.  With
// ω = exp(DIR 2πi/N), N = 8192, wave w = 8e + c, lane j:
//   DIF (natural in: v[s] = x[t + 1024 s] → decimated out):
//     y_c[n] = ω^(nc) Σ_q x[n + 1024 q] ω_8^(qc)            (registers)
//     z_w[m] = (y_c[m] + (-1)^e y_c[m + 512]) ω_1024^(m e)  (after the exchange)
//     X[16 m + w] = DFT_512(z_w)[m]                          (wave-local)
//     on exit lane j of wave w holds X[16 (j + 64 r) + w] in v[r];
//   DIT (that order in → natural out): Y_w = DFT_512(x[16 m + w]),
//     Z_c[k] = Y_c[k mod 512] + ω_1024^k Y_(c+8)[k mod 512], k < 1024,
//     X[k + 1024 q] = Σ_c ω_8^(qc) ω^(kc) Z_c[k]: on exit v[q] = X[t + 1024 q].
// Three workgroup barriers per transform (Stockham: ten).  tab: the
// forward-sign table of length N (W_N^t read per transform, not held);
// tq = Twiddles<9, true>::load(t & 63, tab, 4).  PRE: a barrier before the
// first LDS write.
// ---------------------------------------------------------------------------
// ω_16^u (u < 8), ω_16 = exp(DIR 2πi/16), times a (u a constant once unrolled)
template <int DIR>
__device__ __forceinline__ double2 w16_mul(double2 a, int u) {
  constexpr double c1 = 0.92387953251128675613, s1 = 0.38268343236508977173;
  if (u == 0) return a;
  if (u == 4) return (DIR < 0) ? make_double2(a.y, -a.x) : make_double2(-a.y, a.x);
  if (u == 2 || u == 6) return w8_mul<DIR>(a, u / 2);
  const double cs[8] = {1.0, c1, 0.0, s1, 0.0, -s1, 0.0, -c1};
  const double sn[8] = {0.0, s1, 0.0, c1, 0.0, c1, 0.0, s1};
  return cmul(a, make_double2(cs[u], DIR * sn[u]));
}

template <int DIR, bool PRE = true>
__device__ __forceinline__ void fft16_dif(double2 (&v)[8], int t, const Twiddles<9, true>& tq,
                                          const double2* __restrict__ tab, double2* __restrict__ line) {
  constexpr int NT = 1024, Q = 512;
  asm volatile("" : "+v"(t));
  const double2 wt = tab[t];
  const double2 t8 = tab[8 * (t & 63)];  // ω_1024^j (waves 8-15), issued early
  dft8<DIR>(v);
  {  // ω^(t c), a chain (two powers live)
    const double2 w1 = DIR < 0 ? wt : cconj(wt);
    double2 wp = w1;
#pragma unroll
    for (int c = 1; c < 8; ++c) {
      v[c] = cmul(v[c], wp);
      if (c < 7) wp = cmul(wp, w1);
    }
  }
  if constexpr (PRE) lds_barrier();
  const int b = LPs<true>(t);
#pragma unroll
  for (int c = 0; c < 8; ++c) line[c * NT + b] = v[c];
  lds_barrier();
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), j = t & 63;
  const double2* src = line + (w & 7) * NT + LPs<true>(j);
  if (w < 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = cadd(src[64 * u], src[64 * u + Q]);
  } else {
    const double2 wj = DIR < 0 ? t8 : cconj(t8);
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = w16_mul<DIR>(cmul(csub(src[64 * u], src[64 * u + Q]), wj), u);
  }
  lds_barrier();  // every wave has read its sub-line: the regions are free
  fft_lines<9, DIR, 1, true, true>(reinterpret_cast<double2(&)[1][8]>(v), j, tq, line + w * Q, 0);
}

template <int DIR, bool PRE = true>
__device__ __forceinline__ void fft16_dit(double2 (&v)[8], int t, const Twiddles<9, true>& tq,
                                          const double2* __restrict__ tab, double2* __restrict__ line) {
  constexpr int Q = 512;
  if constexpr (PRE) lds_barrier();
  asm volatile("" : "+v"(t));
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), j = t & 63;
  double2* reg = line + w * Q;
  fft_lines<9, DIR, 1, true, true>(reinterpret_cast<double2(&)[1][8]>(v), j, tq, reg, 0);  // Y_w[j + 64 r]
  const int bj = LPs<true>(j);
#pragma unroll
  for (int r = 0; r < 8; ++r) reg[bj + 64 * r] = v[r];
  const double2 t8 = tab[8 * t], wt = tab[t];  // ω_1024^t (t < 1024), W_N^t: in flight over the barrier
  lds_barrier();
  const double2 wk = DIR < 0 ? t8 : cconj(t8);
  const double2* src = line + LPs<true>(t & (Q - 1));
#pragma unroll
  for (int c = 0; c < 8; ++c) v[c] = cadd(src[c * Q], cmul(src[(c + 8) * Q], wk));
  {
    const double2 w1 = DIR < 0 ? wt : cconj(wt);
    double2 wp = w1;
#pragma unroll
    for (int c = 1; c < 8; ++c) {
      v[c] = cmul(v[c], wp);
      if (c < 7) wp = cmul(wp, w1);
    }
  }
  dft8<DIR>(v);
}

}  // namespace sw
