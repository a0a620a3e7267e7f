// libsw host runtime: context lifecycle, slab decomposition, stepper
// sequencing and the C ABI of include/sw.h.  One HIP stream per context;
// every call that returns data synchronises that stream.  Reference seams
// replaced are cited per function.
#include "sw.h"
#include "sw_internal.hpp"
#include "sw_generic.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>
#include <chrono>

using sw::Geom;
using sw::Phys;

struct KStat {
  const char* name;
  int64_t launches = 0;
  double ms = 0.0;
};

// Device buffers of one slab.  With one slab the two
// phases of each mixed array are the same buffer (mic == mir, mfr == mfc).
struct Slab {
  Geom g{};
  double2* sol = nullptr;                    // compact state, nf fields
  double2* sol2 = nullptr;                   // FilteredAB3: the other state buffer (ping-pong)
  double2* nt1 = nullptr;                    // fsplit: terms 1 and 2 of a split N (k_col_fwd SPLIT)
  double2* nt2 = nullptr;
  double2* hist[3] = {nullptr, nullptr, nullptr};  // FAB3 RHS ring / IFMAB3 N ring
  double2* acc = nullptr;                    // IFMRK4 running stage combination
  double2* nbuf = nullptr;                   // unfused IFMRK4 / sw_calcN: calcN output
  double2* xs = nullptr;                     // stage input / scratch compact
  double2* xs2 = nullptr;                    // ETDRK4: second stage input s₂ (aliases hist[2])
  double* etd = nullptr;                     // ETDRK4: per-mode coefficients [ETD_N][cfield]
  double2* mic = nullptr;                    // calcN inputs, column phase (col_inv / col_step out)
  double2* mir = nullptr;                    // calcN inputs, row phase (row in)
  double2* mfr = nullptr;                    // row outputs, row phase
  double2* mfc = nullptr;                    // row outputs, column phase (col_fwd / col_step in)
  double2* view = nullptr;                   // scratch pointer for collect_full (history slots)
  // aliased-state tracking (sw_config.aliased_state; one slab, 2LQG): the
  // modes the 2/3 rule removes, compact in sw_ctx::ga[r] — region 0 the
  // columns kr >= kc, region 1 the aliased rows of the live columns
  double2* a_sol[2] = {};                    // post-step state there (the reference's prob.sol)
  double2* a_zero[2] = {};                   // zeros: the dealiased pre-update state there
  double2* a_hist[3][2] = {};                // AB3 steppers: N / RHS ring there
  double2* a_acc[2] = {};                    // IFMRK4: running combination there
  double2* a_n[2] = {};                      // IFMRK4: calcN output there
  double2* a_xs[2] = {};                     // stage-input scratch (discarded: calcN dealiases)
  double2* a_xs2[2] = {};                    // ETDRK4: s₂ there
  double* a_etd[2] = {};                     // ETDRK4: the coefficient table there
  double2* a_nbuf[2] = {};                   // this calcN's output there (aliases a_hist or a_n)
  double2* a_mrow = nullptr;                 // row-pass x-spectra kr >= kc of the forward fields
  double2* a_mrow_mem = nullptr;             // its allocation (one slab per process, rank != 0: this
                                             // rank's block only; a_mrow = a_mrow_mem - slab · block)
                                             // (slab 0 owns it; every slab's row pass writes its rows)
  Geom ga[2]{};                              // this slab's aliased regions (alias_geom; region 0 on slab 0)
};

struct sw_ctx {
  sw_config cfg{};
  Phys p{};
  int nf = 0, ninv = 0, nfwd = 0;
  int kmodel = 0;                            // kernel family (MLQG -> QG2)
  int P = 1;                                 // slabs in the decomposition
  bool dist = false;                         // one slab per process (P > 1)
  bool hostx = false;                        // dist with the host-staged exchange hook
  ncclComm_t nccl = nullptr;                 // dist without the hook: RCCL
  char *hsend = nullptr, *hrecv = nullptr;   // pinned staging of the host-staged exchange
  size_t hbytes = 0;
  hipStream_t stream = nullptr;
  // pipelined slab exchange: transposes on a side stream,
  // ordered against the compute stream by events
  hipStream_t comm = nullptr;
  hipEvent_t ev_row = nullptr, ev_join = nullptr;
  hipEvent_t ev_fwd[8] = {}, ev_col[8] = {};
  hipEvent_t ev_chunk[8] = {};               // row chunk k of the last inverse group has arrived
  hipEvent_t ev_rowc[8] = {};                // row chunk k has been transformed (its forward rows written)
  bool overlap = false;                      // pipelined exchange (default: RCCL; SW_OVERLAP=0/1)
  sw_link_model link{};                      // the link probe of sw_create (sw_get_link_model)
  // grids that are not powers of two (MultiLayerQG + FilteredRK4 on
  // 2^a 3^b 5^c points, simulation/MattParameters.jl:8): the generic engine
  // (sw_generic.hpp) on the full-array state in sl[0].sol
  sw::gen::Engine* gen = nullptr;
  int row_chunks = 1;                        // pipelined: row pass in chunks behind the last inverse transposes
  double2 *tw_x = nullptr, *tw_y = nullptr;
  std::vector<Slab> sl;                      // slabs held by this process
  int head = 0;
  bool mixed_valid = false;                  // mir == transposed col_inv(sol) (fused pipeline primed)
  bool fuse_all = false;                     // SW_FUSE_ALL=1: fused pass for every pair (experiments)
  bool fsplit = false;                       // k_col_fwd one term per block, completed by the update
  int fwd_step = -1;                         // use_fwd_step: -1 where measured faster, SW_FWD_STEP=0/1 off/on
  bool stream_state = false;                 // state/history accesses non-temporal (StepPtrs::stream)
  double2* stage = nullptr;                  // full (nkr,nl,nf) staging
  float* stage32 = nullptr;                  // SW_PREC_F32: the caller-precision copy of stage / dflt
  double2* gbuf = nullptr;                   // dist: all-gathered compact slabs
  double2* abuf = nullptr;                   // dist + aliased_state: all-gathered aliased regions
  double* dflt = nullptr;                    // physical staging / reductions
  double* ecols = nullptr;                   // per-column energy sums [global column][SW_NSUM]
  double* esum = nullptr;                    // energy sums / gathered maxima (sw_diag)
  int* flag = nullptr;
  // sw_step's blow-up check folded into the updates (StepPtrs::nan): armed
  // (scan) for the steps of one sw_step / sw_step_record call; sflag[0] is
  // this slab's flag, sflag[1..P] the gathered flags (one slab per process)
  int* sflag = nullptr;
  bool scan = false;
  // one slab per context or every slab in this process: the flag lives in
  // pinned, device-mapped host memory (the updates store 1 there over PCIe,
  // only on a blow-up), so reading it after the steps costs no copy
  int* hflag = nullptr;      // host view
  int* hflag_dev = nullptr;  // device view of the same word
  // FF Diagnostic(kinetic_energy / potential_energy; freq) recorded on the
  // device during sw_step (sw_set_energy_diagnostics)
  int64_t diag_freq = 0, diag_cap = 0, diag_n = 0;
  double* erec = nullptr;                    // records: [rec][SW_NSUM] sums, or (one slab per
                                             // process) [rec][kcl][SW_NSUM] column sums
  std::vector<int64_t> diag_steps;
  std::vector<double> diag_t;
  std::vector<double> esums_host;            // energy sums of the records gathered so far
  int64_t esums_n = 0;                       // records gathered (sw_get_energy_diagnostics)
  // sw_step_record: the last step of the call records into erec1 ([SW_NSUM]
  // sums, or this rank's [kcl][SW_NSUM] column sums)
  bool force_rec = false;
  double* erec1 = nullptr;
  double* erec1_host = nullptr;              // one slab: erec1 is pinned, device-mapped host memory
  // sw_comm_profile: event pairs on the compute stream around every wait for
  // the side stream's transposes (pipelined) or around each transpose run on
  // it (sequential), and the bytes a slab sends to the other slabs
  bool time_waits = false;
  std::vector<hipEvent_t> wev;
  int nwait = 0;
  double xbytes = 0.0;
  double t = 0.0;
  int64_t step = 0;
  int euler_left = 0;                        // sw_reset_history: forward-Euler start-up steps still to run
                                             // (cleared by sw_set_history; the clock does not move it)
  bool alias = false;                        // sw_config.aliased_state
  std::string err;
  // profiling
  bool prof = false;
  std::vector<KStat> stats;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> pev;  // profiled launches: event pairs not yet read (prof_flush)
  std::vector<int> pkid;
  int npev = 0;
  // SW_PROF_COLD=1: before each profiled kernel a read of this 512 MiB buffer
  // evicts L2 and the 256 MiB Infinity Cache, so each kernel reads its inputs
  // from HBM (the cold per-kernel table in bench.py)
  double* cold = nullptr;
  unsigned long long* cold_out = nullptr;
};

thread_local sw::ProfEv sw::prof_ev;  // (sw_internal.hpp, Timer below)

namespace {

int fail(sw_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                 \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return fail(ctx, SW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)

#define NCCLCHK(ctx, expr)                                                               \
  do {                                                                                   \
    ncclResult_t r_ = (expr);                                                            \
    if (r_ != ncclSuccess)                                                               \
      return fail(ctx, SW_E_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_));   \
  } while (0)

#ifndef SW_ROW_SP_DEFAULT
#define SW_ROW_SP_DEFAULT 0
#endif

int ilog2(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return l;
}
bool pow2(int n) { return n > 0 && (n & (n - 1)) == 0; }

// FF getaliasedwavenumbers: 1-based iL = floor((1-af)/2 n) + 1,
// iR = ceil((1+af)/2 n)
void alias_range(int n, double af, int& iL, int& iR) {
  const double L = (1 - af) / 2, R = (1 + af) / 2;
  iL = (int)std::floor(L * n) + 1;
  iR = (int)std::ceil(R * n);
}

// lines per block of the column kernels (Blk<log2ny>::NB in sw_kernels.hip)
int col_lines_per_block(int ny) {
  const int NT = ny / 8;
  return NT >= SW_BLK_THREADS ? 1 : std::min(SW_BLK_THREADS / NT, 32);
}

#ifndef SW_TILE_F4_QG
#define SW_TILE_F4_QG 13
#endif
// geometry of slab s of P
Geom make_geom(const sw_config& k, int P, int s) {
  Geom g{};
  g.nx = k.nx;
  g.ny = k.ny;
  g.log2nx = ilog2(k.nx);
  g.log2ny = ilog2(k.ny);
  g.nkr = k.nx / 2 + 1;
  g.nl = k.ny;
  int iLx, iRx, iLy, iRy;
  alias_range(k.nx, k.aliased_fraction, iLx, iRx);
  alias_range(k.ny, k.aliased_fraction, iLy, iRy);
  g.kc = iLx - 1;
  g.lc = iLy - 1;
  g.lr2 = iRy;
  if (k.aliased_fraction == 0) {
    // FF with aliased_fraction = 0 zeroes only the Nyquist column kr = nx/2
    // (kc = nx/2 above) and the Nyquist row l = -ny/2
    g.lc = k.ny / 2;
    g.lr2 = k.ny / 2 + 1;
  }
  g.Lr = g.lc + (k.ny - g.lr2);
  g.LrP = (g.Lr + 7) / 8 * 8;
  g.Lx = k.Lx;
  g.Ly = k.Ly;
  g.mk = (2 * M_PI / k.Lx * k.nx) / k.nx;
  g.ml = (2 * M_PI / k.Ly * k.ny) / k.ny;
  g.dx = k.Lx / k.nx;
  g.dy = k.Ly / k.ny;
  g.nslab = P;
  g.slab = s;
  if (P == 1) {
    g.kcl = (g.kc + 63) / 64 * 64;  // XCD-aware column mapping needs multiples of 64
  } else {
    const int gran = std::max(8, col_lines_per_block(k.ny));
    g.kcl = ((g.kc + P - 1) / P + gran - 1) / gran * gran;
  }
  g.ntl = g.kcl / 8;
  g.kr0 = s * g.kcl;
  g.kcn = std::max(0, std::min(g.kcl, g.kc - g.kr0));
  g.nyl = k.ny / P;
  g.log2nyl = ilog2(g.nyl);
  g.y0 = s * g.nyl;
  g.cfield = (long long)std::max(g.kcn, 1) * g.LrP;
  g.mfield = (long long)g.kcl * g.ny;
  // inverse mixed-field tiles column-major (sw_internal.hpp mtile_local;
  // SW_TILE_CM=0 selects row-major)
  g.tcm = 1;
  if (const char* e = std::getenv("SW_TILE_CM")) g.tcm = e[0] == '1';
  // forward tiles: lines in column order on one slab (SW_LORD_F; the row
  // pass's closed-form offsets assume it), in row order on several
  // (row-chunked forward transposes, §6); SW_FWD_ORD=1 keeps column order
  int ford = SW_LORD_F;
  if (P > 1) {
    ford = 0;
    if (const char* e = std::getenv("SW_FWD_ORD")) ford = e[0] == '1';
  }
  // forward tiles of 4 columns × 2 rows (fa = 2) where the 2LQG/MultiLayerQG
  // row is the half-length one at 2^SW_TILE_F4_QG points and up: its forward
  // stores then fill 64 B of each line per row, and partial 2×4 lines no
  // longer leave L2 before their four rows meet (config 5: row writes 1.54×
  // -> 1.13× of their bytes, row 1838 -> 1617 µs, the column pass reading
  // them 479 -> 625 µs, +2 % per step; profiles/r04/ab_rowh.md).
  // SW_TILE_FA=1/2 overrides.
  g.fa = 1;
  if ((k.model == SW_MODEL_QG2 || k.model == SW_MODEL_MLQG) && g.log2nx >= SW_TILE_F4_QG) g.fa = 2;
  if (const char* e = std::getenv("SW_TILE_FA")) g.fa = (e[0] == '2') ? 2 : 1;
  // RSW / 2LQG / MultiLayerQG / Thomas–Yamada column inverse with one output
  // per block on short lines, where a one-line block is one or two waves (round 5,
  // DESIGN.md §3d, measured: 512-point lines, and 1024 for Thomas–Yamada);
  // SW_INV_SPLIT=0/1 forces it off/on
  g.isplit = g.log2ny <= (k.model == SW_MODEL_TY ? 10 : 9);
  if (const char* e = std::getenv("SW_INV_SPLIT")) g.isplit = e[0] == '1';
  // the RSW and 2LQG / MultiLayerQG rows in two blocks, Thomas–Yamada's in
  // four (k_row SPLIT), on short rows (round 5);
  // SW_ROW_SPLIT=0/1 forces it off/on
  g.rsplit = g.log2nx <= 9;
  if (const char* e = std::getenv("SW_ROW_SPLIT")) g.rsplit = e[0] == '1';
  // the decimated RSW row over two one-line blocks (k_row_rsw_sp, VERDICT
  // r05 #1); SW_ROW_SP=0/1 forces it off/on
  g.rsp = SW_ROW_SP_DEFAULT;
  if (const char* e = std::getenv("SW_ROW_SP")) g.rsp = e[0] == '1';
  g.fsy = ford ? 1 : g.kcl >> g.fa;
  g.fsk = ford ? g.nyl >> (3 - g.fa) : 1;
  return g;
}

int alloc(sw_ctx* c, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) return fail(c, SW_E_NOMEM, std::string("hipMalloc failed: ") + hipGetErrorString(e));
  e = hipMemsetAsync(*p, 0, bytes, c->stream);
  if (e != hipSuccess) return fail(c, SW_E_HIP, hipGetErrorString(e));
  return 0;
}

std::vector<double2> twiddles(int N) {
  std::vector<double2> tw(N);
  for (int m = 0; m < N; ++m) {
    const long double a = 2.0L * 3.141592653589793238462643383279502884L * (long double)m / (long double)N;
    tw[m] = make_double2((double)std::cos(a), (double)-std::sin(a));
  }
  return tw;
}

// The aliased modes FF's dealias! zeroes as two compact regions
// the mode-wise kernels (k_step_elem, k_energy_cols, k_scatter_modes) walk
// like the live set: r = 0 the columns kr in [kc, nx/2], every row (held by
// slab 0: its y-transforms need every row, which every slab's row pass
// writes into its block of the x-spectra — in one process directly, one slab
// per process through an all-gather per calcN); r = 1 the slab's own live
// columns, rows l in [lc, lr2) (lrow_of(j) = lc + j).
Geom alias_geom(const Geom& g, int r) {
  Geom a = g;
  if (r == 0) {
    a.kr0 = g.kc;
    a.kcn = g.slab == 0 ? g.nkr - g.kc : 0;
    a.lc = g.ny;
    a.lr2 = g.ny;
    a.Lr = g.ny;
  } else {
    a.kr0 = g.kr0;
    a.kcn = g.kcn;
    a.lc = 0;
    a.lr2 = g.lc;
    a.Lr = g.lr2 - g.lc;
  }
  a.kcl = a.kcn;
  a.LrP = (a.Lr + 7) / 8 * 8;
  a.cfield = (long long)std::max(a.kcn, 1) * a.LrP;
  return a;
}

// --- algorithmic bytes per kernel launch ---------------------
// summed over the slabs this process holds; F = live compact field,
// Mc = live mixed field in the column phase, Mr = in the row phase
double live_field_bytes(const Geom& g) { return 16.0 * g.kcn * g.Lr; }
double mixed_col_bytes(const Geom& g) { return 16.0 * g.kcn * g.ny; }
double mixed_row_bytes(const Geom& g) { return 16.0 * g.kc * g.nyl; }

enum KId { K_COLINV = 0, K_ROW, K_COLFWD, K_UPD, K_COLSTEP, K_FWDSTEP, K_XCHG, K_GEN, K_NKERN };
const char* kname[K_NKERN] = {"col_inv", "row", "col_fwd", "update", "col_step", "col_fwd_step", "transpose",
                              "generic_step"};

// state/history bytes of one stepper op per live mode, in live-field units
// (reads + writes; AB3 steady state; IFMRK4 averaged over its four stages)
double op_fields(const sw_ctx* c) {
  // the integrating factors are evaluated per mode, never stored (sw_internal.hpp ExpOf)
  const int nf = c->nf, st = c->cfg.stepper;
  // ETDRK4 stages: 1 u in / n1,acc,s1 out; 2 u in / n2,s2 out; 3 s1,acc,n1,n2
  // in / acc,s2 out; 4 acc in / u out; plus the coefficient planes (real: half
  // a field each) 4, 2, 3, 1
  // FilteredRK4 stages: 1 sol in / acc,x out; 2-3 x,sol,acc in / acc,x out;
  // 4 x,sol,acc in / sol out
  if (st == SW_STEP_FILTERED_RK4) return (3.0 * nf + 5.0 * nf + 5.0 * nf + 4.0 * nf) / 4;
  if (st == SW_STEP_ETDRK4) return (4.0 * nf + 3.0 * nf + 6.0 * nf + 2.0 * nf) / 4 + (2.0 + 1.0 + 1.5 + 0.5) / 4;
  if (st == SW_STEP_FILTERED_AB3) return 3 * nf + 2 * nf;  // sol,R-1,R-2 in; sol,RHS out
  if (st == SW_STEP_IFMAB3) return 3 * nf + 2 * nf;        // sol,N-1,N-2 in; sol,N out
  // stages: 1 u in / acc,x out; 2-3 u,acc in / acc,x out; 4 u,acc in / u out
  return (3.0 * nf + 4.0 * nf + 4.0 * nf + 3.0 * nf) / 4;
}

// fsplit: the fields of N's terms 1-2 that k_col_fwd SPLIT writes to nt1/nt2
// (nterms in sw_kernels.hip: RSW N_v, N_η; 2LQG both layers; TY N_ζ twice,
// N_vc), and the calcN-input fields the update reads for the linear terms
// (MultiLayerQG, Thomas–Yamada)
int split_terms(const sw_ctx* c) { return !c->fsplit ? 0 : (c->kmodel == SW_MODEL_TY ? 3 : 2); }
int split_xin(const sw_ctx* c) {
  return !c->fsplit ? 0 : ((c->cfg.model == SW_MODEL_TY || c->cfg.model == SW_MODEL_MLQG) ? c->nf : 0);
}

// the generic engine's step (one K_GEN scope): SURVEY §8(d)'s model for MLQG
// FilteredRK4 (bench.py b_alg) — per stage 10 logical 2D transforms of
// 16·Ns + 8·Np bytes (6 inverse, 4 forward) and the stage update's 10.5 fields
double gen_step_bytes(const sw_ctx* c) {
  const Geom& g = c->sl[0].g;
  const double Ns = (double)g.nkr * g.nl, Np = (double)g.nx * g.ny;
  return 4 * (10 * (16 * Ns + 8 * Np) + 10.5 * 16 * Ns);
}

double kernel_bytes(const sw_ctx* c, int kid) {
  if (kid == K_GEN) return c->gen ? gen_step_bytes(c) : 0.0;
  double b = 0.0;
  for (const Slab& s : c->sl) {
    const Geom& g = s.g;
    const double F = live_field_bytes(g), Mc = mixed_col_bytes(g), Mr = mixed_row_bytes(g);
    const int nf = c->nf;
    switch (kid) {
      case K_COLINV: b += nf * F + c->ninv * Mc; break;
      case K_ROW: b += (c->ninv + c->nfwd) * Mr; break;
      // fsplit: col_fwd also writes N's terms 1-2 (nt1, nt2);
      // the update reads them and the calcN input (xin) for the linear terms
      case K_COLFWD: b += c->nfwd * Mc + (nf + split_terms(c)) * F; break;
      case K_UPD: {  // + N read; IFMAB3's N already in its history slot is not written again
        const bool n_in_slot = c->cfg.stepper == SW_STEP_IFMAB3 && !c->fsplit;
        b += (op_fields(c) + nf - (n_in_slot ? nf : 0) + split_terms(c) + split_xin(c)) * F;
        break;
      }
      case K_COLSTEP: b += c->nfwd * Mc + op_fields(c) * F + c->ninv * Mc; break;
      case K_FWDSTEP: b += c->nfwd * Mc + op_fields(c) * F; break;  // N never in HBM
      case K_XCHG:  // bytes leaving this slab in one inverse + one forward transpose
        b += (double)(c->ninv + c->nfwd) * (c->P - 1) * g.kcl * g.nyl * 16.0;
        break;
    }
  }
  return b;
}

bool use_fused(const sw_ctx* c);
bool use_fwd_step(const sw_ctx* c);
bool fwd_step_lds(const sw_ctx* c);
static double step_bytes(const sw_ctx* c) {
  const int st = c->cfg.stepper;  // four calcN + update stages per RK4-family step
  const int nstage = (st == SW_STEP_IFMRK4 || st == SW_STEP_ETDRK4 || st == SW_STEP_FILTERED_RK4) ? 4 : 1;
  if (!use_fused(c) && use_fwd_step(c))
    return nstage * (kernel_bytes(c, K_COLINV) + kernel_bytes(c, K_ROW) + kernel_bytes(c, K_FWDSTEP));
  if (!use_fused(c))
    return nstage * (kernel_bytes(c, K_COLINV) + kernel_bytes(c, K_ROW) + kernel_bytes(c, K_COLFWD) +
                     kernel_bytes(c, K_UPD));
  return nstage * (kernel_bytes(c, K_ROW) + kernel_bytes(c, K_COLSTEP));  // primed pipeline
}

constexpr size_t kColdBytes = size_t(512) << 20;
constexpr int kProfPairs = 256;
// Each timed scope's kernels carry an event pair (sw::prof_ev, SW_LAUNCH:
// the dispatches' own start/end timestamps; a scope that launches no kernel,
// and the transposes with their RCCL calls and copies, record the pair as
// stream markers instead); the pairs are read back in batches, when the pool
// is full and at the end of sw_profile_steps.  Marker pairs with a host
// synchronisation per launch (rounds 1-6) put the markers' packets and the
// idle restart into each interval: +2 % against the kernel trace at 2048²,
// +6-9 % under a tracer.
void prof_flush(sw_ctx* c) {
  if (c->npev == 0) return;
  (void)hipEventSynchronize(c->pev[2 * c->npev - 1]);
  for (int i = 0; i < c->npev; ++i) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->pev[2 * i], c->pev[2 * i + 1]);
    c->stats[c->pkid[i]].launches += 1;
    c->stats[c->pkid[i]].ms += ms;
  }
  c->npev = 0;
}
struct Timer {
  sw_ctx* c;
  int kid, i = -1;
  bool marker;
  Timer(sw_ctx* c_, int k, bool marker_ = false) : c(c_), kid(k), marker(marker_) {
    if (!c->prof || c->pev.empty()) return;
    if (c->cold) sw::launch_absmax(c->cold, kColdBytes / sizeof(double), c->cold_out, 0, c->stream);
    if (c->npev == (int)c->pkid.size()) prof_flush(c);
    i = c->npev++;  // (Timers do not nest: one slot per scope)
    c->pkid[i] = kid;
    if (marker) (void)hipEventRecord(c->pev[2 * i], c->stream);
    else sw::prof_ev = {c->pev[2 * i], c->pev[2 * i + 1]};
  }
  ~Timer() {
    if (i < 0) return;
    const bool none = !marker && sw::prof_ev.start;  // no kernel took the pair
    sw::prof_ev = {};
    if (none) (void)hipEventRecord(c->pev[2 * i], c->stream);
    if (marker || none) (void)hipEventRecord(c->pev[2 * i + 1], c->stream);
  }
};

// the compute stream waits for an event of the side stream (sw_comm_profile:
// timed — the span between the two events is comm time the compute stream
// could not hide)
int wait_comm(sw_ctx* c, hipEvent_t ev) {
  const bool tm = c->time_waits && c->nwait + 2 <= (int)c->wev.size();
  if (tm) HIPCHK(c, hipEventRecord(c->wev[c->nwait], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->stream, ev, 0));
  if (tm) {
    HIPCHK(c, hipEventRecord(c->wev[c->nwait + 1], c->stream));
    c->nwait += 2;
  }
  return 0;
}

// The transpose between the column and the row passes: block q
// of every source slab p goes to block p of slab q.  inv: column-phase calcN
// inputs -> row phase; fwd: row outputs -> column phase.  The blocks are
// contiguous in both layouts, so no pack/unpack kernels exist.  Moves the
// listed fields on stream `st` (RCCL: one group of sends/receives).
//
// Rows [r0, r1) of every block (r1 > r0 >= 0: one chunk of the row pass's
// input, or of its output): the inverse fields' lines are row-major 2×4 tiles
// (SW_LORD_I = 0) and so are the forward fields' on several slabs (Geom::fsk
// = 1), so rows [r0, r1) (multiples of 4) of a block are the contiguous
// elements [r0 kcl, r1 kcl) of it in both phases.
int transpose_fields(sw_ctx* c, bool inv, const int* fields, int nfl, hipStream_t st, int r0 = 0, int r1 = -1) {
  if (c->P == 1 || nfl == 0) return 0;
  const Geom& g0 = c->sl[0].g;
  const size_t blk = (size_t)g0.kcl * g0.nyl;  // elements per (slab pair, field)
  const long long MF = g0.mfield;
  if (r1 < 0) r1 = g0.nyl;
  if (r0 != 0 || r1 != g0.nyl) {
    const bool rows_contig = inv ? (SW_TILE_I == 2 && SW_LORD_I == 0) : (SW_TILE_F == 2 && g0.fsk == 1);
    if (!rows_contig || c->hostx || r0 < 0 || r1 > g0.nyl || r0 % 4 || r1 % 4)
      return fail(c, SW_E_INVALID, "row-chunked transpose: row-major tiles, device transports, rows in 4s");
  }
  const size_t off = (size_t)r0 * g0.kcl, cnt = (size_t)(r1 - r0) * g0.kcl;  // within each block
  c->xbytes += (double)nfl * (c->P - 1) * cnt * sizeof(double2);  // one slab's sends to the others
  if (!c->dist) {
    for (int i = 0; i < nfl; ++i) {
      const int o = fields[i];
      for (int p = 0; p < c->P; ++p)
        for (int q = 0; q < c->P; ++q) {
          const double2* src = (inv ? c->sl[p].mic : c->sl[p].mfr) + o * MF + q * blk + off;
          double2* dst = (inv ? c->sl[q].mir : c->sl[q].mfc) + o * MF + p * blk + off;
          HIPCHK(c, hipMemcpyAsync(dst, src, cnt * sizeof(double2), hipMemcpyDeviceToDevice, st));
        }
    }
    return 0;
  }
  const Slab& s = c->sl[0];
  const int me = g0.slab;
  if (c->hostx) {
    // stage [q][field][block] so block q of every field is one contiguous
    // message for rank q (one 2-D copy per field each way)
    const size_t fb = blk * sizeof(double2), rowb = nfl * fb;
    if (rowb * c->P > c->hbytes) return fail(c, SW_E_INVALID, "exchange staging too small");
    for (int i = 0; i < nfl; ++i)
      HIPCHK(c, hipMemcpy2DAsync(c->hsend + i * fb, rowb, (inv ? s.mic : s.mfr) + fields[i] * MF, fb, fb, c->P,
                                 hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (c->cfg.exchange(c->cfg.exchange_user, c->hsend, c->hrecv, rowb, c->P) != 0)
      return fail(c, SW_E_COMM, "exchange hook failed");
    for (int i = 0; i < nfl; ++i)
      HIPCHK(c, hipMemcpy2DAsync((inv ? s.mir : s.mfc) + fields[i] * MF, fb, c->hrecv + i * fb, rowb, fb, c->P,
                                 hipMemcpyHostToDevice, st));
    return 0;
  }
  NCCLCHK(c, ncclGroupStart());
  for (int i = 0; i < nfl; ++i) {
    const double2* src = (inv ? s.mic : s.mfr) + fields[i] * MF;
    double2* dst = (inv ? s.mir : s.mfc) + fields[i] * MF;
    for (int q = 0; q < c->P; ++q) {
      if (q == me) {
        HIPCHK(c, hipMemcpyAsync(dst + me * blk + off, src + me * blk + off, cnt * sizeof(double2),
                                 hipMemcpyDeviceToDevice, st));
      } else {
        NCCLCHK(c, ncclSend(src + q * blk + off, 2 * cnt, ncclDouble, q, c->nccl, st));
        NCCLCHK(c, ncclRecv(dst + q * blk + off, 2 * cnt, ncclDouble, q, c->nccl, st));
      }
    }
  }
  NCCLCHK(c, ncclGroupEnd());
  return 0;
}

// fields [0, nfields) on the compute stream (the sequential schedule)
int transpose(sw_ctx* c, bool inv, int nfields) {
  if (c->P == 1) return 0;
  Timer tm(c, K_XCHG, true);
  int f[16];
  for (int i = 0; i < nfields; ++i) f[i] = i;
  const bool tw = c->time_waits && c->nwait + 2 <= (int)c->wev.size();  // exposed in full
  if (tw) HIPCHK(c, hipEventRecord(c->wev[c->nwait], c->stream));
  if (int rc = transpose_fields(c, inv, f, nfields, c->stream)) return rc;
  if (tw) {
    HIPCHK(c, hipEventRecord(c->wev[c->nwait + 1], c->stream));
    c->nwait += 2;
  }
  return 0;
}

// --- pipelined exchange (P > 1, RCCL or in-process copies) ------------------
// The column pass is launched per field group; each group's transpose runs on
// the side stream while the compute stream transforms the next group:
//  * forward: the row outputs go over in the order the column pass consumes
//    them (fwd_need[f] = the row outputs column field f reads, nterms), and
//    column field f starts as soon as its inputs have arrived;
//  * inverse: the outputs of column group g (inv_out[g]) go over while group
//    g+1 is computed; the row pass waits for the last of them.
// Same kernels, same data, same results as the sequential schedule (tested
// bitwise); only the order of independent work changes.
struct PipeSpec {
  int ninvg, nfc;          // inverse-producing column groups, column fields
  int inv_out[5][3];       // per group: output fields (-1 = none)
  int fwd_need[4][3];      // per column field: forward inputs (-1 = none)
};
const PipeSpec& pipe_spec(int model) {
  // RSW: col_inv/col_step group f -> U,Uy | V | H; N_u <- P, N_v <- K,ζu,
  //      N_η <- Q,vη (k_col_fwd nterms)
  static const PipeSpec rsw = {3, 3, {{0, 3, -1}, {1, -1, -1}, {2, -1, -1}},
                               {{0, -1, -1}, {1, 2, -1}, {3, 4, -1}}};
  // QG2: layer l -> Q_l, Ψ_l, Ψy_l; N_l <- ψx q_l, ψy q_l
  static const PipeSpec qg2 = {2, 2, {{0, 2, 4}, {1, 3, 5}}, {{0, 2, -1}, {1, 3, -1}}};
  // RSW advective form (sw::MODEL_RSWA): U,Uy | V,Vy | H; N_u <- 0, N_v <- 1, N_η <- 2, 3
  static const PipeSpec rswa = {3, 3, {{0, 3, -1}, {1, 4, -1}, {2, -1, -1}}, {{0, -1, -1}, {1, -1, -1}, {2, 3, -1}}};
  if (model == sw::MODEL_RSWA) return rswa;
  // TY: k_col_inv groups and k_col_fwd nterms
  static const PipeSpec ty = {5, 4, {{0, 1, -1}, {2, 3, -1}, {4, 5, -1}, {6, -1, -1}, {7, 8, -1}},
                              {{0, 1, 2}, {3, -1, -1}, {4, 5, -1}, {6, -1, -1}}};
  return model == SW_MODEL_RSW ? rsw : (model == SW_MODEL_TY ? ty : qg2);
}

// (aliased-state tracking runs the sequential calcN, whose last step is the
// aliased modes' column pass)
bool pipelined(const sw_ctx* c) { return c->P > 1 && !c->hostx && c->overlap && !c->prof && !c->alias; }

// after the compute stream has launched the producer of inverse group g.
// The last group goes over in row_chunks chunks of rows, each followed by
// ev_chunk[k]: the row pass of chunk k starts behind it (rows_pipelined)
// while the later chunks are in flight.
int inv_group_async(sw_ctx* c, int g) {
  const PipeSpec& ps = pipe_spec(c->kmodel);
  HIPCHK(c, hipEventRecord(c->ev_col[g], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->comm, c->ev_col[g], 0));
  int f[3], n = 0;
  for (int x : ps.inv_out[g])
    if (x >= 0) f[n++] = x;
  if (g != ps.ninvg - 1 || c->row_chunks <= 1) return transpose_fields(c, true, f, n, c->comm);
  const int per = c->sl[0].g.nyl / c->row_chunks;
  for (int k = 0; k < c->row_chunks; ++k) {
    if (int rc = transpose_fields(c, true, f, n, c->comm, k * per, (k + 1) * per)) return rc;
    HIPCHK(c, hipEventRecord(c->ev_chunk[k], c->comm));
  }
  return 0;
}

// the compute stream waits for everything queued on the side stream
int join_comm(sw_ctx* c) {
  if (!c->comm) return 0;
  HIPCHK(c, hipEventRecord(c->ev_join, c->comm));
  return wait_comm(c, c->ev_join);
}

// the row pass behind the inverse transposes: all at once after the side
// stream has drained, or chunk by chunk behind ev_chunk[k]
int rows_pipelined(sw_ctx* c) {
  if (c->row_chunks <= 1) {
    if (int rc = join_comm(c)) return rc;
    for (Slab& s : c->sl) sw::launch_row(c->kmodel, s.g, c->p, s.mir, s.mfr, c->tw_x, c->stream);
    return 0;
  }
  const int per = c->sl[0].g.nyl / c->row_chunks;
  for (int k = 0; k < c->row_chunks; ++k) {
    if (int rc = wait_comm(c, c->ev_chunk[k])) return rc;
    for (Slab& s : c->sl) sw::launch_row(c->kmodel, s.g, c->p, s.mir, s.mfr, c->tw_x, c->stream, k * per, per);
    HIPCHK(c, hipEventRecord(c->ev_rowc[k], c->stream));
  }
  return 0;
}


// after the compute stream has launched the row pass: forward transposes in
// column-field order, ev_fwd[f] = inputs of column field f have arrived
//
// With the row pass in chunks (row_chunks > 1, rows_pipelined) the forward
// transposes follow it chunk by chunk: chunk k of every forward field goes
// over behind row chunk k (ev_rowc[k]), in column-field order within a chunk,
// while the row pass transforms chunk k+1; ev_fwd[f] follows the last chunk
// of column field f's inputs.
int fwd_async(sw_ctx* c) {
  const PipeSpec& ps = pipe_spec(c->kmodel);
  const int K = (c->row_chunks > 1 && SW_TILE_F == 2 && c->sl[0].g.fsk == 1) ? c->row_chunks : 1;
  if (K <= 1) {
    HIPCHK(c, hipEventRecord(c->ev_row, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->comm, c->ev_row, 0));
  }
  const int per = c->sl[0].g.nyl / K;
  for (int k = 0; k < K; ++k) {
    if (K > 1) HIPCHK(c, hipStreamWaitEvent(c->comm, c->ev_rowc[k], 0));
    bool sent[16] = {};
    for (int fc = 0; fc < ps.nfc; ++fc) {
      int f[3], n = 0;
      for (int x : ps.fwd_need[fc])
        if (x >= 0 && !sent[x]) {
          f[n++] = x;
          sent[x] = true;
        }
      const int rc = K > 1 ? transpose_fields(c, false, f, n, c->comm, k * per, (k + 1) * per)
                           : transpose_fields(c, false, f, n, c->comm);
      if (rc) return rc;
      if (k == K - 1) HIPCHK(c, hipEventRecord(c->ev_fwd[fc], c->comm));
    }
  }
  return 0;
}

sw::StepPtrs step_ptrs(const sw_ctx* c, const Slab& s);
// the last column pass: col_fwd into N, or (op >= 0) the forward transforms
// and the stepper update in one kernel (N never in HBM)
static void last_col_pass(sw_ctx* c, double2* Slab::*X, double2* Slab::*N, int op, int stage, const Slab& s) {
  if (op < 0) {
    sw::launch_col_fwd(c->kmodel, s.g, c->p, s.mfc, s.*N, s.*X, c->tw_y, c->stream, 0, -1, s.nt1, s.nt2);
    return;
  }
  sw::StepPtrs a = step_ptrs(c, s);
  a.stage = stage;
  sw::launch_col_fwd_step(c->kmodel, op, s.g, c->p, a, s.mfc, c->tw_y, c->stream, fwd_step_lds(c));
}

int allgather(sw_ctx* c, const void* mine, void* dst, size_t bytes);
int gather0(sw_ctx* c, const void* mine, void* dst, size_t bytes);
// equation.calcN!(N, X, …): col_inv -> transpose -> row -> transpose -> col_fwd;
// op >= 0: the stepper update of `op` fused into the col_fwd pass (use_fwd_step)
int calcN(sw_ctx* c, double2* Slab::*X, double2* Slab::*N, int op = -1, int stage = 0) {
  const int model = c->kmodel;
  if (c->cfg.nop_calcN) {  // NOPcalcN!: N .= 0 (the aliased modes' N too)
    for (Slab& s : c->sl) {
      HIPCHK(c, hipMemsetAsync(s.*N, 0, (size_t)c->nf * s.g.cfield * sizeof(double2), c->stream));
      if (c->alias)
        for (int r = 0; r < 2; ++r)
          if (s.a_nbuf[r] && s.ga[r].kcn > 0)
            HIPCHK(c, hipMemsetAsync(s.a_nbuf[r], 0, (size_t)c->nf * s.ga[r].cfield * sizeof(double2), c->stream));
    }
    return 0;
  }
  if (pipelined(c)) {
    const PipeSpec& ps = pipe_spec(model);
    for (int g = 0; g < ps.ninvg; ++g) {
      for (Slab& s : c->sl) sw::launch_col_inv(model, s.g, c->p, s.*X, s.mic, c->tw_y, c->stream, g, 1);
      if (int rc = inv_group_async(c, g)) return rc;
    }
    if (int rc = rows_pipelined(c)) return rc;
    if (int rc = fwd_async(c)) return rc;
    if (op >= 0) {  // every field of a column in one block: all exchanges first
      for (int f = 0; f < ps.nfc; ++f)
        if (int rc = wait_comm(c, c->ev_fwd[f])) return rc;
      for (Slab& s : c->sl) last_col_pass(c, X, N, op, stage, s);
      return 0;
    }
    for (int f = 0; f < ps.nfc; ++f) {
      if (int rc = wait_comm(c, c->ev_fwd[f])) return rc;
      for (Slab& s : c->sl)
        sw::launch_col_fwd(model, s.g, c->p, s.mfc, s.*N, s.*X, c->tw_y, c->stream, f, 1, s.nt1, s.nt2);
    }
    return 0;
  }
  {
    Timer tm(c, K_COLINV);
    for (Slab& s : c->sl) sw::launch_col_inv(model, s.g, c->p, s.*X, s.mic, c->tw_y, c->stream);
  }
  if (int rc = transpose(c, true, c->ninv)) return rc;
  {
    Timer tm(c, K_ROW);
    for (Slab& s : c->sl)
      sw::launch_row(model, s.g, c->p, s.mir, s.mfr, c->tw_x, c->stream, 0, -1, c->alias ? c->sl[0].a_mrow : nullptr);
  }
  if (c->alias && c->dist) {  // every rank's block of the aliased x-spectra, for slab 0's region 0 (ma_off)
    const Slab& s = c->sl[0];
    const size_t B = (size_t)c->nfwd * sw::ma_field(s.g);
    if (int rc = gather0(c, s.a_mrow + (size_t)s.g.slab * B, s.a_mrow, B * sizeof(double2))) return rc;
  }
  if (int rc = transpose(c, false, c->nfwd)) return rc;
  {
    Timer tm(c, op >= 0 ? K_FWDSTEP : K_COLFWD);
    for (Slab& s : c->sl) last_col_pass(c, X, N, op, stage, s);
  }
  if (c->alias)  // N at the aliased modes (the reference's calcN! writes them: swqg/TwoLayerQG.jl:171,179)
    for (Slab& s : c->sl)
      for (int r = 0; r < 2; ++r)
        sw::launch_col_fwd_alias(c->kmodel, s.g, s.ga[r], r, c->p, s.mfc, c->sl[0].a_mrow, s.a_nbuf[r], c->tw_y,
                                 c->stream);
  return 0;
}

// one stepforward!(sol, clock, ts, …).  Fused pipeline: the column pass of
// stage s also produces the inverse transforms the row pass of stage s+1
// needs, so a primed step is row -> col_step (two launches).
// The fused column pass is used where it wins (measured): RSW FilteredAB3,
// whose update splits by field.  Other model/stepper pairs run the separate
// col_inv / row / col_fwd / update kernels: their update couples the fields
// at a mode, and both one block per column holding every field (k_col_step,
// SW_FUSE_ALL) and a per-(column, field group) update + inverse kernel that
// re-evaluates the coupled update in every group measured slower at 2048²
// than the separate kernels.
bool use_fused(const sw_ctx* c) {
  // aliased-state tracking runs the separate column passes (k_col_fwd_alias
  // and the aliased updates follow k_col_fwd): never the fused pass
  if (c->cfg.unfused || c->cfg.nop_calcN || c->cfg.model == SW_MODEL_TY || c->cfg.model == SW_MODEL_MLQG ||
      c->cfg.stepper == SW_STEP_FILTERED_RK4 || c->kmodel == sw::MODEL_RSWA || c->alias)
    return false;
  if (c->fuse_all) return true;
  return c->kmodel == SW_MODEL_RSW && c->cfg.stepper == SW_STEP_FILTERED_AB3;
}

// k_col_fwd + k_step_elem as one column pass (k_col_step<…, INV = false>: one
// block per column, every field's N in registers, the update at each live
// mode, no N in HBM); the next calcN's col_inv runs separately.  Built for
// RSW IFMAB3/IFMRK4, 2LQG FilteredAB3/IFMAB3/IFMRK4 and (round 5) MultiLayerQG
// FilteredRK4, whose N adds k_col_fwd's terms from the calcN input
// (mlqg_linear_terms, read per mode beside the update), bitwise equal to the
// two kernels; used where it wins (tools/ab/fwdstep_ab.sh): 2LQG
// FilteredAB3 on lines up to 2048 points (0 spills; 5409 -> 5601 steps/s at
// 2048²).  The coupled IF/RK4 updates hold every field's N next to the
// per-mode exponential and spill (82-180 VGPRs at 2048, 350+ at 8192): 2LQG
// IFMAB3 2048² 5279 -> 4127, RSW IFMAB3 5358 -> 3916, 2LQG IFMRK4 8192² 62.5
// -> 44.9.  SW_FWD_STEP=1 forces it on every built pair, =0 off.
bool use_fwd_step(const sw_ctx* c) {
  if (c->fwd_step == 0 || c->cfg.unfused || c->cfg.nop_calcN || use_fused(c) || c->alias) return false;
  const int m = c->cfg.model, st = c->cfg.stepper;
  const bool built = (c->kmodel == SW_MODEL_RSW && (st == SW_STEP_IFMAB3 || st == SW_STEP_IFMRK4)) ||
                     (m == SW_MODEL_QG2 && (st == SW_STEP_FILTERED_AB3 || st == SW_STEP_IFMAB3 ||
                                            st == SW_STEP_IFMRK4)) ||
                     (m == SW_MODEL_MLQG && st == SW_STEP_FILTERED_RK4);
  if (!built) return false;
  if (c->fwd_step == 1) return true;
  if (c->fwd_step == 2) return fwd_step_lds(c);
  return m == SW_MODEL_QG2 && st == SW_STEP_FILTERED_AB3 && c->sl[0].g.log2ny <= 11;
}
// the LDS-parked variant (k_col_fwd_step_lds, SW_FWD_STEP=2) where its
// line buffer and parked N fit one CU's 160 KB.  (MultiLayerQG FilteredRK4,
// round 5: its register variant spills 16-34 VGPRs at 512-2048, the LDS one
// none; against the separate kernels the LDS one measured 5845-6348 vs
// 6473-6726 steps/s at 512², 3530-3563 vs 3404-3418 at 1024², 752-755 vs
// 758-761 at 2048²: off by default)
bool fwd_step_lds(const sw_ctx* c) {
  return c->fwd_step == 2 && sw::fwd_step_lds_bytes(c->kmodel, c->sl[0].g) <= 160 * 1024;
}

// aliased-state tracking: this calcN's output at the aliased modes
void set_alias_nbuf(sw_ctx* c) {
  if (!c->alias) return;
  const int st = c->cfg.stepper;
  const bool sep = st == SW_STEP_IFMRK4 || st == SW_STEP_ETDRK4 || st == SW_STEP_FILTERED_RK4;  // N into its own buffer
  for (Slab& s : c->sl)
    for (int r = 0; r < 2; ++r) s.a_nbuf[r] = sep ? s.a_n[r] : s.a_hist[c->head][r];
}

sw::StepPtrs alias_step_ptrs(const sw_ctx* c, const Slab& s, int r) {
  sw::StepPtrs a{};
  a.sol = s.a_zero[r];
  a.sol_out = s.a_sol[r];
  a.xs = s.a_xs[r];
  a.euler = (c->step < 3 || c->euler_left > 0) ? 1 : 0;
  a.stream = 0;
  if (c->cfg.stepper == SW_STEP_IFMRK4 || c->cfg.stepper == SW_STEP_FILTERED_RK4) {
    a.h0 = s.a_acc[r];
  } else if (c->cfg.stepper == SW_STEP_ETDRK4) {
    a.h0 = s.a_acc[r];
    a.n1 = s.a_hist[0][r];
    a.n2 = s.a_hist[1][r];
    a.xs2 = s.a_xs2[r];
    a.etd = s.a_etd[r];
  } else {
    a.h0 = s.a_hist[c->head][r];
    a.h1 = s.a_hist[(c->head + 2) % 3][r];
    a.h2 = s.a_hist[(c->head + 1) % 3][r];
  }
  return a;
}

sw::StepPtrs step_ptrs(const sw_ctx* c, const Slab& s) {
  const int st = c->cfg.stepper;
  sw::StepPtrs a{};
  a.sol = s.sol;
  a.sol_out = (st == SW_STEP_FILTERED_AB3) ? s.sol2 : s.sol;
  a.xs = s.xs;
  a.euler = (c->step < 3 || c->euler_left > 0) ? 1 : 0;
  a.stream = c->stream_state ? 1 : 0;
  a.nan = c->scan ? (c->hflag ? c->hflag_dev : c->sflag) : nullptr;
  if (st == SW_STEP_IFMRK4 || st == SW_STEP_FILTERED_RK4) {
    a.h0 = s.acc;
  } else if (st == SW_STEP_ETDRK4) {
    a.h0 = s.acc;
    a.n1 = s.hist[0];
    a.n2 = s.hist[1];
    a.xs2 = s.xs2;
    a.etd = s.etd;
  } else {
    a.h0 = s.hist[c->head];
    a.h1 = s.hist[(c->head + 2) % 3];
    a.h2 = s.hist[(c->head + 1) % 3];
  }
  return a;
}

int run_stage(sw_ctx* c, int op, int stage, double2* Slab::*X) {
  const int model = c->kmodel;
  if (use_fused(c) && pipelined(c) && model == SW_MODEL_RSW && op == sw::OP_FAB3) {
    const PipeSpec& ps = pipe_spec(model);
    if (!c->mixed_valid) {
      for (int g = 0; g < ps.ninvg; ++g) {
        for (Slab& s : c->sl) sw::launch_col_inv(model, s.g, c->p, s.*X, s.mic, c->tw_y, c->stream, g, 1);
        if (int rc = inv_group_async(c, g)) return rc;
      }
    }
    if (int rc = rows_pipelined(c)) return rc;
    if (int rc = fwd_async(c)) return rc;
    for (int f = 0; f < ps.nfc; ++f) {  // column field f -> inverse group f
      if (int rc = wait_comm(c, c->ev_fwd[f])) return rc;
      for (Slab& s : c->sl) {
        sw::StepPtrs a = step_ptrs(c, s);
        a.stage = stage;
        sw::launch_col_step(model, op, s.g, c->p, a, s.mfc, s.mic, c->tw_y, c->stream, f, 1);
      }
      if (int rc = inv_group_async(c, f)) return rc;
    }
    c->mixed_valid = true;  // mir receives the next stage's inverse transforms (joined before use)
    return 0;
  }
  if (use_fused(c)) {
    if (!c->mixed_valid) {
      {
        Timer tm(c, K_COLINV);
        for (Slab& s : c->sl) sw::launch_col_inv(model, s.g, c->p, s.*X, s.mic, c->tw_y, c->stream);
      }
      if (int rc = transpose(c, true, c->ninv)) return rc;
    }
    {
      Timer tm(c, K_ROW);
      for (Slab& s : c->sl) sw::launch_row(model, s.g, c->p, s.mir, s.mfr, c->tw_x, c->stream);
    }
    if (int rc = transpose(c, false, c->nfwd)) return rc;
    {
      Timer tm(c, K_COLSTEP);
      for (Slab& s : c->sl) {
        sw::StepPtrs a = step_ptrs(c, s);
        a.stage = stage;
        sw::launch_col_step(model, op, s.g, c->p, a, s.mfc, s.mic, c->tw_y, c->stream);
      }
    }
    if (int rc = transpose(c, true, c->ninv)) return rc;
    c->mixed_valid = true;  // mir now holds the next stage's inverse transforms
  } else {
    // AB3 steppers: calcN writes straight into this step's history slot, which
    // the update then overwrites in place (N -> RHS or N); nbuf aliases it
    if (op != sw::OP_RK4 && op != sw::OP_ETDRK4 && op != sw::OP_FRK4)
      for (Slab& s : c->sl) s.nbuf = s.hist[c->head];
    set_alias_nbuf(c);
    if (use_fwd_step(c)) {
      if (int rc = calcN(c, X, &Slab::nbuf, op, stage)) return rc;
      c->mixed_valid = false;
      return 0;
    }
    if (int rc = calcN(c, X, &Slab::nbuf)) return rc;
    Timer tm(c, K_UPD);
    for (Slab& s : c->sl) {
      sw::StepPtrs a = step_ptrs(c, s);
      a.stage = stage;
      a.nt1 = s.nt1;  // (fsplit: N's terms 1-2, summed with the linear terms per mode)
      a.nt2 = s.nt2;
      a.xin = s.*X;
      sw::launch_step_elem(c->nf, op, s.g, c->p, a, s.nbuf, s.xs, c->stream);
      // the same update at the aliased modes, from the zero (dealiased) state:
      // the post-step values the reference's update writes there
      // (utils/IFMAB3.jl:142-160; filter after).  NOPcalcN!
      // (rsw/RotatingShallowWater.jl:135) dealiases nothing, so there the
      // update starts from the aliased modes' own values: a copy of them in
      // the zero buffer (not in place: the FilteredAB3 matvec couples fields)
      for (int r = 0; c->alias && r < 2; ++r) {
        if (s.ga[r].kcn <= 0) continue;
        const size_t cb = (size_t)c->nf * s.ga[r].cfield * sizeof(double2);
        if (c->cfg.nop_calcN) HIPCHK(c, hipMemcpyAsync(s.a_zero[r], s.a_sol[r], cb, hipMemcpyDeviceToDevice, c->stream));
        sw::StepPtrs b = alias_step_ptrs(c, s, r);
        b.stage = stage;
        sw::launch_step_elem(c->nf, op, s.ga[r], c->p, b, s.a_nbuf[r], s.a_xs[r], c->stream);
        if (c->cfg.nop_calcN) HIPCHK(c, hipMemsetAsync(s.a_zero[r], 0, cb, c->stream));
        // FilteredRK4 adds L·x of the stage input x, which the reference's
        // next calcN! has dealiased in place (zero here) before
        // addlinearterm! reads it: the stage input there is discarded
        if (op == sw::OP_FRK4 && stage < 4) HIPCHK(c, hipMemsetAsync(s.a_xs[r], 0, cb, c->stream));
      }
    }
    c->mixed_valid = false;
  }
  return 0;
}

// aliased-state energies: 2LQG's, Thomas–Yamada's and MultiLayerQG's energy
// functions read the full post-step array (RSW's the dealiased vars.uh)
bool alias_energy(const sw_ctx* c) {
  return c->alias && (c->cfg.model == SW_MODEL_QG2 || c->cfg.model == SW_MODEL_TY || c->cfg.model == SW_MODEL_MLQG);
}

// The state FF's energy diagnostics read after a step: RSW's
// kinetic_energy(prob)/potential_energy(prob) read vars.uh/vh/ηh, which the
// step's last calcN set from its (dealiased) input (rsw/RotatingShallowWater.jl
// :147-149, 323-333): the pre-update state (FilteredAB3, IFMAB3) or the
// stage-4 input (IFMRK4).  2LQG's recompute from prob.sol (swqg/TwoLayerQG.jl
// :230-252), the post-update state.
// aliased-state tracking: the post-step state's aliased modes add their column
// sums after the ncols live ones (a full-array parsevalsum, in a fixed order);
// returns the column count
int alias_energy_cols(sw_ctx* c, bool post_step_state, int ncols) {
  // 2LQG energies read prob.sol (the post-step state); RSW's read vars.uh,
  // the dealiased calcN input (rsw/RotatingShallowWater.jl:323-333)
  // (Thomas–Yamada's read prob.sol too: thomasyamada/ThomasYamada.jl:333-360)
  // (GF MultiLayerQG.energies: qh = sol, the full array)
  if (!c->alias || !post_step_state || !alias_energy(c)) return ncols;
  // region 0 (slab 0), then every slab's region 1 in slab order: the global
  // column order, whatever the decomposition (bitwise the same sums)
  for (int r = 0; r < 2; ++r)
    for (Slab& s : c->sl) {
      if (s.ga[r].kcn <= 0) continue;
      sw::launch_energy_cols(c->cfg.model, s.ga[r], c->p, s.a_sol[r], c->ecols + SW_NSUM * (size_t)ncols, c->stream);
      ncols += s.ga[r].kcn;
    }
  return ncols;
}

// energy columns of one rank's record (one slab per process): the kcl live
// columns, then (alias_energy) region 0's nkr - kc columns (slab 0; zeros on
// the others) and the slab's region 1 padded to kcl columns
size_t rank_cols(const sw_ctx* c) {
  const Geom& g = c->sl[0].g;
  return (size_t)g.kcl + (alias_energy(c) ? (size_t)(g.nkr - g.kc) + g.kcl : 0);
}
// one record's sums from every rank's columns (rank q's at all + q * per +
// off), added in the undecomposed run's global column order — the live
// columns, region 0, every slab's region 1 — so bitwise the same for any
// decomposition (padding columns hold zeros)
void sum_rank_cols(const sw_ctx* c, const double* all, size_t per, size_t off, double* sums) {
  const Geom& g = c->sl[0].g;
  const size_t kcl = g.kcl, na = (size_t)(g.nkr - g.kc);
  for (int k = 0; k < SW_NSUM; ++k) {
    double acc = 0.0;
    for (int q = 0; q < c->P; ++q)
      for (size_t col = 0; col < kcl; ++col) acc += all[q * per + off + col * SW_NSUM + k];
    if (alias_energy(c)) {
      for (size_t col = 0; col < na; ++col) acc += all[off + (kcl + col) * SW_NSUM + k];
      for (int q = 0; q < c->P; ++q)
        for (size_t col = 0; col < kcl; ++col) acc += all[q * per + off + (kcl + na + col) * SW_NSUM + k];
    }
    sums[k] = acc;
  }
}

// one energy record of state X into dst: the sums [SW_NSUM], or (one slab per
// process) this rank's column sums [rank_cols][SW_NSUM], added over ranks at
// retrieval
void record_energy_to(sw_ctx* c, double2* Slab::*X, double* dst) {
  if (c->gen) {
    sw::gen::energy_sums(c->gen, c->sl[0].*X, dst);
    return;
  }
  if (c->dist) {
    const Slab& s = c->sl[0];
    sw::launch_energy_cols(c->cfg.model, s.g, c->p, s.*X, dst, c->stream);
    if (alias_energy(c)) {
      const size_t na = (size_t)(s.g.nkr - s.g.kc);
      double* d0 = dst + SW_NSUM * (size_t)s.g.kcl;
      (void)hipMemsetAsync(d0, 0, SW_NSUM * (na + s.g.kcl) * sizeof(double), c->stream);
      if (X == &Slab::sol)  // (the post-step state, as alias_energy_cols)
        for (int r = 0; r < 2; ++r)
          if (s.ga[r].kcn > 0)
            sw::launch_energy_cols(c->cfg.model, s.ga[r], c->p, s.a_sol[r], d0 + (r ? SW_NSUM * na : 0), c->stream);
    }
    return;
  }
  for (Slab& s : c->sl) sw::launch_energy_cols(c->cfg.model, s.g, c->p, s.*X, c->ecols + SW_NSUM * s.g.kr0, c->stream);
  const int ncols = alias_energy_cols(c, X == &Slab::sol, c->P * c->sl[0].g.kcl);
  sw::launch_energy_final(c->ecols, ncols, dst, c->stream);
}

// the records of this step: the scheduled one (sw_set_energy_diagnostics)
// and/or the forced one (sw_step_record)
void record_energy(sw_ctx* c, double2* Slab::*X, bool rec, bool frec) {
  if (rec)
    record_energy_to(c, X, c->erec + (c->dist ? (size_t)c->diag_n * rank_cols(c) * SW_NSUM : SW_NSUM * c->diag_n));
  if (frec) record_energy_to(c, X, c->erec1);
}

// the generic engine's step (FilteredRK4, MultiLayerQG): its four stages, then
// the records of a MultiLayerQG step (prob.sol after the step)
int gen_step_once(sw_ctx* c) {
  const bool rec = c->diag_freq > 0 && (c->step + 1) % c->diag_freq == 0 && c->diag_n < c->diag_cap;
  const bool frec = c->force_rec;
  {
    Timer tm(c, K_GEN);
    sw::gen::step(c->gen, c->scan ? (c->hflag ? c->hflag_dev : c->sflag) : nullptr);
  }
  HIPCHK(c, hipGetLastError());
  c->t += c->cfg.dt;
  c->step += 1;
  record_energy(c, &Slab::sol, rec, frec);
  if (rec) {
    c->diag_steps.push_back(c->step);
    c->diag_t.push_back(c->t);
    c->diag_n += 1;
  }
  return 0;
}

int step_once(sw_ctx* c) {
  if (c->gen) return gen_step_once(c);
  const int st = c->cfg.stepper;
  const bool rec = c->diag_freq > 0 && (c->step + 1) % c->diag_freq == 0 && c->diag_n < c->diag_cap;
  const bool frec = c->force_rec;
  const bool rsw = c->cfg.model == SW_MODEL_RSW;
  if ((rec || frec) && rsw && st == SW_STEP_IFMAB3) record_energy(c, &Slab::sol, rec, frec);  // updated in place below
  if (st == SW_STEP_FILTERED_AB3 || st == SW_STEP_IFMAB3) {
    if (int rc = run_stage(c, st == SW_STEP_FILTERED_AB3 ? sw::OP_FAB3 : sw::OP_IFMAB3, 0, &Slab::sol))
      return rc;
    c->head = (c->head + 1) % 3;  // RHS₋₂ <- RHS₋₁ <- RHS by rotation (utils/IFMAB3.jl:165-166)
    if (st == SW_STEP_FILTERED_AB3)
      for (Slab& s : c->sl) std::swap(s.sol, s.sol2);
  } else if (st == SW_STEP_FILTERED_RK4) {  // FF RK4substeps! + RK4update! + filter
    for (int stage = 1; stage <= 4; ++stage)
      if (int rc = run_stage(c, sw::OP_FRK4, stage, stage == 1 ? &Slab::sol : &Slab::xs)) return rc;
  } else if (st == SW_STEP_ETDRK4) {  // FF ETDRK4substeps! + ETDRK4update!
    for (int stage = 1; stage <= 4; ++stage)
      if (int rc = run_stage(c, sw::OP_ETDRK4, stage,
                             stage == 1 ? &Slab::sol : (stage == 2 ? &Slab::xs : &Slab::xs2)))
        return rc;
  } else {  // IFMRK4
    for (int stage = 1; stage <= 4; ++stage)
      if (int rc = run_stage(c, sw::OP_RK4, stage, stage == 1 ? &Slab::sol : &Slab::xs)) return rc;
  }
  c->t += c->cfg.dt;
  c->step += 1;
  if (c->euler_left > 0) c->euler_left -= 1;
  if (rsw && st == SW_STEP_FILTERED_AB3) record_energy(c, &Slab::sol2, rec, frec);  // the pre-update buffer
  else if (rsw && (st == SW_STEP_IFMRK4 || st == SW_STEP_FILTERED_RK4))
    record_energy(c, &Slab::xs, rec, frec);  // stage-4 input
  else if (!rsw) record_energy(c, &Slab::sol, rec, frec);
  if (rec) {
    c->diag_steps.push_back(c->step);
    c->diag_t.push_back(c->t);
    c->diag_n += 1;
  }
  return 0;
}

size_t full_bytes(const sw_ctx* c) {
  const Geom& g = c->sl[0].g;
  return (size_t)c->nf * g.nkr * g.nl * sizeof(double2);
}

// caller buffers hold fp64 or (SW_PREC_F32) fp32 elements: the caller's size
// of a buffer whose fp64 size is f64_bytes
size_t caller_bytes(const sw_ctx* c, size_t f64_bytes) {
  return c->cfg.precision == SW_PREC_F32 ? f64_bytes / 2 : f64_bytes;
}

// host buffer in the caller's precision -> fp64 device array (f64_bytes)
int upload(sw_ctx* c, const void* host, void* dst, size_t f64_bytes) {
  if (c->cfg.precision != SW_PREC_F32) {
    HIPCHK(c, hipMemcpyAsync(dst, host, f64_bytes, hipMemcpyHostToDevice, c->stream));
    return 0;
  }
  const long long n = (long long)(f64_bytes / sizeof(double));
  HIPCHK(c, hipMemcpyAsync(c->stage32, host, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
  sw::launch_widen(c->stage32, static_cast<double*>(dst), n, c->stream);
  HIPCHK(c, hipGetLastError());
  return 0;
}

// fp64 device array (f64_bytes) -> host buffer in the caller's precision
int download(sw_ctx* c, const void* src, void* host, size_t f64_bytes) {
  if (c->cfg.precision != SW_PREC_F32) {
    HIPCHK(c, hipMemcpyAsync(host, src, f64_bytes, hipMemcpyDeviceToHost, c->stream));
    return 0;
  }
  const long long n = (long long)(f64_bytes / sizeof(double));
  sw::launch_narrow(static_cast<const double*>(src), c->stage32, n, c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(host, c->stage32, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  return 0;
}

// columns of the full (nkr, nl) array written by slab q's scatter
void scatter_cols(const Geom& g, int& lo, int& hi) {
  lo = std::min(g.kr0, g.nkr);
  hi = (g.slab == g.nslab - 1) ? g.nkr : std::min(g.kr0 + g.kcl, g.nkr);
}

// dist: every rank's `bytes` at `mine` -> dst[rank * bytes] on every rank
// (in place allowed: mine == dst + rank * bytes)
int allgather(sw_ctx* c, const void* mine, void* dst, size_t bytes) {
  if (!c->hostx) {
    NCCLCHK(c, ncclAllGather(mine, dst, bytes, ncclUint8, c->nccl, c->stream));
    return 0;
  }
  if (bytes * c->P > c->hbytes) return fail(c, SW_E_INVALID, "exchange staging too small");
  HIPCHK(c, hipMemcpyAsync(c->hsend, mine, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int q = 1; q < c->P; ++q) std::memcpy(c->hsend + q * bytes, c->hsend, bytes);
  if (c->cfg.exchange(c->cfg.exchange_user, c->hsend, c->hrecv, bytes, c->P) != 0)
    return fail(c, SW_E_COMM, "exchange hook failed");
  HIPCHK(c, hipMemcpyAsync(dst, c->hrecv, bytes * c->P, hipMemcpyHostToDevice, c->stream));
  return 0;
}

// dist: every rank's `bytes` at `mine` -> dst[rank * bytes] on rank 0 only
// (mine == dst + rank * bytes; on the other ranks dst holds their block
// alone).  The aliased-state x-spectra of the row pass feed slab 0's
// region-0 column pass alone (the aliased columns kr >= kc live there): RCCL
// grouped send/recv moves (P - 1) blocks into rank 0 instead of the
// all-gather's P (P - 1).  The host-staged twin
// (VERDICT r05 #4a) routes the same way: each rank's block goes in the send
// slot of rank 0 only, and only rank 0 copies what it receives, so the CPU
// and single-GPU multi-process tests run this routing, not an all-gather.
int gather0(sw_ctx* c, const void* mine, void* dst, size_t bytes) {
  const bool root = c->sl[0].g.slab == 0;  // one slab per process: the slab index is the rank
  if (c->hostx) {
    if (bytes * c->P > c->hbytes) return fail(c, SW_E_INVALID, "exchange staging too small");
    HIPCHK(c, hipMemcpyAsync(c->hsend, mine, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // (an all-to-all of equal blocks: slots 1..P-1 go to ranks that drop them)
    if (c->cfg.exchange(c->cfg.exchange_user, c->hsend, c->hrecv, bytes, c->P) != 0)
      return fail(c, SW_E_COMM, "exchange hook failed");
    if (root)
      HIPCHK(c, hipMemcpyAsync(static_cast<char*>(dst) + bytes, c->hrecv + bytes, bytes * (c->P - 1),
                               hipMemcpyHostToDevice, c->stream));
    return 0;
  }
  NCCLCHK(c, ncclGroupStart());
  if (root) {
    for (int q = 1; q < c->P; ++q)
      NCCLCHK(c, ncclRecv(static_cast<char*>(dst) + q * bytes, bytes, ncclUint8, q, c->nccl, c->stream));
  } else {
    NCCLCHK(c, ncclSend(mine, bytes, ncclUint8, 0, c->nccl, c->stream));
  }
  NCCLCHK(c, ncclGroupEnd());
  return 0;
}

// c->stage <- the full (nkr, nl, nf) array of the per-slab compact field set
int collect_full(sw_ctx* c, double2* Slab::*X) {
  if (c->gen) {  // the generic engine's state is the full array already
    HIPCHK(c, hipMemcpyAsync(c->stage, c->sl[0].*X, full_bytes(c), hipMemcpyDeviceToDevice, c->stream));
    return 0;
  }
  if (!c->dist) {
    for (Slab& s : c->sl) {
      int lo, hi;
      scatter_cols(s.g, lo, hi);
      sw::launch_scatter(c->nf, s.g, lo, hi, s.*X, c->stage, c->stream);
    }
    HIPCHK(c, hipGetLastError());
    return 0;
  }
  // RCCL: all-gather every slab's compact fields, padded to kcl columns
  const Slab& s = c->sl[0];
  const size_t fpad = (size_t)s.g.kcl * s.g.LrP, slot = (size_t)c->nf * fpad;
  double2* mine = c->gbuf + (size_t)s.g.slab * slot;
  for (int f = 0; f < c->nf; ++f)
    HIPCHK(c, hipMemcpyAsync(mine + f * fpad, s.*X + f * s.g.cfield, s.g.cfield * sizeof(double2),
                             hipMemcpyDeviceToDevice, c->stream));
  if (int rc = allgather(c, mine, c->gbuf, slot * sizeof(double2))) return rc;
  for (int q = 0; q < c->P; ++q) {
    Geom gq = make_geom(c->cfg, c->P, q);
    gq.cfield = (long long)fpad;
    int lo, hi;
    scatter_cols(gq, lo, hi);
    sw::launch_scatter(c->nf, gq, lo, hi, c->gbuf + (size_t)q * slot, c->stage, c->stream);
  }
  HIPCHK(c, hipGetLastError());
  return 0;
}

// the OR over every slab of the device flag f[0] (f[1..P]: the gathered
// flags, one slab per process); synchronises the stream
int read_flag(sw_ctx* c, int* f, int& h) {
  std::vector<int> all(c->P + 1, 0);
  const int n = c->dist ? c->P : 1;
  if (c->dist)
    if (int rc = allgather(c, f, f + 1, sizeof(int))) return rc;
  HIPCHK(c, hipMemcpyAsync(all.data(), c->dist ? f + 1 : f, n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  h = 0;
  for (int i = 0; i < n; ++i) h |= all[i];
  return 0;
}

// NaN/Inf anywhere in the live modes of the state: a pass over it (sw_diag)
int nan_flag(sw_ctx* c, int& h) {
  HIPCHK(c, hipMemsetAsync(c->flag, 0, sizeof(int), c->stream));
  if (c->gen) sw::gen::nan_scan(c->gen, c->sl[0].sol, c->flag);
  else
    for (Slab& s : c->sl) sw::launch_nan_check(c->nf, s.g, s.sol, c->flag, c->stream);
  HIPCHK(c, hipGetLastError());
  return read_flag(c, c->flag, h);
}

// sw_step's check (rsw/RSWDriver.jl:213-218) without the pass: the updates of
// the steps between scan_arm and scan_read flag any non-finite value they
// store into the state (StepPtrs::nan).  A non-finite value in a step's new
// state reaches every mode of the next (the transforms spread it), so this
// flags exactly the step blocks whose final state the pass would have
// flagged, and fails loudly on an intermediate one too.
int scan_arm(sw_ctx* c) {
  c->scan = c->cfg.check_nan != 0;
  if (!c->scan) return 0;
  if (c->hflag)
    *c->hflag = 0;  // (every earlier step has completed: sw_step / sw_step_record end synchronised)
  else
    HIPCHK(c, hipMemsetAsync(c->sflag, 0, sizeof(int), c->stream));
  return 0;
}
int scan_read(sw_ctx* c, int& h) {
  c->scan = false;
  if (!c->hflag) return read_flag(c, c->sflag, h);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  h = *reinterpret_cast<volatile int*>(c->hflag);
  return 0;
}

// --- the link probe (sw_get_link_model, VERDICT r05 #4b-c) ---------------
// one exchange of m bytes per peer — every peer (shift 0) or one peer at a
// time (send to rank + shift, receive from rank - shift) — through the
// context's transport: RCCL grouped send/recv on the compute stream, timed by
// events, or the host hook (an all-to-all; wall clock).  The payload is
// whatever the mixed-field buffers / staging hold (no state exists yet).
int probe_round(sw_ctx* c, size_t m, int shift, double& us) {
  Slab& s = c->sl[0];
  const int r = s.g.slab, P = c->P;
  if (c->hostx) {
    const auto t0 = std::chrono::steady_clock::now();
    if (c->cfg.exchange(c->cfg.exchange_user, c->hsend, c->hrecv, m, P) != 0)
      return fail(c, SW_E_COMM, "exchange hook failed");
    us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    return 0;
  }
  char* snd = reinterpret_cast<char*>(s.mic);
  char* rcv = reinterpret_cast<char*>(s.mfr);
  const int to = (r + shift) % P, from = (r - shift + P) % P;
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  NCCLCHK(c, ncclGroupStart());
  for (int q = 0; q < P; ++q) {
    if (q == r) continue;
    if (shift == 0 || q == to) NCCLCHK(c, ncclSend(snd + q * m, m, ncclUint8, q, c->nccl, c->stream));
    if (shift == 0 || q == from) NCCLCHK(c, ncclRecv(rcv + q * m, m, ncclUint8, q, c->nccl, c->stream));
  }
  NCCLCHK(c, ncclGroupEnd());
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  HIPCHK(c, hipEventSynchronize(c->ev1));
  float ms = 0.f;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  us = ms * 1e3;
  return 0;
}

// the fastest of 5 rounds after 2 warm-up rounds (the first send to a peer
// also sets up its connection)
int probe_best(sw_ctx* c, size_t m, int shift, double& us) {
  us = 1e300;
  for (int i = 0; i < 7; ++i) {
    double t = 0.0;
    if (int rc = probe_round(c, m, shift, t)) return rc;
    if (i >= 2) us = std::min(us, t);
  }
  return 0;
}

// t(m) = α + m/β from the grouped exchange at m1 < m2 (the slowest rank's
// times, all-gathered, so every rank's schedule decision is the same), and
// each peer's rate alone at m2.  Collective.
int link_probe(sw_ctx* c) {
  c->link = sw_link_model{};
  c->link.transport = c->hostx ? SW_XPORT_HOST : SW_XPORT_RCCL;
  if (!c->dist) return 0;
  if (const char* e = std::getenv("SW_LINK_PROBE"))
    if (e[0] == '0') return 0;
  const Slab& s = c->sl[0];
  const size_t mixed = (size_t)std::min(c->ninv, c->nfwd) * s.g.mfield * sizeof(double2);
  const size_t cap = (c->hostx ? c->hbytes : mixed) / c->P;  // bytes per peer the buffers hold
  const size_t m2 = std::min((size_t)4 << 20, cap) & ~(size_t)255;
  const size_t m1 = std::min((size_t)64 << 10, m2 / 8) & ~(size_t)255;
  if (m1 == 0) return 0;
  double t[2];
  if (int rc = probe_best(c, m1, 0, t[0])) return rc;
  if (int rc = probe_best(c, m2, 0, t[1])) return rc;
  double* dv = nullptr;
  HIPCHK(c, hipMalloc((void**)&dv, 2 * sizeof(double) * c->P));
  std::vector<double> all(2 * c->P, 0.0);
  int rc = 0;
  if (hipMemcpy(dv + 2 * s.g.slab, t, sizeof(t), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(c, SW_E_HIP, "link probe copy failed");
  if (!rc) rc = allgather(c, dv + 2 * s.g.slab, dv, sizeof(t));
  if (!rc && hipMemcpyAsync(all.data(), dv, all.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    rc = fail(c, SW_E_HIP, "link probe copy failed");
  if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(c, SW_E_HIP, "link probe sync failed");
  (void)hipFree(dv);
  if (rc) return rc;
  double T1 = 0.0, T2 = 0.0;
  for (int q = 0; q < c->P; ++q) {
    T1 = std::max(T1, all[2 * q]);
    T2 = std::max(T2, all[2 * q + 1]);
  }
  double beta = T2 > T1 ? (double)(m2 - m1) / (T2 - T1) : (double)m2 / T2;  // bytes per µs
  double alpha = std::max(0.0, T1 - (double)m1 / beta);
  c->link.probed = 1;
  c->link.latency_us = alpha;
  c->link.GBps = beta * 1e-3;
  c->link.nhalf_bytes = alpha * beta;
  if (!c->hostx)
    for (int d = 1; d < c->P && d <= 8; ++d) {
      double td = 0.0;
      if (int rc2 = probe_best(c, m2, d, td)) return rc2;
      c->link.peer_GBps[d - 1] = (double)m2 / td * 1e-3;
    }
  return 0;
}

void free_slab(Slab& s) {
  void* ptrs[] = {s.sol, s.sol2, s.hist[0], s.hist[1], s.hist[2], s.acc, s.xs, s.mic, s.mfr, s.etd, s.nt1, s.nt2};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (s.nbuf && s.nbuf != s.hist[0] && s.nbuf != s.hist[1] && s.nbuf != s.hist[2]) (void)hipFree(s.nbuf);
  if (s.mir && s.mir != s.mic) (void)hipFree(s.mir);
  if (s.mfc && s.mfc != s.mfr) (void)hipFree(s.mfc);
  for (int r = 0; r < 2; ++r) {
    void* a[] = {s.a_sol[r], s.a_zero[r], s.a_hist[0][r], s.a_hist[1][r], s.a_hist[2][r], s.a_acc[r], s.a_n[r],
                 s.a_xs[r],  s.a_xs2[r],  s.a_etd[r]};
    for (void* q : a)
      if (q) (void)hipFree(q);
  }
  if (s.a_mrow_mem) (void)hipFree(s.a_mrow_mem);  // (slab 0's; the other local slabs point to it)
}

// aliased-state tracking: every slab's compact aliased pair (arr(s)[r]) <->
// c->stage (the full array)
// One slab per process: every rank's regions, all-gathered (region 1 padded
// to kcl columns; region 0 from slab 0), then scattered into every rank's
// full array, as collect_full does for the live modes.
int alias_slot(const sw_ctx* c, size_t& r1pad, size_t& r0sz) {
  const Geom& g = c->sl[0].g;
  r1pad = (size_t)g.kcl * alias_geom(g, 1).LrP;
  r0sz = (size_t)(g.nkr - g.kc) * alias_geom(g, 0).LrP;
  return c->nf;
}
template <typename Arr>
int alias_scatter(sw_ctx* c, Arr arr) {
  if (!c->alias) return 0;
  if (!c->dist) {
    for (Slab& s : c->sl)
      for (int r = 0; r < 2; ++r) sw::launch_scatter_modes(c->nf, s.ga[r], arr(s)[r], c->stage, c->stream);
    return 0;
  }
  Slab& s = c->sl[0];
  size_t r1pad, r0sz;
  const int nf = alias_slot(c, r1pad, r0sz);
  const size_t slot = (size_t)nf * (r1pad + r0sz);
  double2* mine = c->abuf + (size_t)s.g.slab * slot;
  for (int r = 0; r < 2; ++r) {
    if (s.ga[r].kcn <= 0) continue;
    double2* dst = mine + (r == 1 ? 0 : (size_t)nf * r1pad);
    const size_t stride = r == 1 ? r1pad : r0sz;
    for (int f = 0; f < nf; ++f)
      HIPCHK(c, hipMemcpyAsync(dst + f * stride, arr(s)[r] + f * s.ga[r].cfield, s.ga[r].cfield * sizeof(double2),
                               hipMemcpyDeviceToDevice, c->stream));
  }
  if (int rc = allgather(c, mine, c->abuf, slot * sizeof(double2))) return rc;
  for (int q = 0; q < c->P; ++q) {
    const Geom gq = make_geom(c->cfg, c->P, q);
    for (int r = 0; r < 2; ++r) {
      Geom ga = alias_geom(gq, r);
      if (ga.kcn <= 0) continue;
      ga.cfield = (long long)(r == 1 ? r1pad : r0sz);
      sw::launch_scatter_modes(nf, ga, c->abuf + (size_t)q * slot + (r == 1 ? 0 : (size_t)nf * r1pad), c->stage,
                               c->stream);
    }
  }
  HIPCHK(c, hipGetLastError());
  return 0;
}
template <typename Arr>
void alias_gather(sw_ctx* c, Arr arr) {
  if (!c->alias) return;
  for (Slab& s : c->sl)
    for (int r = 0; r < 2; ++r) sw::launch_gather_modes(c->nf, s.ga[r], c->stage, arr(s)[r], c->stream);
}
auto A_SOL = [](Slab& s) -> double2** { return s.a_sol; };
auto A_NBUF = [](Slab& s) -> double2** { return s.a_nbuf; };
inline auto a_hist(int h) {
  return [h](Slab& s) -> double2** { return s.a_hist[h]; };
}

}  // namespace

extern "C" {

void sw_config_default(sw_config* cfg) {
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->abi_version = SW_ABI_VERSION;
  cfg->model = SW_MODEL_RSW;
  cfg->stepper = SW_STEP_FILTERED_AB3;
  cfg->nx = cfg->ny = 128;
  cfg->Lx = cfg->Ly = 2 * M_PI;
  cfg->aliased_fraction = 1.0 / 3.0;
  cfg->dt = 5e-2;
  cfg->f = 1.0;
  cfg->Cg = 1.0;
  cfg->nu = 1.0e-16;
  cfg->nnu = 4;
  cfg->U = 0.5;
  cfg->mu = 1e-2;
  cfg->F = 2 * 3.0 * 3.0 / 1.0 / 0.2;
  cfg->use_filter = 0;
  cfg->filter_order = 4;
  cfg->filter_innerK = 0.65;
  cfg->filter_outerK = 1.0;
  cfg->filter_tol = 1e-15;
  cfg->device = 0;
  cfg->check_nan = 1;
  cfg->nranks = 1;
  cfg->rank = 0;
  cfg->local_slabs = 1;
}

const char* sw_last_error(const sw_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

static void setup_phys(sw_ctx* c) {
  const sw_config& k = c->cfg;
  Phys& p = c->p;
  p.f = k.f;
  p.Cg2 = k.Cg * k.Cg;
  p.nu = k.nu;
  p.nnu = k.nnu;
  p.U = k.U;
  p.mu = k.mu;
  p.F = k.F;
  p.Ro = k.Ro;
  p.model = k.model;
  if (k.model == SW_MODEL_MLQG) {  // MultiLayerQG.Params, 2 layers, no topography
    const double gp = k.b[0] - k.b[1];
    p.F = k.f0 * k.f0 / (gp * k.H[0]);
    p.F2 = k.f0 * k.f0 / (gp * k.H[1]);
    p.U1 = k.Ulayer[0];
    p.U2 = k.Ulayer[1];
    p.Qy1 = k.beta - p.F * (k.Ulayer[1] - k.Ulayer[0]);
    p.Qy2 = k.beta - p.F2 * (k.Ulayer[0] - k.Ulayer[1]);
  }
  p.dt = k.dt;
  p.use_filter = (k.stepper == SW_STEP_FILTERED_AB3 || k.stepper == SW_STEP_FILTERED_RK4) ? 1 : (k.use_filter ? 1 : 0);
  p.forder = k.filter_order;
  p.innerK = k.filter_innerK;
  p.decay = -std::log(k.filter_tol) / std::pow(k.filter_outerK - k.filter_innerK, (double)k.filter_order);

}

// A grid that is not a power of two per side: the generic engine
// (sw_generic.hpp) for MultiLayerQG + FilteredRK4 — TwoLayerSimulation with
// simulation/MattParameters.jl (nx = 384) — on one device.  Slabs in one
// process (local_slabs == nranks) hold the whole grid (the results are the
// undecomposed run's: bitwise equal for any P); one slab per process, the
// aliased-state mode and other model/stepper pairs are refused.
int create_generic(sw_ctx* c) {
  const sw_config& k = c->cfg;
  int rx[24], ry[24];
  if (!sw::gen::radices(k.nx, rx) || !sw::gen::radices(k.ny, ry))
    return fail(c, SW_E_INVALID,
                "nx, ny must be powers of two in [32, 8192], or (MultiLayerQG with FilteredRK4) even sizes of the "
                "form 2^a 3^b 5^c in [16, 4096]");
  if (k.model != SW_MODEL_MLQG || k.stepper != SW_STEP_FILTERED_RK4)
    return fail(c, SW_E_INVALID,
                "grids that are not powers of two: MultiLayerQG with FilteredRK4 only (simulation/MattParameters.jl)");
  if (!(k.aliased_fraction >= 0 && k.aliased_fraction < 1))
    return fail(c, SW_E_INVALID, "aliased_fraction must be in [0,1)");
  if (k.precision != SW_PREC_F64 && k.precision != SW_PREC_F32)
    return fail(c, SW_E_INVALID, "precision must be SW_PREC_F64 or SW_PREC_F32");
  if (k.aliased_state) return fail(c, SW_E_INVALID, "aliased_state: power-of-two grids only");
  if (k.nnu < 0 || k.nnu > 255 || k.filter_order < 0 || k.filter_order > 255)
    return fail(c, SW_E_INVALID, "nnu and filter_order must be in [0, 255]");
  const int P = k.nranks < 1 ? 1 : k.nranks;
  const int nlocal = k.local_slabs <= 1 ? 1 : k.local_slabs;
  if (P > 1 && nlocal != P)
    return fail(c, SW_E_INVALID, "grids that are not powers of two: one process holds every slab (local_slabs = nranks)");
  int ndev = 0;
  HIPCHK(c, hipGetDeviceCount(&ndev));
  if (k.device < 0 || k.device >= ndev) return fail(c, SW_E_INVALID, "bad device ordinal");
  HIPCHK(c, hipSetDevice(k.device));
  HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIPCHK(c, hipEventCreate(&c->ev0));
  HIPCHK(c, hipEventCreate(&c->ev1));
  c->P = 1;  // (every slab on this device: the undecomposed grid)
  c->dist = false;
  setup_phys(c);
  c->nf = 2;
  c->kmodel = SW_MODEL_QG2;
  c->sl.resize(1);
  Slab& s = c->sl[0];
  s.g = make_geom(k, 1, 0);
  const Geom& g = s.g;
  if (g.kc <= 0 || g.lc > g.lr2) return fail(c, SW_E_INVALID, "degenerate dealiasing geometry");
  int rc;
  if ((rc = alloc(c, (void**)&s.sol, full_bytes(c)))) return rc;
  HIPCHK(c, hipMemsetAsync(s.sol, 0, full_bytes(c), c->stream));
  if ((rc = alloc(c, (void**)&c->stage, full_bytes(c)))) return rc;
  if (k.precision == SW_PREC_F32)
    if ((rc = alloc(c, (void**)&c->stage32, full_bytes(c) / 2))) return rc;
  if ((rc = alloc(c, (void**)&c->dflt, (size_t)g.nx * g.ny * sizeof(double)))) return rc;
  if ((rc = alloc(c, (void**)&c->flag, 1024 * sizeof(int)))) return rc;
  if ((rc = alloc(c, (void**)&c->sflag, 2 * sizeof(int)))) return rc;
  if ((rc = alloc(c, (void**)&c->esum, (SW_NSUM + 2) * sizeof(double)))) return rc;
  HIPCHK(c, hipHostMalloc((void**)&c->hflag, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  HIPCHK(c, hipHostGetDevicePointer((void**)&c->hflag_dev, c->hflag, 0));
  *c->hflag = 0;
  std::string err;
  if ((rc = sw::gen::create(c->gen, k, c->p, g, s.sol, c->stream, err))) return fail(c, rc, err);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (const char* e = std::getenv("SW_CHECK_NAN")) {
    if (e[0] == '1') c->cfg.check_nan = 1;
#ifdef SW_EXPERIMENTS
    else c->cfg.check_nan = 0;
#endif
  }
  c->stats.resize(K_NKERN);
  for (int i = 0; i < K_NKERN; ++i) c->stats[i].name = kname[i];
  return SW_OK;
}

int sw_create(sw_ctx** out, const sw_config* cfg) {
  if (!out || !cfg) return SW_E_INVALID;
  *out = nullptr;
  if (cfg->abi_version != SW_ABI_VERSION) return SW_E_INVALID;
  sw_ctx* c = new sw_ctx();
  c->cfg = *cfg;
  *out = c;
  const sw_config& k = c->cfg;
  if (k.model < SW_MODEL_RSW || k.model > SW_MODEL_MLQG) return fail(c, SW_E_INVALID, "unknown model");
  if (k.stepper < 0 || k.stepper > 4) return fail(c, SW_E_INVALID, "unknown stepper");
  if (k.model == SW_MODEL_MLQG && k.stepper != SW_STEP_FILTERED_RK4 && k.stepper != SW_STEP_FILTERED_AB3)
    return fail(c, SW_E_INVALID, "MultiLayerQG steps with FilteredRK4 (or FilteredAB3): its L is the hyperviscosity alone");
  if (k.model == SW_MODEL_MLQG && (!(k.H[0] > 0) || !(k.H[1] > 0) || k.b[0] == k.b[1]))
    return fail(c, SW_E_INVALID, "MultiLayerQG needs H > 0 and b[0] != b[1]");
  if ((k.model == SW_MODEL_TY) != (k.stepper == SW_STEP_ETDRK4))
    return fail(c, SW_E_INVALID, "ETDRK4 (diagonal L) is the Thomas-Yamada stepper and TY steps with ETDRK4 only");
  if (!pow2(k.nx) || !pow2(k.ny)) return create_generic(c);
  if (k.nx < 32 || k.ny < 32 || k.nx > 8192 || k.ny > 8192)
    return fail(c, SW_E_INVALID, "nx, ny must be powers of two in [32, 8192]");
  if (!sw::length_built(ilog2(k.nx)) || !sw::length_built(ilog2(k.ny)))
    return fail(c, SW_E_INVALID, "nx or ny: transform length not built into this library (one-length build)");
  if (!(k.aliased_fraction >= 0 && k.aliased_fraction < 1))
    return fail(c, SW_E_INVALID, "aliased_fraction must be in [0,1)");
  if (k.filter_order < 0) return fail(c, SW_E_INVALID, "filter_order must be >= 0");
  if (k.precision != SW_PREC_F64 && k.precision != SW_PREC_F32)
    return fail(c, SW_E_INVALID, "precision must be SW_PREC_F64 or SW_PREC_F32");
  if (k.aliased_state) {
    const bool ab_or_if = k.stepper == SW_STEP_IFMAB3 || k.stepper == SW_STEP_IFMRK4 ||
                          k.stepper == SW_STEP_FILTERED_AB3;
    if (!(((k.model == SW_MODEL_QG2 || k.model == SW_MODEL_RSW) && ab_or_if) ||
          (k.model == SW_MODEL_TY && k.stepper == SW_STEP_ETDRK4) || k.model == SW_MODEL_MLQG))
      return fail(c, SW_E_INVALID,
                  "aliased_state: RSW or 2LQG with IFMAB3, IFMRK4 or FilteredAB3, Thomas-Yamada with ETDRK4, "
                  "or MultiLayerQG");
    // (one slab per process: region 0's y-transforms need every row of the
    // row pass's aliased x-spectra, all-gathered per calcN)
    const int amodel = k.model == SW_MODEL_RSW ? sw::MODEL_RSWA : k.model == SW_MODEL_MLQG ? sw::MODEL_QG2 : k.model;
    if (!sw::row_alias_built(amodel, ilog2(k.nx)))
      return fail(c, SW_E_INVALID, "aliased_state: the row pass's aliased output is not built at this nx");
  }
  const int P = k.nranks;
  if (!pow2(P) || k.ny / P < 32)
    return fail(c, SW_E_INVALID, "nranks must be a power of two with ny / nranks >= 32");
  const int nlocal = k.local_slabs <= 1 ? 1 : k.local_slabs;
  if (nlocal != 1 && nlocal != P) return fail(c, SW_E_INVALID, "local_slabs must be 1 or nranks");
  if (P > 1 && nlocal == 1 && (k.rank < 0 || k.rank >= P)) return fail(c, SW_E_INVALID, "bad rank");
  if (P > 1 && nlocal == 1 && !k.comm_unique_id && !k.exchange)
    return fail(c, SW_E_INVALID, "nranks > 1 with one slab per process needs comm_unique_id or exchange");
  c->P = P;
  c->dist = P > 1 && nlocal == 1;
  c->hostx = c->dist && k.exchange;

  int ndev = 0;
  HIPCHK(c, hipGetDeviceCount(&ndev));
  if (k.device < 0 || k.device >= ndev) return fail(c, SW_E_INVALID, "bad device ordinal");
  HIPCHK(c, hipSetDevice(k.device));
  HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  HIPCHK(c, hipEventCreate(&c->ev0));
  HIPCHK(c, hipEventCreate(&c->ev1));
  if (P > 1) {
    HIPCHK(c, hipStreamCreateWithFlags(&c->comm, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_row, hipEventDisableTiming));
    HIPCHK(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    for (int i = 0; i < 8; ++i) {
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_fwd[i], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_col[i], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_chunk[i], hipEventDisableTiming));
      HIPCHK(c, hipEventCreateWithFlags(&c->ev_rowc[i], hipEventDisableTiming));
    }
    // Pipelined by default across GPUs (RCCL over xGMI runs beside the column
    // kernels) where each per-(peer, field) message is >= 1 MiB; below that a
    // transpose is latency-bound and the per-group schedule's 3 + 3 grouped
    // send/recv calls per calcN cost more than they overlap, so the
    // sequential schedule (one group per direction) runs there (e.g. the
    // 2048² metric problem on 8 GPUs: 360 KB messages).  With every slab in
    // this process the "transposes" are copies through the same HBM the
    // kernels stream, and splitting the column pass into per-field launches
    // only costs (tools/overlap_check.py): sequential there.
    {
      const Geom g0 = make_geom(k, P, 0);
      const size_t msg = (size_t)g0.kcl * g0.nyl * sizeof(double2);
      c->overlap = c->dist && !c->hostx && msg >= ((size_t)1 << 20);
    }
    if (const char* e = std::getenv("SW_OVERLAP")) c->overlap = e[0] == '1';
  }
  if (c->dist && !c->hostx) {
    ncclUniqueId id;
    std::memcpy(&id, k.comm_unique_id, sizeof(id));
    NCCLCHK(c, ncclCommInitRank(&c->nccl, P, id, k.rank));
  }

  c->sl.resize(nlocal);
  for (int i = 0; i < nlocal; ++i) c->sl[i].g = make_geom(k, P, c->dist ? k.rank : i);
  {
    const Geom& g = c->sl[0].g;
    if (g.kc <= 0 || g.Lr <= 0 || g.lc > g.lr2) return fail(c, SW_E_INVALID, "degenerate dealiasing geometry");
  }
  // device ipow is unrolled over 8 exponent bits (sw_internal.hpp)
  if (k.nnu < 0 || k.nnu > 255 || k.filter_order < 0 || k.filter_order > 255)
    return fail(c, SW_E_INVALID, "nnu and filter_order must be in [0, 255]");

  setup_phys(c);

  c->nf = k.model == SW_MODEL_RSW ? 3 : (k.model == SW_MODEL_TY ? 4 : 2);
  c->kmodel = k.model == SW_MODEL_MLQG ? SW_MODEL_QG2 : k.model;  // MLQG runs the 2LQG kernels
  // RSW: the vorticity form of the calcN is exact on the live modes of the
  // 2/3 rule; with aliased_fraction = 0 (no dealiased band) the reference's
  // advective form runs instead (sw::MODEL_RSWA; SW_RSW_ADV=1 forces it)
  if (k.model == SW_MODEL_RSW) {
    // the aliased modes need the reference's own products (aliased_state)
    bool adv = k.aliased_fraction == 0 || k.aliased_state;
    if (const char* e = std::getenv("SW_RSW_ADV")) adv = adv || e[0] == '1';
    if (adv) c->kmodel = sw::MODEL_RSWA;
  }
  // mixed fields per calcN: RSW U,V,H,Uy in / P,K,ζu,Q,vη out;
  // QG2 Q,Ψ,Ψy per layer in / ψx q, ψy q per layer out; TY ζ,ψ,ût,∂y ut,
  // uc,∂y uc,vc,pc,∂y pc in / 7 combined product spectra out (k_row)
  c->ninv = c->kmodel == sw::MODEL_RSWA ? 5 : k.model == SW_MODEL_RSW ? 4 : (k.model == SW_MODEL_TY ? 9 : 6);
  c->nfwd = c->kmodel == sw::MODEL_RSWA ? 4 : k.model == SW_MODEL_RSW ? 5 : (k.model == SW_MODEL_TY ? 7 : 4);

  // the forward column pass with one term of N per block on short columns
  // (k_col_fwd SPLIT; round 5): built for RSW (vorticity
  // form), 2LQG / MultiLayerQG and Thomas–Yamada, on by default on 512-point
  // columns for RSW, MultiLayerQG and Thomas–Yamada (2LQG IFMAB3 measured
  // neutral to -1 %); SW_FWD_SPLIT=0/1 forces it off/on where it is built
  {
    const bool built = (c->kmodel == SW_MODEL_RSW || c->kmodel == SW_MODEL_QG2 || c->kmodel == SW_MODEL_TY) &&
                       !k.aliased_state && !k.nop_calcN;
    c->fsplit = built && k.model != SW_MODEL_QG2 && ilog2(k.ny) <= 9;
    if (const char* e = std::getenv("SW_FWD_SPLIT")) c->fsplit = built && e[0] == '1';
    // only the separate col_fwd + update path reads the split:
    // the fused column step and the forward + update pass never allocate it
    if (const char* e = std::getenv("SW_FUSE_ALL")) c->fuse_all = e[0] == '1';
    if (const char* e = std::getenv("SW_FWD_STEP")) c->fwd_step = e[0] == '1' ? 1 : (e[0] == '2' ? 2 : 0);
    if (use_fused(c) || use_fwd_step(c)) c->fsplit = false;
  }
  int rc;
  for (Slab& s : c->sl) {
    const Geom& g = s.g;
    const size_t cb = (size_t)g.cfield * sizeof(double2);
    const size_t mb = (size_t)g.mfield * sizeof(double2);
    if ((rc = alloc(c, (void**)&s.sol, c->nf * cb))) return rc;
    if (c->fsplit)
      for (double2** q : {&s.nt1, &s.nt2})
        if ((rc = alloc(c, (void**)q, c->nf * cb))) return rc;
    if ((rc = alloc(c, (void**)&s.xs, c->nf * cb))) return rc;
    if (k.stepper == SW_STEP_FILTERED_AB3)
      if ((rc = alloc(c, (void**)&s.sol2, c->nf * cb))) return rc;
    if ((rc = alloc(c, (void**)&s.mic, c->ninv * mb))) return rc;
    if ((rc = alloc(c, (void**)&s.mfr, c->nfwd * mb))) return rc;
    s.mir = s.mic;
    s.mfc = s.mfr;
    if (P > 1) {
      if ((rc = alloc(c, (void**)&s.mir, c->ninv * mb))) return rc;
      if ((rc = alloc(c, (void**)&s.mfc, c->nfwd * mb))) return rc;
    }
    if (k.stepper == SW_STEP_IFMRK4 || k.stepper == SW_STEP_ETDRK4 || k.stepper == SW_STEP_FILTERED_RK4) {
      if ((rc = alloc(c, (void**)&s.acc, c->nf * cb))) return rc;
      if ((rc = alloc(c, (void**)&s.nbuf, c->nf * cb))) return rc;
    }
    if (k.stepper == SW_STEP_ETDRK4) {  // N₁, N₂, s₂ and the coefficient table
      for (int i = 0; i < 3; ++i)
        if ((rc = alloc(c, (void**)&s.hist[i], c->nf * cb))) return rc;
      s.xs2 = s.hist[2];
      if ((rc = alloc(c, (void**)&s.etd, (size_t)sw::ETD_N * g.cfield * sizeof(double)))) return rc;
      sw::launch_etd_coeffs(g, c->p, s.etd, c->stream);
      HIPCHK(c, hipGetLastError());
    } else if (k.stepper != SW_STEP_IFMRK4 && k.stepper != SW_STEP_FILTERED_RK4) {
      for (int i = 0; i < 3; ++i)
        if ((rc = alloc(c, (void**)&s.hist[i], c->nf * cb))) return rc;
    }
  }
  c->alias = k.aliased_state != 0;
  size_t alias_cols = 0;
  for (Slab& s : c->sl) {
    if (!c->alias) break;
    for (int r = 0; r < 2; ++r) {
      s.ga[r] = alias_geom(s.g, r);
      if (s.ga[r].kcn <= 0) continue;
      alias_cols += s.ga[r].kcn;
      const size_t cb = (size_t)c->nf * s.ga[r].cfield * sizeof(double2);
      for (double2** q : {&s.a_sol[r], &s.a_zero[r], &s.a_xs[r]})
        if ((rc = alloc(c, (void**)q, cb))) return rc;
      const bool rk = k.stepper == SW_STEP_IFMRK4 || k.stepper == SW_STEP_FILTERED_RK4;
      if (rk || k.stepper == SW_STEP_ETDRK4) {
        if ((rc = alloc(c, (void**)&s.a_acc[r], cb))) return rc;
        if ((rc = alloc(c, (void**)&s.a_n[r], cb))) return rc;
      }
      if (k.stepper == SW_STEP_ETDRK4) {  // N₁, N₂, s₂ and the coefficients at the aliased modes
        for (double2** q : {&s.a_hist[0][r], &s.a_hist[1][r], &s.a_xs2[r]})
          if ((rc = alloc(c, (void**)q, cb))) return rc;
        if ((rc = alloc(c, (void**)&s.a_etd[r], (size_t)sw::ETD_N * s.ga[r].cfield * sizeof(double)))) return rc;
        sw::launch_etd_coeffs(s.ga[r], c->p, s.a_etd[r], c->stream);
        HIPCHK(c, hipGetLastError());
      } else if (!rk) {
        for (int i = 0; i < 3; ++i)
          if ((rc = alloc(c, (void**)&s.a_hist[i][r], cb))) return rc;
      }
    }
    if (s.ga[0].kcn > 0) {  // slab 0: every slab's block of rows (one slab per process: gather0)
      const size_t mrow = (size_t)c->nfwd * (s.g.nkr - s.g.kc) * s.g.ny * sizeof(double2);
      if ((rc = alloc(c, (void**)&s.a_mrow_mem, mrow))) return rc;
      s.a_mrow = s.a_mrow_mem;
    } else if (c->dist) {  // one slab per process, rank != 0: its own block
      const size_t B = (size_t)c->nfwd * sw::ma_field(s.g);
      if ((rc = alloc(c, (void**)&s.a_mrow_mem, B * sizeof(double2)))) return rc;
      s.a_mrow = s.a_mrow_mem - (size_t)s.g.slab * B;  // the row pass writes block `slab` only
    } else {
      s.a_mrow = c->sl[0].a_mrow;
    }
  }
  const Geom& g = c->sl[0].g;
  if ((rc = alloc(c, (void**)&c->stage, full_bytes(c)))) return rc;
  if (k.precision == SW_PREC_F32)  // >= one physical field in fp32 too
    if ((rc = alloc(c, (void**)&c->stage32, full_bytes(c) / 2))) return rc;
  if ((rc = alloc(c, (void**)&c->dflt, (size_t)g.nx * g.ny * sizeof(double)))) return rc;
  if ((rc = alloc(c, (void**)&c->flag, 1024 * sizeof(int)))) return rc;
  if ((rc = alloc(c, (void**)&c->sflag, (c->P + 1) * sizeof(int)))) return rc;
  if (!c->dist) {
    HIPCHK(c, hipHostMalloc((void**)&c->hflag, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(c, hipHostGetDevicePointer((void**)&c->hflag_dev, c->hflag, 0));
    *c->hflag = 0;
  }
  size_t ecols = (size_t)P * g.kcl + alias_cols;
  if (c->dist && alias_energy(c))  // + region 0, every slab's region 1 and their gather scratch (sw_diag)
    ecols = (size_t)P * g.kcl + ((size_t)(g.nkr - g.kc) + (size_t)P * g.kcl) +
            (size_t)P * ((size_t)(g.nkr - g.kc) + g.kcl);
  if ((rc = alloc(c, (void**)&c->ecols, SW_NSUM * ecols * sizeof(double)))) return rc;
  if ((rc = alloc(c, (void**)&c->esum, (SW_NSUM + 2 * (size_t)P) * sizeof(double)))) return rc;
  if (c->dist) {
    const size_t gb = (size_t)P * c->nf * g.kcl * g.LrP * sizeof(double2);
    if ((rc = alloc(c, (void**)&c->gbuf, gb))) return rc;
    size_t ab = 0, mb = 0;  // aliased state: the regions' and the row pass's x-spectra all-gathers
    if (c->alias) {
      size_t r1pad, r0sz;
      const int nf = alias_slot(c, r1pad, r0sz);
      ab = (size_t)P * nf * (r1pad + r0sz) * sizeof(double2);
      if ((rc = alloc(c, (void**)&c->abuf, ab))) return rc;
      mb = (size_t)c->nfwd * (g.nkr - g.kc) * g.ny * sizeof(double2);
    }
    if (c->hostx) {
      // largest message set: a transpose, the compact all-gather or the physical rows
      const size_t tb = (size_t)std::max(c->ninv, c->nfwd) * (size_t)g.mfield * sizeof(double2);
      const size_t pb = (size_t)g.nx * g.ny * sizeof(double);
      c->hbytes = std::max(std::max(tb, std::max(gb, pb)), std::max(ab, mb));
      HIPCHK(c, hipHostMalloc((void**)&c->hsend, c->hbytes, hipHostMallocDefault));
      HIPCHK(c, hipHostMalloc((void**)&c->hrecv, c->hbytes, hipHostMallocDefault));
    }
  }
  {
    auto tx = twiddles(k.nx);
    HIPCHK(c, hipMalloc((void**)&c->tw_x, tx.size() * sizeof(double2)));
    HIPCHK(c, hipMemcpy(c->tw_x, tx.data(), tx.size() * sizeof(double2), hipMemcpyHostToDevice));
    auto ty = twiddles(k.ny);
    HIPCHK(c, hipMalloc((void**)&c->tw_y, ty.size() * sizeof(double2)));
    HIPCHK(c, hipMemcpy(c->tw_y, ty.data(), ty.size() * sizeof(double2), hipMemcpyHostToDevice));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // Row-chunked pipeline: with the pipelined exchange, the row
  // pass runs in chunks of local rows behind the last inverse group's
  // transposes, in 4 chunks where each per-(peer, field) message of a chunk
  // stays >= 1 MiB (latency-bound below); SW_ROW_CHUNKS=k forces k (1, 2, 4, 8).
  // A chunk is a multiple of 64 rows (the row pass's XCD interleave) and of
  // the row blocks' lines; the inverse tiles must be row-major 2×4.  The
  // forward transposes follow the row chunks (fwd_async) where the forward
  // tiles are row-major too (the default on several slabs).
  if (P > 1) {
    const Geom& g = c->sl[0].g;
    // the link model (round 6, VERDICT r05 #4b-c): pipelined where this
    // decomposition's per-(peer, field) message reaches n½ = α·β of the probed
    // links (clamped to [64 KiB, 16 MiB]); without a probe the fixed 1 MiB
    if ((rc = link_probe(c))) return rc;
    const double msg = (double)g.kcl * g.nyl * sizeof(double2);
    double thr = (double)((size_t)1 << 20);
    if (c->link.probed) thr = std::min(std::max(c->link.nhalf_bytes, 65536.0), 16777216.0);
    if (c->link.probed && c->dist && !c->hostx) c->overlap = msg >= thr;
    if (const char* e = std::getenv("SW_OVERLAP")) c->overlap = e[0] == '1';
    c->link.msg_bytes = msg;
    int k = msg / 4 >= thr ? 4 : (msg / 2 >= thr && c->link.probed ? 2 : 1);
    int unit = 64;
    if (const char* e = std::getenv("SW_ROW_CHUNKS")) {
      k = std::atoi(e);
      unit = 1;
    }
    unit = std::max(unit, std::max(4, sw::row_lines_per_block(c->kmodel, g.log2nx)));
    while (k > 1 && (k > 8 || g.nyl % (k * unit) != 0)) k /= 2;
    c->row_chunks = (SW_TILE_I == 2 && SW_LORD_I == 0 && k > 1) ? k : 1;
    c->link.pipelined = (c->dist && !c->hostx && c->overlap && !c->alias) ? 1 : 0;
    c->link.row_chunks = c->link.pipelined ? c->row_chunks : 1;
  }
  // Cache policy of the stepper state (sw_kernels.hip state_ld): a step
  // whose traffic on this GPU exceeds the 256 MiB Infinity Cache evicts the
  // state before the next step reads it, so the state goes non-temporal and
  // the cache keeps the mixed fields between the passes instead (2048²
  // FilteredAB3 +7 %); a smaller step keeps the state cached (1024² +9 %
  // temporal).  SW_STREAM_STATE=0/1 overrides.
  c->stream_state = step_bytes(c) > 256.0 * 1024 * 1024;
  if (const char* e = std::getenv("SW_STREAM_STATE")) c->stream_state = e[0] == '1';
  // SW_CHECK_NAN=1 turns the NaN check of sw_step on; only an experiment
  // build (-DSW_EXPERIMENTS, tools/build_variants.sh) lets =0 turn off a
  // caller's check_nan = 1
  if (const char* e = std::getenv("SW_CHECK_NAN")) {
    if (e[0] == '1') c->cfg.check_nan = 1;
#ifdef SW_EXPERIMENTS
    else c->cfg.check_nan = 0;
#endif
  }
  c->stats.resize(K_NKERN);
  for (int i = 0; i < K_NKERN; ++i) c->stats[i].name = kname[i];
  return SW_OK;
}

void sw_destroy(sw_ctx* c) {
  if (!c) return;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  sw::gen::destroy(c->gen);
  for (Slab& s : c->sl) free_slab(s);
  if (c->erec1_host) {  // (erec1 is its device view)
    (void)hipHostFree(c->erec1_host);
    c->erec1 = nullptr;
  }
  void* ptrs[] = {c->tw_x, c->tw_y, c->stage, c->stage32, c->gbuf, c->abuf, c->dflt, c->flag, c->sflag, c->ecols, c->esum, c->erec,
                  c->erec1, c->cold, c->cold_out};
  for (void* q : ptrs)
    if (q) (void)hipFree(q);
  if (c->nccl) (void)ncclCommDestroy(c->nccl);
  for (hipEvent_t e : {c->ev_row, c->ev_join})
    if (e) (void)hipEventDestroy(e);
  for (int i = 0; i < 8; ++i) {
    if (c->ev_fwd[i]) (void)hipEventDestroy(c->ev_fwd[i]);
    if (c->ev_col[i]) (void)hipEventDestroy(c->ev_col[i]);
    if (c->ev_chunk[i]) (void)hipEventDestroy(c->ev_chunk[i]);
    if (c->ev_rowc[i]) (void)hipEventDestroy(c->ev_rowc[i]);
  }
  if (c->comm) (void)hipStreamDestroy(c->comm);
  if (c->hsend) (void)hipHostFree(c->hsend);
  if (c->hflag) (void)hipHostFree(c->hflag);
  if (c->hrecv) (void)hipHostFree(c->hrecv);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  for (hipEvent_t e : c->wev) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->pev) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

static bool ready(const sw_ctx* c) { return c && !c->sl.empty() && c->sl[0].sol && c->stage; }

int sw_get_dims(const sw_ctx* c, int32_t* nkr, int32_t* nl, int32_t* nf) {
  if (!ready(c)) return SW_E_STATE;
  if (nkr) *nkr = c->sl[0].g.nkr;
  if (nl) *nl = c->sl[0].g.nl;
  if (nf) *nf = c->nf;
  return SW_OK;
}

int sw_set_state(sw_ctx* c, const void* sol, size_t bytes) {
  if (!ready(c)) return SW_E_STATE;
  if (!sol || bytes != caller_bytes(c, full_bytes(c))) return fail(c, SW_E_INVALID, "sw_set_state: size mismatch");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = upload(c, sol, c->stage, full_bytes(c))) return rc;
  if (c->gen) {  // full-array state: a copy, then dealias!
    HIPCHK(c, hipMemcpyAsync(c->sl[0].sol, c->stage, full_bytes(c), hipMemcpyDeviceToDevice, c->stream));
    sw::gen::dealias(c->gen, c->sl[0].sol);
  } else {
    for (Slab& s : c->sl) sw::launch_gather(c->nf, s.g, c->stage, s.sol, c->stream);
  }
  alias_gather(c, A_SOL);  // sol .= q0h keeps them until updatevars!/calcN! dealias
  c->mixed_valid = false;
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SW_OK;
}

int sw_get_state(const sw_ctx* cc, void* sol, size_t bytes) {
  sw_ctx* c = const_cast<sw_ctx*>(cc);
  if (!ready(c)) return SW_E_STATE;
  if (!sol || bytes != caller_bytes(c, full_bytes(c))) return fail(c, SW_E_INVALID, "sw_get_state: size mismatch");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = collect_full(c, &Slab::sol)) return rc;
  if (int rc = alias_scatter(c, A_SOL)) return rc;
  if (int rc = download(c, c->stage, sol, full_bytes(c))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SW_OK;
}

int sw_set_clock(sw_ctx* c, double t, int64_t step) {
  if (!c) return SW_E_STATE;
  if (step < 0) return fail(c, SW_E_INVALID, "negative step");
  c->t = t;
  c->step = step;
  return SW_OK;
}

int sw_get_clock(const sw_ctx* c, double* t, int64_t* step) {
  if (!c) return SW_E_STATE;
  if (t) *t = c->t;
  if (step) *step = c->step;
  return SW_OK;
}

int sw_step(sw_ctx* c, int64_t nsteps) {
  if (!ready(c)) return SW_E_STATE;
  if (nsteps < 0) return fail(c, SW_E_INVALID, "negative nsteps");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (nsteps > 0)
    if (int rc = scan_arm(c)) return rc;
  for (int64_t i = 0; i < nsteps; ++i)
    if (int rc = step_once(c)) return rc;
  if (int rc = join_comm(c)) return rc;  // primed inverse transposes still on the side stream
  HIPCHK(c, hipGetLastError());
  if (c->scan) {
    int h = 0;
    if (int rc = scan_read(c, h)) return rc;
    if (h) return fail(c, SW_E_NAN, "Solution is NaN");
  } else {
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return SW_OK;
}

int sw_calcN(sw_ctx* c, const void* sol, void* N, size_t bytes) {
  if (!ready(c)) return SW_E_STATE;
  if (!sol || !N || bytes != caller_bytes(c, full_bytes(c))) return fail(c, SW_E_INVALID, "sw_calcN: size mismatch");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  c->mixed_valid = false;  // mixed arrays are used as scratch
  if (int rc = upload(c, sol, c->stage, full_bytes(c))) return rc;
  if (c->gen) {  // N = calcN(dealias(sol)) on the full array
    sw::gen::calcN(c->gen, c->stage, c->gen->N);
    HIPCHK(c, hipMemcpyAsync(c->stage, c->gen->N, full_bytes(c), hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipGetLastError());
    if (int rc = download(c, c->stage, N, full_bytes(c))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return SW_OK;
  }
  for (Slab& s : c->sl) {
    sw::launch_gather(c->nf, s.g, c->stage, s.xs, c->stream);
    // scratch output: the ring slot that the next step overwrites anyway
    if (c->cfg.stepper != SW_STEP_IFMRK4 && c->cfg.stepper != SW_STEP_ETDRK4 &&
        c->cfg.stepper != SW_STEP_FILTERED_RK4)
      s.nbuf = s.hist[c->head];
  }
  set_alias_nbuf(c);
  if (int rc = calcN(c, &Slab::xs, &Slab::nbuf)) return rc;
  for (Slab& s : c->sl) {  // a split N completed (the updates complete it per mode)
    if (!s.nt1) continue;
    sw::StepPtrs a{};
    a.nt1 = s.nt1;
    a.nt2 = s.nt2;
    a.xin = s.xs;
    sw::launch_assemble_terms(c->nf, s.g, c->p, a, s.nbuf, c->stream);
  }
  if (int rc = collect_full(c, &Slab::nbuf)) return rc;
  if (int rc = alias_scatter(c, A_NBUF)) return rc;
  if (int rc = download(c, c->stage, N, full_bytes(c))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SW_OK;
}

// one physical field (updatevars!) of the current state into c->dflt: this
// rank's rows (one slab per process) or every row (all slabs here)
static int physical_to_dflt(sw_ctx* c, int32_t fid) {
  if (c->gen) {
    sw::gen::physical(c->gen, c->sl[0].sol, fid, c->dflt);
    HIPCHK(c, hipGetLastError());
    return 0;
  }
  c->mixed_valid = false;  // mixed arrays are used as scratch
  for (Slab& s : c->sl) {
    sw::launch_make_spec(c->cfg.model, fid, s.g, c->p, s.sol, s.xs, c->stream);
    sw::launch_col_inv1(s.g, s.xs, s.mic, c->tw_y, c->stream);
  }
  if (int rc = transpose(c, true, 1)) return rc;
  for (Slab& s : c->sl) sw::launch_row_c2r1(s.g, s.mir, c->dflt, c->tw_x, c->stream);
  HIPCHK(c, hipGetLastError());
  return 0;
}

static bool valid_phys_id(const sw_ctx* c, int32_t fid) {
  const int id = fid & 7, layer = fid >> 3;
  if (c->cfg.model == SW_MODEL_RSW) return fid >= 0 && fid <= 3;
  if (c->cfg.model == SW_MODEL_TY) return (fid >= 0 && fid <= 5) || fid == 8 || fid == 9;
  return fid >= 0 && layer <= 1 && id != SW_PHYS_ETA && id <= 5;
}

int sw_get_physical(sw_ctx* c, int32_t fid, void* out, size_t bytes) {
  if (!ready(c)) return SW_E_STATE;
  const Geom& g0 = c->sl[0].g;
  const size_t pbytes = (size_t)g0.nx * g0.ny * sizeof(double);
  if (!out || bytes != caller_bytes(c, pbytes)) return fail(c, SW_E_INVALID, "sw_get_physical: size mismatch");
  if (!valid_phys_id(c, fid))
    return fail(c, SW_E_INVALID, c->cfg.model == SW_MODEL_RSW ? "RSW physical ids are 0..3"
                                 : c->cfg.model == SW_MODEL_TY ? "TY physical ids are 0..5, 8, 9"
                                                               : "bad QG2 physical id");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  // updatevars! begins with dealias!(sol, grid) (swqg/TwoLayerQG.jl:115)
  for (int r = 0; c->alias && r < 2; ++r)
    for (Slab& s : c->sl)
      if (s.ga[r].kcn > 0)
        HIPCHK(c, hipMemsetAsync(s.a_sol[r], 0, (size_t)c->nf * s.ga[r].cfield * sizeof(double2), c->stream));
  if (int rc = physical_to_dflt(c, fid)) return rc;
  if (c->dist) {
    const size_t rows = (size_t)g0.nyl * g0.nx;
    if (int rc = allgather(c, c->dflt + (size_t)g0.y0 * g0.nx, c->dflt, rows * sizeof(double))) return rc;
  }
  if (int rc = download(c, c->dflt, out, pbytes)) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SW_OK;
}

// k_absmax's order-preserving key -> the double
static double key_double(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & ~0x8000000000000000ull) : ~k;
  double d;
  std::memcpy(&d, &b, sizeof(d));
  return d;
}

// energy sums (k_energy_partial triples) -> (KE, KE2, PE)
// (rsw/RotatingShallowWater.jl:323-333; swqg/TwoLayerQG.jl:230-250, KE per
// layer), with the parsevalsum(2) normalisation
static void energies_from_sums(const sw_ctx* c, const double a[SW_NSUM], double& ke, double& ke2, double& pe,
                               double* wg = nullptr) {
  const Geom& g = c->sl[0].g;
  const double norm = g.Lx * g.Ly / ((double)g.nx * g.nx * (double)g.ny * g.ny);
  // TY wave_geostrophic_energy (:353-367): (wave KE, wave PE, geo KE, geo PE)
  if (wg)
    for (int i = 0; i < 4; ++i) wg[i] = c->cfg.model == SW_MODEL_TY ? norm * a[3 + i] : 0.0;
  if (c->cfg.model == SW_MODEL_RSW) {
    ke = norm * a[0] / (2 * g.Lx * g.Ly);
    ke2 = 0.0;
    pe = 0.5 * c->p.Cg2 * norm * a[1] / (g.Lx * g.Ly);
  } else if (c->cfg.model == SW_MODEL_MLQG) {
    // MultiLayerQG.energies: KE_j = parsevalsum(K²|ψ_j|²)/(2 Lx Ly) H_j/H,
    // PE = parsevalsum(|ψ₂ - ψ₁|²)/(2 Lx Ly) f₀²/g′/H
    const sw_config& k = c->cfg;
    const double Ht = k.H[0] + k.H[1];
    ke = norm * a[0] / (2 * g.Lx * g.Ly) * k.H[0] / Ht;
    ke2 = norm * a[1] / (2 * g.Lx * g.Ly) * k.H[1] / Ht;
    pe = norm * a[2] / (2 * g.Lx * g.Ly) * k.f0 * k.f0 / (k.b[0] - k.b[1]) / Ht;
  } else if (c->cfg.model == SW_MODEL_TY) {
    // thomasyamada/ThomasYamada.jl:333-345: plain parsevalsum2 values
    ke = norm * a[1];
    ke2 = norm * a[0];
    pe = norm * a[2];
  } else {
    ke = norm * a[0] / (g.Lx * g.Ly);
    ke2 = norm * a[1] / (g.Lx * g.Ly);
    pe = 1.0 / (2 * g.Lx * g.Ly) * c->p.F * norm * a[2];
  }
}

// Energy records [esums_n, diag_n) -> c->esums_host [rec][SW_NSUM] (each
// record is gathered once).  Single process: erec holds the sums.  One slab
// per process (collective): erec holds this rank's column sums
// [rec][kcl][SW_NSUM]; they are gathered, in chunks that fit the host staging
// of the host-staged transport, and added in global column order, so the
// result is bitwise the same for any decomposition.
static int gather_new_energy_sums(sw_ctx* c) {
  const int64_t n0 = c->esums_n, n1 = c->diag_n;
  c->esums_host.resize((size_t)n1 * SW_NSUM, 0.0);
  if (n1 <= n0) return 0;
  if (!c->dist) {
    HIPCHK(c, hipMemcpyAsync(c->esums_host.data() + (size_t)n0 * SW_NSUM, c->erec + (size_t)n0 * SW_NSUM,
                             (size_t)(n1 - n0) * SW_NSUM * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->esums_n = n1;
    return 0;
  }
  const size_t rec = rank_cols(c) * SW_NSUM;  // doubles per record and rank
  int64_t chunk = n1 - n0;
  if (c->hostx) chunk = std::max<int64_t>(1, std::min<int64_t>(chunk, c->hbytes / (c->P * rec * sizeof(double))));
  std::vector<double> all((size_t)chunk * rec * c->P);
  double* tmp = nullptr;
  HIPCHK(c, hipMalloc((void**)&tmp, all.size() * sizeof(double)));
  int rc = 0;
  for (int64_t r0 = n0; r0 < n1 && !rc; r0 += chunk) {
    const int64_t m = std::min(chunk, n1 - r0);
    const size_t per = (size_t)m * rec;
    rc = allgather(c, c->erec + (size_t)r0 * rec, tmp, per * sizeof(double));
    if (!rc && hipMemcpyAsync(all.data(), tmp, per * c->P * sizeof(double), hipMemcpyDeviceToHost, c->stream) !=
                   hipSuccess)
      rc = fail(c, SW_E_HIP, "energy gather copy failed");
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(c, SW_E_HIP, "energy gather sync failed");
    for (int64_t r = 0; r < m && !rc; ++r)
      sum_rank_cols(c, all.data(), per, (size_t)r * rec, c->esums_host.data() + (size_t)(r0 + r) * SW_NSUM);
  }
  (void)hipStreamSynchronize(c->stream);
  (void)hipFree(tmp);
  if (rc) return rc;
  c->esums_n = n1;
  return 0;
}

int sw_diag(sw_ctx* c, int32_t id, double* out) {
  if (!ready(c) || !out) return SW_E_STATE;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (id == SW_DIAG_NAN) {
    int h = 0;
    if (int rc = nan_flag(c, h)) return rc;
    *out = h ? 1.0 : 0.0;
    return SW_OK;
  }
  if (id == SW_DIAG_CFL) {
    // rsw/RSWDriver.jl:207-208, swqg/TwoLayerDriver.jl:100-101:
    // dt · max(maximum(|vars.u|)/dx, maximum(|vars.v|)/dy), both layers for 2LQG;
    // thomasyamada/TYdriver.jl:150: signed maxima of u_c, v_c, u_T, v_T
    const Geom& g0 = c->sl[0].g;
    // signed maxima: thomasyamada/TYdriver.jl:150, simulation/TwoLayerSimulation.jl:124
    const bool ty = c->cfg.model == SW_MODEL_TY || c->cfg.model == SW_MODEL_MLQG;
    const int nlay = c->cfg.model == SW_MODEL_RSW ? 1 : 2;
    unsigned long long* mx = reinterpret_cast<unsigned long long*>(c->flag + 512);  // [u, v] maxima keys
    HIPCHK(c, hipMemsetAsync(mx, 0, 2 * sizeof(unsigned long long), c->stream));
    const size_t off = c->dist ? (size_t)g0.y0 * g0.nx : 0;
    const long long n = (long long)(c->dist ? g0.nyl : g0.ny) * g0.nx;
    for (int layer = 0; layer < nlay; ++layer)
      for (int comp = 0; comp < 2; ++comp) {
        if (int rc = physical_to_dflt(c, layer * 8 + (comp == 0 ? SW_PHYS_U : SW_PHYS_V))) return rc;
        sw::launch_absmax(c->dflt + off, n, mx + comp, ty ? 1 : 0, c->stream);
      }
    HIPCHK(c, hipGetLastError());
    unsigned long long kmax[2] = {0, 0};
    if (c->dist) {
      std::vector<unsigned long long> all(2 * (size_t)c->P);
      if (int rc = allgather(c, mx, c->esum, 2 * sizeof(unsigned long long))) return rc;
      HIPCHK(c, hipMemcpyAsync(all.data(), c->esum, all.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (int q = 0; q < c->P; ++q) {
        kmax[0] = std::max(kmax[0], all[2 * q]);
        kmax[1] = std::max(kmax[1], all[2 * q + 1]);
      }
    } else {
      HIPCHK(c, hipMemcpyAsync(kmax, mx, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    *out = c->cfg.dt * std::max(key_double(kmax[0]) / g0.dx, key_double(kmax[1]) / g0.dy);
    return SW_OK;
  }
  const bool wgid = id >= SW_DIAG_WAVE_KE && id <= SW_DIAG_GEO_PE;
  if (id != SW_DIAG_KE && id != SW_DIAG_PE && id != SW_DIAG_KE1 && id != SW_DIAG_KE2 && id != SW_DIAG_BT && !wgid)
    return fail(c, SW_E_INVALID, "unknown diagnostic");
  if (((id == SW_DIAG_BT || wgid) && c->cfg.model != SW_MODEL_TY) ||
      ((id == SW_DIAG_KE1 || id == SW_DIAG_KE2) && c->cfg.model == SW_MODEL_TY))
    return fail(c, SW_E_INVALID, "diagnostic not defined for this model");
  int ncols = c->P * c->sl[0].g.kcl;
  if (c->gen) {
    sw::gen::energy_sums(c->gen, c->sl[0].sol, c->esum);
  } else {
  for (Slab& s : c->sl) sw::launch_energy_cols(c->cfg.model, s.g, c->p, s.sol, c->ecols + SW_NSUM * s.g.kr0, c->stream);
  if (c->dist) {
    const Slab& s = c->sl[0];
    const Geom& g0 = s.g;
    if (int rc = allgather(c, c->ecols + SW_NSUM * g0.kr0, c->ecols, SW_NSUM * (size_t)g0.kcl * sizeof(double))) return rc;
    if (alias_energy(c)) {
      // every rank's aliased columns, in the undecomposed order: region 0
      // (slab 0), then every slab's region 1 (padded to kcl: zeros)
      const size_t na = (size_t)(g0.nkr - g0.kc), kcl = g0.kcl, slot = (na + kcl) * SW_NSUM;
      double* ord = c->ecols + SW_NSUM * (size_t)ncols;
      double* scr = ord + SW_NSUM * (na + c->P * kcl);
      double* mine = scr + (size_t)g0.slab * slot;
      HIPCHK(c, hipMemsetAsync(mine, 0, slot * sizeof(double), c->stream));
      for (int r = 0; r < 2; ++r)
        if (s.ga[r].kcn > 0)
          sw::launch_energy_cols(c->cfg.model, s.ga[r], c->p, s.a_sol[r], mine + (r ? SW_NSUM * na : 0), c->stream);
      if (int rc = allgather(c, mine, scr, slot * sizeof(double))) return rc;
      HIPCHK(c, hipMemcpyAsync(ord, scr, SW_NSUM * na * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
      for (int q = 0; q < c->P; ++q)
        HIPCHK(c, hipMemcpyAsync(ord + SW_NSUM * (na + q * kcl), scr + q * slot + SW_NSUM * na,
                                 SW_NSUM * kcl * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
      ncols += (int)(na + c->P * kcl);
    }
  } else {
    ncols = alias_energy_cols(c, true, ncols);
  }
  sw::launch_energy_final(c->ecols, ncols, c->esum, c->stream);
  }
  HIPCHK(c, hipGetLastError());
  std::vector<double> sums(SW_NSUM);
  HIPCHK(c, hipMemcpyAsync(sums.data(), c->esum, SW_NSUM * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  double ke, ke2, pe, wg[4];
  energies_from_sums(c, sums.data(), ke, ke2, pe, wg);
  if (wgid) {
    *out = wg[id - SW_DIAG_WAVE_KE];
    return SW_OK;
  }
  // RSW KE; 2LQG KE = KE_1 + KE_2 (the driver's tuple summed), KE2 = KE_2;
  // TY: KE, PE the baroclinic pair, BT barotropic
  if (c->cfg.model == SW_MODEL_TY) *out = id == SW_DIAG_KE ? ke : (id == SW_DIAG_BT ? ke2 : pe);
  else if (id == SW_DIAG_KE) *out = ke + ke2;
  else if (id == SW_DIAG_KE1) *out = ke;
  else if (id == SW_DIAG_KE2) *out = ke2;
  else *out = pe;
  return SW_OK;
}

// stepforward!(prob, n) whose last step also yields the energies FF's
// Diagnostic functions read after it (the record semantics of
// sw_set_energy_diagnostics), for a caller that steps lazily and needs them at
// a diagnostic step (integration/julia/SWLib.jl, FF's increment!)
int sw_step_record(sw_ctx* c, int64_t nsteps, sw_energy_record* out) {
  if (!ready(c) || !out) return SW_E_STATE;
  if (nsteps < 1) return fail(c, SW_E_INVALID, "sw_step_record: nsteps must be >= 1");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const size_t per = c->dist ? rank_cols(c) * SW_NSUM : SW_NSUM;
  if (!c->erec1) {
    if (c->dist) {
      if (int rc = alloc(c, (void**)&c->erec1, per * sizeof(double))) return rc;
    } else {  // the record's sums land in pinned host memory: no copy after the steps (round 6)
      HIPCHK(c, hipHostMalloc((void**)&c->erec1_host, per * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent));
      HIPCHK(c, hipHostGetDevicePointer((void**)&c->erec1, c->erec1_host, 0));
    }
  }
  if (int rc = scan_arm(c)) return rc;
  for (int64_t i = 0; i + 1 < nsteps; ++i)
    if (int rc = step_once(c)) return rc;
  c->force_rec = true;
  const int rcs = step_once(c);
  c->force_rec = false;
  if (rcs) return rcs;
  if (int rc = join_comm(c)) return rc;
  HIPCHK(c, hipGetLastError());
  std::vector<double> sums(SW_NSUM, 0.0);
  if (c->dist) {  // collective: every rank's column sums, added in global column order
    std::vector<double> all(per * c->P);
    double* tmp = nullptr;
    HIPCHK(c, hipMalloc((void**)&tmp, all.size() * sizeof(double)));
    int rc = allgather(c, c->erec1, tmp, per * sizeof(double));
    if (!rc && hipMemcpyAsync(all.data(), tmp, all.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream) !=
                   hipSuccess)
      rc = fail(c, SW_E_HIP, "energy record copy failed");
    if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(c, SW_E_HIP, "energy record sync failed");
    (void)hipFree(tmp);
    if (rc) return rc;
    sum_rank_cols(c, all.data(), per, 0, sums.data());
  } else {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const volatile double* hs = c->erec1_host;
    for (int k = 0; k < SW_NSUM; ++k) sums[k] = hs[k];
  }
  out->step = c->step;
  out->t = c->t;
  energies_from_sums(c, sums.data(), out->ke, out->ke2, out->pe, out->wg);
  if (c->scan) {
    int h = 0;
    if (int rc = scan_read(c, h)) return rc;
    if (h) return fail(c, SW_E_NAN, "Solution is NaN");
  }
  return SW_OK;
}

// The slab exchange explained (multi-GPU bench lines): nsteps steps of the
// production schedule, each timed on the compute stream, with the time that
// stream spent waiting for transposes (wait_comm; the sequential schedule's
// transposes in full) and the bytes this slab sent.
int sw_get_link_model(const sw_ctx* c, sw_link_model* out) {
  if (!ready(c) || !out) return SW_E_STATE;
  *out = c->link;
  return SW_OK;
}

int sw_comm_profile(sw_ctx* c, int64_t nsteps, sw_comm_stats* out) {
  if (!ready(c) || !out) return SW_E_STATE;
  if (nsteps < 1) return fail(c, SW_E_INVALID, "sw_comm_profile: nsteps must be >= 1");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (c->wev.empty()) {
    c->wev.resize(256);
    for (hipEvent_t& e : c->wev) HIPCHK(c, hipEventCreate(&e));
  }
  if (int rc = join_comm(c)) return rc;
  double step_ms = 0.0, wait_ms = 0.0;
  c->xbytes = 0.0;
  int rc = 0;
  for (int64_t i = 0; i < nsteps && !rc; ++i) {
    c->time_waits = true;
    c->nwait = 0;
    if (hipEventRecord(c->ev0, c->stream) != hipSuccess) rc = fail(c, SW_E_HIP, "event record failed");
    if (!rc) rc = step_once(c);
    if (!rc) rc = join_comm(c);
    c->time_waits = false;
    if (rc) break;
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    HIPCHK(c, hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    step_ms += ms;
    for (int k = 0; k + 1 < c->nwait; k += 2) {
      HIPCHK(c, hipEventElapsedTime(&ms, c->wev[k], c->wev[k + 1]));
      wait_ms += ms;
    }
  }
  c->time_waits = false;
  if (rc) return rc;
  HIPCHK(c, hipGetLastError());
  out->nranks = c->P;
  out->transport = c->P == 1 ? SW_XPORT_NONE : (!c->dist ? SW_XPORT_LOCAL : (c->hostx ? SW_XPORT_HOST : SW_XPORT_RCCL));
  int cnt = 0;
  if (c->nccl) NCCLCHK(c, ncclCommCount(c->nccl, &cnt));
  out->rccl_ranks = cnt;
  out->pipelined = pipelined(c) ? 1 : 0;
  out->row_chunks = pipelined(c) ? c->row_chunks : 1;
  out->reserved = 0;
  out->step_us = step_ms * 1e3 / nsteps;
  out->exposed_us = wait_ms * 1e3 / nsteps;
  out->bytes_sent = c->xbytes / nsteps;
  return SW_OK;
}

int sw_set_energy_diagnostics(sw_ctx* c, int64_t freq, int64_t capacity) {
  if (!ready(c)) return SW_E_STATE;
  if (freq < 0 || capacity < 0) return fail(c, SW_E_INVALID, "freq and capacity must be >= 0");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->erec) (void)hipFree(c->erec);
  c->erec = nullptr;
  c->diag_freq = freq;
  c->diag_cap = freq > 0 ? capacity : 0;
  c->diag_n = 0;
  c->diag_steps.clear();
  c->diag_t.clear();
  c->esums_host.clear();
  c->esums_n = 0;
  if (c->diag_cap > 0) {
    const size_t per = c->dist ? rank_cols(c) * SW_NSUM : SW_NSUM;
    if (int rc = alloc(c, (void**)&c->erec, (size_t)c->diag_cap * per * sizeof(double))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return SW_OK;
}

int sw_get_energy_diagnostics(sw_ctx* c, sw_energy_record* out, int64_t max_records, int64_t* n_records) {
  if (!ready(c)) return SW_E_STATE;
  if (max_records < 0 || (max_records > 0 && !out)) return fail(c, SW_E_INVALID, "bad record buffer");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (max_records == 0) {  // query: the number of records held
    if (n_records) *n_records = c->diag_n;
    return SW_OK;
  }
  const int64_t n = std::min<int64_t>(c->diag_n, max_records);
  // one slab per process: every rank gathers the new records (collective)
  if (int rc = gather_new_energy_sums(c)) return rc;
  for (int64_t r = 0; r < n; ++r) {
    out[r].step = c->diag_steps[r];
    out[r].t = c->diag_t[r];
    energies_from_sums(c, &c->esums_host[(size_t)SW_NSUM * r], out[r].ke, out[r].ke2, out[r].pe, out[r].wg);
  }
  if (n_records) *n_records = n;
  return SW_OK;
}

int sw_profile_steps(sw_ctx* c, int64_t nsteps, sw_kernel_stat* out, int32_t max_stats, int32_t* n_stats) {
  if (!ready(c)) return SW_E_STATE;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  for (auto& s : c->stats) {
    s.launches = 0;
    s.ms = 0.0;
  }
  if (int rc = join_comm(c)) return rc;
  const char* ce = std::getenv("SW_PROF_COLD");
  if (ce && ce[0] == '1' && !c->cold) {
    if (int rc = alloc(c, (void**)&c->cold, kColdBytes)) return rc;
    if (int rc = alloc(c, (void**)&c->cold_out, 64)) return rc;
  }
  if (!(ce && ce[0] == '1') && c->cold) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->cold);
    (void)hipFree(c->cold_out);
    c->cold = nullptr;
    c->cold_out = nullptr;
  }
  if (c->pev.empty()) {
    c->pev.resize(2 * kProfPairs);
    c->pkid.resize(kProfPairs);
    for (hipEvent_t& e : c->pev) HIPCHK(c, hipEventCreate(&e));
  }
  c->npev = 0;
  c->prof = true;
  int rc = 0;
  for (int64_t i = 0; i < nsteps && !rc; ++i) rc = step_once(c);
  c->prof = false;
  if (rc) {
    (void)hipStreamSynchronize(c->stream);
    c->npev = 0;
    return rc;
  }
  HIPCHK(c, hipGetLastError());
  prof_flush(c);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int n = 0;
  for (int i = 0; i < K_NKERN && n < max_stats; ++i) {
    if (c->stats[i].launches == 0) continue;
    std::snprintf(out[n].name, sizeof(out[n].name), "%s", c->stats[i].name);
    out[n].launches = c->stats[i].launches;
    out[n].avg_ms = c->stats[i].ms / c->stats[i].launches;
    // one transpose stat = one direction; kernel_bytes(K_XCHG) counts both
    out[n].alg_bytes = i == K_XCHG ? kernel_bytes(c, i) / 2 : kernel_bytes(c, i);
    ++n;
  }
  if (n_stats) *n_stats = n;
  return SW_OK;
}

double sw_step_alg_bytes(const sw_ctx* c) {
  if (!ready(c)) return 0.0;
  if (c->gen) return gen_step_bytes(c);
  return step_bytes(c);
}

// the ring slot holding RHS/N of `slot` steps ago (1 or 2), -1 if none
static int hist_index(const sw_ctx* c, int32_t slot) {
  const int st = c->cfg.stepper;
  if ((st != SW_STEP_FILTERED_AB3 && st != SW_STEP_IFMAB3) || slot < 1 || slot > 2) return -1;
  return (c->head + 3 - slot) % 3;  // step_ptrs: h1 = hist[(head+2)%3], h2 = hist[(head+1)%3]
}

int sw_history_slots(const sw_ctx* c, int32_t* nslots) {
  if (!ready(c) || !nslots) return SW_E_STATE;
  const int st = c->cfg.stepper;
  *nslots = (st == SW_STEP_FILTERED_AB3 || st == SW_STEP_IFMAB3) ? 2 : 0;
  return SW_OK;
}

int sw_get_history(const sw_ctx* cc, int32_t slot, void* buf, size_t bytes) {
  sw_ctx* c = const_cast<sw_ctx*>(cc);
  if (!ready(c)) return SW_E_STATE;
  const int h = hist_index(c, slot);
  if (h < 0) return fail(c, SW_E_INVALID, "sw_get_history: no such history slot for this stepper");
  if (!buf || bytes != caller_bytes(c, full_bytes(c))) return fail(c, SW_E_INVALID, "sw_get_history: size mismatch");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = join_comm(c)) return rc;
  for (Slab& s : c->sl) s.view = s.hist[h];
  if (int rc = collect_full(c, &Slab::view)) return rc;
  if (int rc = alias_scatter(c, a_hist(h))) return rc;
  if (int rc = download(c, c->stage, buf, full_bytes(c))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return SW_OK;
}

int sw_set_history(sw_ctx* c, int32_t slot, const void* buf, size_t bytes) {
  if (!ready(c)) return SW_E_STATE;
  const int h = hist_index(c, slot);
  if (h < 0) return fail(c, SW_E_INVALID, "sw_set_history: no such history slot for this stepper");
  if (!buf || bytes != caller_bytes(c, full_bytes(c))) return fail(c, SW_E_INVALID, "sw_set_history: size mismatch");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = join_comm(c)) return rc;
  if (int rc = upload(c, buf, c->stage, full_bytes(c))) return rc;
  for (Slab& s : c->sl) sw::launch_gather(c->nf, s.g, c->stage, s.hist[h], c->stream);
  alias_gather(c, a_hist(h));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->euler_left = 0;  // the history is valid again: AB3 from the next step (clock.step >= 3)
  return SW_OK;
}

int sw_reset_history(sw_ctx* c) {
  if (!ready(c)) return SW_E_STATE;
  c->euler_left = 3;
  return SW_OK;
}

// --- fp64 restart blob (sw_checkpoint_bytes / sw_get_checkpoint / sw_set_checkpoint)
namespace {
struct CkptHeader {
  char magic[8];                       // "SWCKPT01"
  int32_t abi, model, stepper, nx, ny, nf, nslots, euler_left;
  double t;
  int64_t step;
  int64_t aliased_state;                // the context's sw_config.aliased_state (ABI 9; 0 before)
};
static_assert(sizeof(CkptHeader) == 64, "checkpoint header is 64 bytes");
const char kCkptMagic[8] = {'S', 'W', 'C', 'K', 'P', 'T', '0', '1'};

int ckpt_slots(const sw_ctx* c) {
  const int st = c->cfg.stepper;
  return (st == SW_STEP_FILTERED_AB3 || st == SW_STEP_IFMAB3) ? 2 : 0;
}
size_t ckpt_bytes(const sw_ctx* c) { return sizeof(CkptHeader) + (size_t)(1 + ckpt_slots(c)) * full_bytes(c); }
}  // namespace

int sw_checkpoint_bytes(const sw_ctx* c, size_t* bytes) {
  if (!ready(c) || !bytes) return SW_E_STATE;
  *bytes = ckpt_bytes(c);
  return SW_OK;
}

int sw_get_checkpoint(const sw_ctx* cc, void* buf, size_t bytes) {
  sw_ctx* c = const_cast<sw_ctx*>(cc);
  if (!ready(c)) return SW_E_STATE;
  if (!buf || bytes != ckpt_bytes(c)) return fail(c, SW_E_INVALID, "sw_get_checkpoint: size mismatch");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = join_comm(c)) return rc;
  CkptHeader h{};
  std::memcpy(h.magic, kCkptMagic, 8);
  h.abi = SW_ABI_VERSION;
  h.model = c->cfg.model;
  h.stepper = c->cfg.stepper;
  h.nx = c->cfg.nx;
  h.ny = c->cfg.ny;
  h.nf = c->nf;
  h.nslots = ckpt_slots(c);
  h.euler_left = c->euler_left;
  h.t = c->t;
  h.step = c->step;
  h.aliased_state = c->alias ? 1 : 0;
  char* out = static_cast<char*>(buf);
  std::memcpy(out, &h, sizeof(h));
  const size_t fb = full_bytes(c);
  for (int k = 0; k <= h.nslots; ++k) {  // fp64 always: no narrowing to the caller precision
    if (k == 0) {
      if (int rc = collect_full(c, &Slab::sol)) return rc;
      if (int rc = alias_scatter(c, A_SOL)) return rc;
    } else {
      const int hi = hist_index(c, k);
      for (Slab& s : c->sl) s.view = s.hist[hi];
      if (int rc = collect_full(c, &Slab::view)) return rc;
      if (int rc = alias_scatter(c, a_hist(hi))) return rc;
    }
    HIPCHK(c, hipMemcpyAsync(out + sizeof(h) + k * fb, c->stage, fb, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return SW_OK;
}

// any nonzero (nkr, nl, nf) mode of the blob's state or history outside the
// 2/3-rule live set (kr >= kc, or l in [lc, lr2)): only an aliased_state
// context writes those
static bool ckpt_has_aliased_modes(const sw_ctx* c, const CkptHeader& h, const void* buf) {
  const sw::Geom& g = c->sl[0].g;
  const double* d = reinterpret_cast<const double*>(static_cast<const char*>(buf) + sizeof(CkptHeader));
  const size_t nkr = g.nkr, nl = g.nl;
  for (int k = 0; k <= h.nslots; ++k)
    for (int f = 0; f < c->nf; ++f)
      for (size_t l = 0; l < nl; ++l) {
        const bool dead_row = (int)l >= g.lc && (int)l < g.lr2;
        const double* row = d + 2 * (((size_t)(k * c->nf + f) * nl + l) * nkr);
        for (size_t kr = dead_row ? 0 : (size_t)g.kc; kr < nkr; ++kr)
          if (row[2 * kr] != 0.0 || row[2 * kr + 1] != 0.0) return true;
      }
  return false;
}

int sw_set_checkpoint(sw_ctx* c, const void* buf, size_t bytes) {
  if (!ready(c)) return SW_E_STATE;
  if (!buf || bytes != ckpt_bytes(c)) return fail(c, SW_E_INVALID, "sw_set_checkpoint: size mismatch");
  CkptHeader h;
  std::memcpy(&h, buf, sizeof(h));
  if (std::memcmp(h.magic, kCkptMagic, 8) != 0) return fail(c, SW_E_INVALID, "sw_set_checkpoint: not a libsw checkpoint");
  // the blob layout is that of ABI 7 (its introduction) up to this one
  if (h.abi < 7 || h.abi > SW_ABI_VERSION) return fail(c, SW_E_INVALID, "sw_set_checkpoint: unknown checkpoint ABI");
  // the problem first: the aliased-mode scan below reads
  // h.nslots + 1 arrays, which bytes == ckpt_bytes(c) bounds only for a blob
  // of this problem and stepper
  if (h.model != c->cfg.model || h.stepper != c->cfg.stepper || h.nx != c->cfg.nx || h.ny != c->cfg.ny ||
      h.nf != c->nf || h.nslots != ckpt_slots(c) || h.step < 0 || h.euler_left < 0 || h.euler_left > 3)
    return fail(c, SW_E_INVALID, "sw_set_checkpoint: checkpoint of a different problem or stepper");
  // an aliased-state blob carries modes a default context drops: that one
  // does not continue bitwise.  Before ABI 9 the header's field
  // was reserved (0) whatever the writer tracked: the blob's own
  // aliased modes tell — nonzero only where the writer tracked them.  A blob
  // whose aliased modes are all zero is valid for either context (a default
  // context's, or an aliased_state one's before its first step from a
  // dealiased state: ADVICE r05), so only the unambiguous case is refused.
  if (h.abi >= 9) {
    if (h.aliased_state != (c->alias ? 1 : 0))
      return fail(c, SW_E_INVALID, "sw_set_checkpoint: aliased_state differs from the checkpoint's");
  } else if (!c->alias && ckpt_has_aliased_modes(c, h, buf)) {
    return fail(c, SW_E_INVALID,
                "sw_set_checkpoint: an ABI < 9 checkpoint holding aliased modes (written with aliased_state) "
                "into a context without aliased_state");
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = join_comm(c)) return rc;
  const char* in = static_cast<const char*>(buf);
  const size_t fb = full_bytes(c);
  for (int k = 0; k <= h.nslots; ++k) {
    HIPCHK(c, hipMemcpyAsync(c->stage, in + sizeof(h) + k * fb, fb, hipMemcpyHostToDevice, c->stream));
    if (c->gen) {  // (FilteredRK4: the state alone)
      HIPCHK(c, hipMemcpyAsync(c->sl[0].sol, c->stage, fb, hipMemcpyDeviceToDevice, c->stream));
      sw::gen::dealias(c->gen, c->sl[0].sol);
    } else {
      for (Slab& s : c->sl)
        sw::launch_gather(c->nf, s.g, c->stage, k == 0 ? s.sol : s.hist[hist_index(c, k)], c->stream);
    }
    if (k == 0) alias_gather(c, A_SOL);
    else alias_gather(c, a_hist(hist_index(c, k)));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));  // the staging buffer is reused
  }
  c->t = h.t;
  c->step = h.step;
  c->euler_left = h.euler_left;
  c->mixed_valid = false;
  return SW_OK;
}

int sw_slab_geometry(const sw_config* cfg, int32_t slab, int32_t out[8]) {
  if (!cfg || !out || cfg->abi_version != SW_ABI_VERSION) return SW_E_INVALID;
  const int P = cfg->nranks < 1 ? 1 : cfg->nranks;
  if (!pow2(P) || !pow2(cfg->nx) || !pow2(cfg->ny) || cfg->nx < 32 || cfg->ny < 32 || cfg->nx > 8192 ||
      cfg->ny > 8192 || slab < 0 || slab >= P || !(cfg->aliased_fraction >= 0 && cfg->aliased_fraction < 1))
    return SW_E_INVALID;
  const Geom g = make_geom(*cfg, P, slab);
  const int32_t v[8] = {g.kc, g.kcl, g.kr0, g.kcn, g.nyl, g.y0, g.Lr, g.LrP};
  std::memcpy(out, v, sizeof(v));
  return SW_OK;
}

int sw_comm_unique_id(void* out128) {
  if (!out128) return SW_E_INVALID;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return SW_E_COMM;
  std::memcpy(out128, &id, sizeof(id));
  return SW_OK;
}

}  // extern "C"
