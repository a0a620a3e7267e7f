// libsw generic engine: grids whose sizes are not powers of two.
//
// The pseudo-spectral path of sw_kernels.hip is built around power-of-two
// line transforms (radix-2/4/8 Stockham, 8 points per thread, 2×4 mixed
// tiles, slab transposes).  The reference's parameter files set one grid that
// is not: simulation/MattParameters.jl:8, nx = 384 = 3·2⁷, for
// TwoLayerSimulation (GeophysicalFlows MultiLayerQG, 2 layers, FilteredRK4,
// aliased_fraction = 0; VERDICT r05 missing #4).  This engine runs that
// model/stepper pair on any even grid of 2^a·3^b·5^c points per side (16 …
// 3328): mixed-radix (2, 3, 4, 5) Stockham line transforms in LDS, the
// state on the full (nkr, nl) array (Julia's prob.sol layout, the aliased
// modes held at zero as libsw's default mode does), the calcN as the
// reference's op sequence (simulation/TwoLayerSimulation.jl:37-47; GF
// calcN_advection! + bottom drag, oracle/sw_oracle.py mlqg_calcN), the FF
// FilteredRK4 stages (op_frk4's arithmetic), energies, physical fields and
// the NaN scan on the device.  Correctness first: these grids are small (384²
// is 0.15 M points); each pass is a plain kernel per transform direction.
#pragma once
#include <string>

#include "sw.h"
#include "sw_internal.hpp"

namespace sw {
namespace gen {

// n = 2^a 3^b 5^c (even, 16 … 4096): the radix sequence (4s, then 2, 3s,
// 5s) into rad; returns the count, 0 if n does not factor
int radices(int n, int rad[24]);

struct Engine {
  Geom g{};      // nx, ny, nkr, nl, Lx, Ly, mk, ml, dx, dy, kc, lc, lr2 (mode-wise helpers)
  Phys p{};
  int radx[24]{}, nradx = 0, rady[24]{}, nrady = 0;
  hipStream_t s = nullptr;
  double2* sol = nullptr;   // state [2][nl][nkr] (the caller's Slab owns it)
  double2* xs = nullptr;    // RK4 stage input
  double2* acc = nullptr;   // RK4 accumulator
  double2* N = nullptr;     // calcN output
  double2* spec = nullptr;  // 6 spectral work fields [6][nl][nkr]
  double* phys = nullptr;   // 6 physical work fields [6][ny][nx]
  double* cols = nullptr;   // energy column sums [nkr][3]
  double2* twx = nullptr;   // forward twiddles exp(-2πi j/nx), j < nx
  double2* twy = nullptr;   // … along y
  int bx = 1;               // rows per block of the x transforms
  bool fused = false;       // three kernels per stage (k_gcol_inv, k_grow, k_gcol_fwd)
  double2* xs2 = nullptr;   // the fused stages' second stage-input buffer
  bool ct = true;           // compile-time fused kernels for the lengths that have them (SW_GEN_CT)
  bool graph_on = false;    // the fused step replayed as a hipGraph (SW_GEN_GRAPH)
  hipGraphExec_t gexec = nullptr;
  int* gflag = nullptr;     // the blow-up flag the graph was captured with
};

int create(Engine*& e, const sw_config& k, const Phys& p, const Geom& g, double2* sol, hipStream_t s,
           std::string& err);
void destroy(Engine* e);
// N = calcN(dealias(X)) on the full array (aliased modes of N: 0)
void calcN(Engine* e, const double2* X, double2* N);
// one FilteredRK4 step of e->sol; nanflag: the blow-up flag (StepPtrs::nan) or null
void step(Engine* e, int* nanflag);
// X -> X with the aliased modes zeroed (dealias!)
void dealias(Engine* e, double2* X);
// updatevars! field fid (8·layer + SW_PHYS_{U,V,ZETA,Q,PSI}) of X into out [ny][nx]
void physical(Engine* e, const double2* X, int fid, double* out);
// the MultiLayerQG energy sums of X, in energies_from_sums' layout (a[0..2]; SW_NSUM doubles)
void energy_sums(Engine* e, const double2* X, double* out);
// NaN/Inf anywhere in X: flag := 1
void nan_scan(Engine* e, const double2* X, int* flag);

}  // namespace gen
}  // namespace sw
