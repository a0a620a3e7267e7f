/*
 * libsw — MI355X-native pseudo-spectral time-step core (C ABI).
 *
 * Drop-in boundary for the per-timestep hot path of ndefilippis/JuliaRaytracingSW
 * (SURVEY.md §8b).  The reference plugs a time stepper into FourierFlows by
 * defining
 *     FourierFlows.stepforward!(sol, clock, ts::IFMAB3TimeStepper, equation,
 *                               vars, params, grid)          utils/IFMAB3.jl:157
 * which calls equation.calcN!(N, sol, t, clock, vars, params, grid)
 * (rsw/RotatingShallowWater.jl:140, swqg/TwoLayerQG.jl:152).  Drivers call
 * FF's stepforward!(prob, diags, nsteps) (rsw/RSWDriver.jl:212,
 * swqg/TwoLayerDriver.jl:105).  Every entry point below replaces one of those
 * seams; a Julia `ccall` shim binding them is given in INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only; no exceptions cross the ABI.
 *  - Host buffers hold fp64 (or, with sw_config.precision = SW_PREC_F32,
 *    fp32) elements; sizes below are for fp64 and halve for fp32.
 *  - Return codes: 0 = ok, < 0 = error (see SW_E_*); sw_last_error() has text.
 *  - Spectral state layout = Julia column-major (nkr, nl, nfield) of interleaved
 *    complex (re, im) doubles: element (kr, l, f) at ((f*nl + l)*nkr + kr).
 *    Byte-identical to a Julia Array{ComplexF64,3} `prob.sol`.
 *  - Physical fields: Julia (nx, ny) column-major doubles, x fastest.
 *  - The library owns all device memory.  Caller buffers are host memory and
 *    are copied synchronously.  A context is driven by one host thread.
 */
#ifndef SW_H
#define SW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SW_ABI_VERSION 9

/* models */
#define SW_MODEL_RSW 0   /* rsw/RotatingShallowWater.jl: fields (u, v, η), 3×3 L   */
#define SW_MODEL_QG2 1   /* swqg/TwoLayerQG.jl: fields (q1, q2), 2×2 L             */
#define SW_MODEL_TY  2   /* thomasyamada/ThomasYamada.jl: fields (ζ_T, u_c, v_c, p_c),
                            real diagonal L = -ν K^(2nν), stepper ETDRK4 */
#define SW_MODEL_MLQG 3  /* GeophysicalFlows MultiLayerQG, nlayers = 2, as
                            simulation/TwoLayerSimulation.jl:37-47 builds it: fields
                            (q1, q2); aliased_fraction may be 0 (the reference's) */

/* steppers */
#define SW_STEP_FILTERED_AB3 0 /* FF FilteredAB3 with per-mode matvec L·sol */
#define SW_STEP_IFMAB3       1 /* utils/IFMAB3.jl:68-169                               */
#define SW_STEP_IFMRK4       2 /* Lawson IF-RK4, the build's definition of utils/IFMRK4.jl (A9) */
#define SW_STEP_ETDRK4       3 /* FF ETDRK4TimeStepper (ThomasYamada.Problem default, :60) */
#define SW_STEP_FILTERED_RK4 4 /* FF FilteredRK4 (simulation/Parameters.jl:25), RSW/QG2/MLQG */

/* caller-buffer precision (sw_config.precision): the element type of every
 * host buffer crossing the ABI (state, calcN, history, physical fields).  The
 * reference's production drivers run T = Float32 (rsw/RSWDriver.jl:164,
 * swqg/TwoLayerDriver.jl:63): with SW_PREC_F32 their ComplexF32 `prob.sol` and
 * Float32 `vars` arrays are exchanged as they are; libsw computes in fp64
 * either way and rounds once on the way out. */
#define SW_PREC_F64 0    /* ComplexF64 / Float64 buffers (16 / 8 bytes)       */
#define SW_PREC_F32 1    /* ComplexF32 / Float32 buffers (8 / 4 bytes)        */

/* error codes */
#define SW_OK            0
#define SW_E_INVALID    -1  /* bad argument / unsupported configuration   */
#define SW_E_NOMEM      -2  /* device allocation failed                   */
#define SW_E_HIP        -3  /* HIP runtime error                          */
#define SW_E_COMM       -4  /* RCCL error                                 */
#define SW_E_NAN        -5  /* NaN/Inf detected in the state after a step */
#define SW_E_STATE      -6  /* call out of order                          */

/* physical-field ids for sw_get_physical (updatevars! equivalents)
 * RSW (rsw/RotatingShallowWater.jl:101-116): u, v, η, ζ=∂x v − ∂y u − f η
 * QG2 (swqg/TwoLayerQG.jl:113-129), per layer (layer = id / 8): q, ψ, ζ, u, v
 * TY  (thomasyamada/ThomasYamada.jl:67-92): 0 u_c, 1 v_c, 2 p_c, 3 ζ_T, 4 q_c,
 *     5 ψ_T, 8 u_T, 9 v_T */
#define SW_PHYS_U     0
#define SW_PHYS_V     1
#define SW_PHYS_ETA   2
#define SW_PHYS_ZETA  3
#define SW_PHYS_Q     4
#define SW_PHYS_PSI   5

/* diagnostic ids for sw_diag */
#define SW_DIAG_NAN   0  /* 1.0 if any NaN/Inf in the state              */
#define SW_DIAG_KE    1  /* RSW: kinetic_energy; QG2: KE layer 1 + layer 2 */
#define SW_DIAG_PE    2  /* potential_energy                              */
#define SW_DIAG_CFL   3  /* clock.dt · max(max|u|/dx, max|v|/dy) of the physical
                            velocities, both layers for QG2 (rsw/RSWDriver.jl:207-208,
                            swqg/TwoLayerDriver.jl:100-101)                  */
#define SW_DIAG_KE2   4  /* QG2: KE of layer 2 alone (the tuple's 2nd entry) */
#define SW_DIAG_KE1   5  /* QG2: KE of layer 1 alone (the tuple's 1st entry) */
/* TY (thomasyamada/ThomasYamada.jl:333-345): SW_DIAG_KE = baroclinic_energy[1]
 * (|u_c|² + |v_c|²), SW_DIAG_PE = baroclinic_energy[2] (|p_c|²), SW_DIAG_BT =
 * barotropic_energy; SW_DIAG_CFL = dt · max of maximum(u_c)/dx, maximum(v_c)/dy,
 * maximum(u_T)/dx, maximum(v_T)/dy (signed maxima, thomasyamada/TYdriver.jl:150) */
#define SW_DIAG_BT    6
/* TY wave_geostrophic_energy (thomasyamada/ThomasYamada.jl:353-367, the
 * TYUtils.jl:40-51 balanced/wave split of (u_c, v_c, p_c)), reduced on the
 * device: ((WAVE_KE, WAVE_PE), (GEO_KE, GEO_PE)) */
#define SW_DIAG_WAVE_KE 7
#define SW_DIAG_WAVE_PE 8
#define SW_DIAG_GEO_KE  9
#define SW_DIAG_GEO_PE  10

/* Host-staged transport (optional, one slab per process).  When set, libsw
 * moves every inter-slab exchange through host memory and calls
 *     exchange(user, send, recv, block_bytes, nranks)
 * instead of RCCL: `send` holds nranks contiguous blocks of block_bytes, block
 * q destined for rank q; on return block p of `recv` must hold the block rank
 * p sent to this rank (an all-to-all, e.g. MPI_Alltoall or a gloo
 * all_to_all).  Return 0 on success.  Used where RCCL cannot run (several
 * ranks on one GPU, CPU interconnect tests); results are bitwise identical. */
typedef int (*sw_exchange_fn)(void* user, const void* send, void* recv, size_t block_bytes,
                              int32_t nranks);

typedef struct sw_config {
  int32_t abi_version;      /* must be SW_ABI_VERSION                      */
  int32_t model;            /* SW_MODEL_*                                  */
  int32_t stepper;          /* SW_STEP_*                                   */
  int32_t nx, ny;           /* grid points (powers of two, 16 … 8192)      */
  double  Lx, Ly;           /* domain lengths                              */
  double  aliased_fraction; /* FF TwoDGrid aliased_fraction, in (0,1)      */
  double  dt;               /* time step                                   */
  /* physics — RSW Params (rsw/RotatingShallowWater.jl:18-23)              */
  double  f, Cg;            /* Coriolis, gravity-wave speed (Cg2 = Cg²)    */
  double  nu;               /* hyperviscosity ν                            */
  int32_t nnu;              /* hyperviscous order nν                       */
  /* physics — QG2 Params (swqg/TwoLayerQG.jl:23-30)                       */
  double  U, mu, F;         /* shear, bottom drag, F = 2f0²/Cg²/δρρ0       */
  /* filter — FF makefilter kwargs (utils/IFMAB3.jl:80-84)                 */
  int32_t use_filter;       /* IF steppers only; FilteredAB3 always filters */
  int32_t filter_order;
  double  filter_innerK, filter_outerK, filter_tol;
  /* device / multi-GPU                                                    */
  int32_t device;           /* HIP device ordinal                          */
  int32_t check_nan;        /* if nonzero, sw_step returns SW_E_NAN on blow-up */
  int32_t nop_calcN;        /* 1: N ≡ 0, the reference's NOPcalcN! hook
                               (rsw/RotatingShallowWater.jl:135-138,305)    */
  int32_t unfused;          /* debug/reference: separate col_fwd + update +
                               col_inv kernels instead of the fused column
                               pass (results are bitwise identical)        */
  /* slab decomposition: the grid is split into nranks slabs
   * (kr columns for the column passes, y rows for the row pass).
   *   local_slabs <= 1: this process holds slab `rank` on `device`; the
   *     transposes are RCCL all-to-alls over comm_unique_id (nranks > 1).
   *   local_slabs == nranks: this process holds every slab on `device`; the
   *     transposes are device copies (same data movement, one GPU).
   * nranks must be a power of two with ny / nranks >= 32.                 */
  int32_t nranks, rank, local_slabs;
  const void* comm_unique_id; /* ncclUniqueId bytes (128), from sw_comm_unique_id */
  sw_exchange_fn exchange;    /* optional host-staged transport instead of RCCL */
  void* exchange_user;
  /* physics — TY Params (thomasyamada/ThomasYamada.jl:21-25)               */
  double  Ro;               /* Rossby number                               */
  /* physics — MLQG (GeophysicalFlows MultiLayerQG.Problem keywords, 2 layers;
   * μ, ν, nν above): f₀, β, rest depths H, buoyancies b (g′ = b₁ − b₂) and
   * imposed zonal flows U per layer                                        */
  double  f0, beta;
  double  H[2], b[2], Ulayer[2];
  /* caller-buffer element type (SW_PREC_*), the reference's `T`            */
  int32_t precision;
  /* 1: also carry the modes the 2/3 rule removes (RSW or 2LQG with IFMAB3,
   * IFMRK4 or FilteredAB3, Thomas-Yamada with ETDRK4, MultiLayerQG with
   * FilteredRK4 or FilteredAB3 — with aliased_fraction = 0 the Nyquist
   * column and row GF's calcN!/updatevars! dealias!; nx up to 8192; one
   * slab, several slabs in one process, or one slab per process (the aliased
   * columns' row-pass x-spectra all-gathered per calcN); RSW then runs its
   * calcN in the reference's advective form).  The reference's calcN!
   * returns N there (swqg/TwoLayerQG.jl:171,179; rsw/RotatingShallowWater.jl
   * :140-230) and its update writes them into prob.sol (utils/IFMAB3.jl
   * :142-160) until the next calcN!/updatevars! dealiases: sw_calcN,
   * sw_get_state, the history/checkpoint I/O and the 2LQG/TY/MLQG energy
   * diagnostics (records and sw_diag; RSW's read the dealiased vars.uh) then
   * cover the full array, as the reference's do.  Off (0, the default): live
   * modes only, zeros elsewhere.  sw_get_physical
   * (updatevars!) clears them. */
  int32_t aliased_state;
} sw_config;

typedef struct sw_ctx sw_ctx;

typedef struct sw_kernel_stat {
  char    name[48];
  int64_t launches;
  double  avg_ms;          /* mean HIP-event duration per launch           */
  double  alg_bytes;       /* algorithmic HBM bytes per launch */
} sw_kernel_stat;

/* Fill *cfg with the reference defaults (RotatingShallowWater.Problem, :70-85). */
void sw_config_default(sw_config* cfg);

/* Problem(dev; …) + Equation + XTimeStepper construction
 * (rsw/RotatingShallowWater.jl:70-99, swqg/TwoLayerQG.jl:55-90,
 *  utils/IFMAB3.jl:68-88).  State and history start at zero, clock at 0. */
int sw_create(sw_ctx** ctx, const sw_config* cfg);
void sw_destroy(sw_ctx* ctx);
const char* sw_last_error(const sw_ctx* ctx);

/* sizes: nkr, nl, nfield (for the caller's buffers) */
int sw_get_dims(const sw_ctx* ctx, int32_t* nkr, int32_t* nl, int32_t* nfield);

/* set_solution! (rsw/RotatingShallowWater.jl:309-321, swqg/TwoLayerQG.jl:220-228):
 * copies `sol` (column-major (nkr,nl,nf) complex128) and dealiases it. */
int sw_set_state(sw_ctx* ctx, const void* sol, size_t bytes);
/* Array(prob.sol): the (dealiased) state, aliased modes = 0. */
int sw_get_state(const sw_ctx* ctx, void* sol, size_t bytes);

/* The stepper's memory across steps, for checkpoint/restart with bitwise
 * continuation (the reference keeps it in the TimeStepper: FF FilteredAB3's
 * RHS₋₁/RHS₋₂, utils/IFMAB3.jl:15-18 N₋₁/N₋₂, rotated at :165-166).
 * sw_history_slots: 2 for FilteredAB3 / IFMAB3 (slot 1 = the previous step's
 * RHS/N, slot 2 = the one before), 0 for the RK4/ETDRK4 steppers (no memory).
 * Layout as the state.  sw_reset_history: the next three steps start the AB3
 * steppers with forward Euler, as at clock.step < 3 (a restart from a state
 * without saved history, which is what the reference's
 * load_from_snapshot! restart amounts to, rsw/RSWDriver.jl:10-36); it
 * counts steps, not the clock (sw_set_clock does not move it).
 * sw_set_history makes the history valid again and cancels a pending reset. */
int sw_history_slots(const sw_ctx* ctx, int32_t* nslots);
int sw_get_history(const sw_ctx* ctx, int32_t slot, void* buf, size_t bytes);
int sw_set_history(sw_ctx* ctx, int32_t slot, const void* buf, size_t bytes);
int sw_reset_history(sw_ctx* ctx);

/* Restart blob (ABI 7): the stepper's whole memory in fp64 whatever
 * sw_config.precision says — libsw keeps state and history in fp64, so a
 * ComplexF32 copy through sw_get_state / sw_get_history would round them and
 * the continuation would not be bitwise.  Layout: a 64-byte header (magic
 * "SWCKPT01", ABI, model, stepper, nx, ny, nf, history slots, pending Euler
 * start-up steps, t, step), then the state and each history slot as Julia
 * (nkr, nl, nf) ComplexF64 arrays.  sw_set_checkpoint restores state,
 * history, clock and start-up count of the same problem (SW_E_INVALID
 * otherwise); the next sw_step continues bit for bit.  One slab per process:
 * every rank calls both (collective). */
int sw_checkpoint_bytes(const sw_ctx* ctx, size_t* bytes);
int sw_get_checkpoint(const sw_ctx* ctx, void* buf, size_t bytes);
int sw_set_checkpoint(sw_ctx* ctx, const void* buf, size_t bytes);

int sw_set_clock(sw_ctx* ctx, double t, int64_t step);
int sw_get_clock(const sw_ctx* ctx, double* t, int64_t* step);

/* stepforward!(prob, nsteps): nsteps × stepforward!(sol, clock, ts, …). */
int sw_step(sw_ctx* ctx, int64_t nsteps);

/* equation.calcN!(N, sol, …) on a caller state (no stepping, clock untouched):
 * N = calcN(dealias(sol)), column-major (nkr,nl,nf) complex128; aliased modes 0. */
int sw_calcN(sw_ctx* ctx, const void* sol, void* N, size_t bytes);

/* updatevars! equivalent: one physical field of the current state. */
int sw_get_physical(sw_ctx* ctx, int32_t field_id, void* out, size_t bytes);

/* Scalar diagnostics of the current state (SW_DIAG_*). */
int sw_diag(sw_ctx* ctx, int32_t diag_id, double* out);

/* FF Diagnostic(kinetic_energy, prob; freq) + Diagnostic(potential_energy, …)
 * recorded on the device while stepping (rsw/RSWDriver.jl:193-196,
 * swqg/TwoLayerDriver.jl:86-89, FF increment! after each step): after every
 * step with clock.step % freq == 0, libsw reduces the energies of the state
 * the reference's functions read at that point — RSW: vars.uh/vh/ηh, i.e. the
 * (dealiased) input of the step's last calcN (rsw/RotatingShallowWater.jl
 * :147-149, 323-333); 2LQG: prob.sol after the step (swqg/TwoLayerQG.jl
 * :230-252) — with no host synchronisation.  freq = 0 disables; at most
 * `capacity` records are kept (later ones are dropped).  Resets the records. */
typedef struct sw_energy_record {
  int64_t step;            /* clock.step after the step                     */
  double  t;               /* clock.t after the step                        */
  double  ke;              /* RSW: kinetic energy; QG2: KE of layer 1;
                              TY: baroclinic kinetic (|u_c|² + |v_c|²)      */
  double  ke2;             /* QG2: KE of layer 2 (0 for RSW); TY: barotropic */
  double  pe;              /* potential energy (TY: baroclinic |p_c|²)       */
  double  wg[4];           /* TY: wave KE, wave PE, geostrophic KE,
                              geostrophic PE (SW_DIAG_WAVE_KE..GEO_PE); else 0 */
} sw_energy_record;
int sw_set_energy_diagnostics(sw_ctx* ctx, int64_t freq, int64_t capacity);
/* Copies up to max_records records (oldest first); *n_records = the count.
 * One slab per process: every rank must call it (it gathers the slabs). */
int sw_get_energy_diagnostics(sw_ctx* ctx, sw_energy_record* out, int64_t max_records,
                              int64_t* n_records);

/* ABI 9.  stepforward!(prob, nsteps) (nsteps >= 1) whose last step also
 * yields, in *rec, the energies FF's Diagnostic functions read right after
 * it (kinetic_energy(prob), potential_energy(prob) …: the record semantics
 * above, independent of sw_set_energy_diagnostics).  For a caller that defers
 * FF's per-step stepforward!(sol, clock, ts, …) calls (utils/IFMAB3.jl:157)
 * and runs them when FF's increment! (after every step of FF's
 * stepforward!(prob, diags, n)) asks for an energy: integration/julia/SWLib.jl.
 * SW_E_NAN as sw_step (rec is filled first).  One slab per process: every
 * rank calls it (collective). */
int sw_step_record(sw_ctx* ctx, int64_t nsteps, sw_energy_record* rec);

/* ABI 9.  The slab exchange of a decomposed problem explained (DESIGN.md §6;
 * the reference has no multi-GPU path: north-star scope): nsteps steps of the
 * production schedule (the state advances), each timed with events on the
 * compute stream.  One slab per process: every rank calls it (collective). */
#define SW_XPORT_NONE  0   /* one slab                                            */
#define SW_XPORT_RCCL  1   /* one slab per process, RCCL grouped send/recv         */
#define SW_XPORT_HOST  2   /* one slab per process, the caller's exchange hook     */
#define SW_XPORT_LOCAL 3   /* every slab in this process (device copies)           */
typedef struct sw_comm_stats {
  int32_t nranks;          /* P, slabs of the decomposition                        */
  int32_t transport;       /* SW_XPORT_*                                           */
  int32_t rccl_ranks;      /* ncclCommCount of libsw's communicator (0: no RCCL)   */
  int32_t pipelined;       /* 1: transposes on the side stream per field group
                              (event-ordered); 0: sequential on the compute stream */
  int32_t row_chunks;      /* pipelined: the row pass in this many chunks behind
                              the last inverse group's transposes                  */
  int32_t reserved;
  double  step_us;         /* compute-stream time per step                         */
  double  exposed_us;      /* per step: compute-stream time spent waiting for the
                              transposes (sequential: the transposes themselves)   */
  double  bytes_sent;      /* per step: bytes this slab's transposes send to the
                              other slabs                                          */
} sw_comm_stats;
int sw_comm_profile(sw_ctx* ctx, int64_t nsteps, sw_comm_stats* out);

/* ABI 9, round 6.  The link model a one-slab-per-process context measured at
 * sw_create (collective there): a grouped exchange of m bytes with every peer
 * at two sizes, t(m) = α + m/β (the slowest rank's times, so every rank
 * decides alike), and one peer at a time (a shift: send to rank + d, receive
 * from rank - d) at 4 MiB.  The slab schedule follows from it: the transposes
 * are pipelined on the side stream when this decomposition's per-(peer,
 * field) message is at least n½ = α·β (the size at which a message moves at
 * half the link rate), and the last inverse group goes in row chunks while a
 * chunk's messages stay at least n½ (before round 6: a fixed 1 MiB).
 * SW_LINK_PROBE=0 skips the probe (the 1 MiB rule); SW_OVERLAP and
 * SW_ROW_CHUNKS still force the schedule.  The reference has no multi-GPU
 * path (north-star scope). */
typedef struct sw_link_model {
  int32_t probed;           /* 1: measured (one slab per process, P > 1)           */
  int32_t transport;        /* SW_XPORT_* the probe ran on                         */
  int32_t pipelined;        /* the schedule chosen: 1 pipelined, 0 sequential      */
  int32_t row_chunks;       /* row chunks of the pipelined schedule                */
  double  latency_us;       /* α                                                   */
  double  GBps;             /* β: per peer and direction, every peer at once      */
  double  nhalf_bytes;      /* α·β                                                 */
  double  msg_bytes;        /* this decomposition's per-(peer, field) message      */
  double  peer_GBps[8];     /* peer_GBps[d-1]: one peer at a time, to rank + d, d < P
                               (RCCL only; 0 otherwise and beyond P - 1)           */
} sw_link_model;
int sw_get_link_model(const sw_ctx* ctx, sw_link_model* out);

/* Per-kernel HIP-event timing of `nsteps` steps (the state advances).
 * Fills up to max_stats entries; *n_stats receives the count.  With
 * SW_PROF_COLD=1 in the environment a read of a 512 MiB buffer precedes each
 * timed kernel (L2 and Infinity Cache evicted: inputs from HBM alone). */
int sw_profile_steps(sw_ctx* ctx, int64_t nsteps, sw_kernel_stat* stats,
                     int32_t max_stats, int32_t* n_stats);

/* Algorithmic HBM bytes of one step of the configured path. */
double sw_step_alg_bytes(const sw_ctx* ctx);

/* Multi-GPU: write an RCCL unique id (128 bytes); rank 0 calls it and
 * broadcasts the bytes to every rank before sw_create. */
int sw_comm_unique_id(void* out128);

/* Slab geometry of `slab` for cfg (nx, ny, aliased_fraction, nranks), no GPU
 * needed: out[0..7] = kc (live kr columns), kcl (columns per
 * slab), kr0 (first column of the slab), kcn (live columns held), nyl (rows
 * per slab), y0 (first row), Lr (live l rows), LrP (padded column length). */
int sw_slab_geometry(const sw_config* cfg, int32_t slab, int32_t out[8]);

#ifdef __cplusplus
}
#endif
#endif /* SW_H */
