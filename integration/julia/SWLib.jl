# SWLib.jl — the FourierFlows-side binding of libsw (include/sw.h, ABI 9).
#
# A maintainer's addition to the reference's run directories (INTEGRATION.md
# says how it is installed).  After `SWLib.attach!(Model)` for a model module
# (RotatingShallowWater, TwoLayerQG, ThomasYamada, GeophysicalFlows'
# MultiLayerQG) the reference drivers run unchanged:
#
#   * `Model.Problem(GPU(); kw...)` (rsw/RSWDriver.jl:135,164,
#     swqg/TwoLayerDriver.jl:30,63, thomasyamada/TYdriver.jl:117-129,
#     simulation/TwoLayerSimulation.jl:14,37) builds FourierFlows' host-side
#     objects (grid, vars, params, equation, clock, sol) on CPU() and a libsw
#     context that owns the state on the MI355X.  The CUDA-only construction —
#     TwoDGrid(GPU()) with CUFFT plans, populate_L!'s @cuda Lop_kernel
#     (rsw/RotatingShallowWater.jl:276-289), IFMAB3TimeStepper's @cuda
#     kernel_exp (utils/IFMAB3.jl:44-66) — never runs: under SWLib FourierFlows'
#     GPU() device means "state on the libsw device, every array the driver
#     sees on the host".  `Problem(CPU())` stays the reference's own FFTW path
#     unless LIBSW_CPU=1.
#   * FourierFlows' own `stepforward!(prob, diags, n)` (rsw/RSWDriver.jl:212,
#     swqg/TwoLayerDriver.jl:105, TYdriver.jl:172,217,
#     TwoLayerSimulation.jl:128) runs unchanged: its per-step seam
#     `stepforward!(sol, clock, ts::SWStepper, …)` (the method
#     utils/IFMAB3.jl:157 defines for its own stepper) only counts the step;
#     the counted steps run on the device in one `sw_step` when the host next
#     needs the state — an energy Diagnostic's value at FF's `increment!`
#     (`sw_step_record`), `updatevars!`, `set_solution!`, or the first read
#     of a physical field of `prob.vars` (`SWField`: the drivers' NaN scan
#     right after the block, rsw/RSWDriver.jl:213, swqg/TwoLayerDriver.jl:106,
#     so a blow-up throws on the frame it happened in) — and prob.sol is
#     downloaded only at updatevars!/set_solution!, never per step.
#   * `set_solution!` / `set_q!`, `updatevars!`, `enforce_reality_condition!`
#     and the energy functions the Diagnostics call, of a libsw problem, go
#     through the C ABI; for any other problem the reference's own method runs
#     (`invoke`).  SWLib defines no FourierFlows method whose arguments are
#     all FourierFlows' (or Base's) types: the only FF function it extends is
#     the per-step seam, on `ts::SWStepper`.
#
# FourierFlows / GeophysicalFlows are not vendored in the reference (SURVEY
# §8c); the FF/GF names used here are the ones the reference itself calls.
# Julia is not installed where this file was written, so it is checked by
# text (tests/test_julia_shim.py) and its C call sequence is replayed through
# ctypes (tests/driver_replay.py, tests/test_gpu_driver_replay.py).
module SWLib

using FourierFlows
using FourierFlows: AbstractTimeStepper, AbstractDiagnostic, CPU, GPU, Device
using LinearAlgebra: mul!

const libsw = get(ENV, "LIBSW", joinpath(@__DIR__, "libsw.so"))

# ---------------------------------------------------------------- include/sw.h
const SW_ABI_VERSION = Int32(9)
const SW_MODEL_RSW, SW_MODEL_QG2, SW_MODEL_TY, SW_MODEL_MLQG = Int32(0), Int32(1), Int32(2), Int32(3)
const STEPPERS = Dict("FilteredAB3" => Int32(0), "IFMAB3" => Int32(1), "IFMRK4" => Int32(2),
                      "ETDRK4" => Int32(3), "FilteredRK4" => Int32(4))
const SW_E_NAN = Cint(-5)
const SW_DIAG_KE, SW_DIAG_PE, SW_DIAG_KE2, SW_DIAG_KE1, SW_DIAG_BT = Int32(1), Int32(2), Int32(4), Int32(5), Int32(6)
const SW_DIAG_WAVE_KE = Int32(7)   # .. SW_DIAG_GEO_PE = 10
const SW_PREC_F64, SW_PREC_F32 = Int32(0), Int32(1)
# sw_get_physical ids: RSW u v η ζ; 2LQG/MLQG layer*8 + (u 0, v 1, ζ 3, q 4, ψ 5);
# TY u_c 0, v_c 1, p_c 2, ζ_T 3, q_c 4, ψ_T 5, u_T 8, v_T 9
const PHYS_U, PHYS_V, PHYS_ETA, PHYS_ZETA, PHYS_Q, PHYS_PSI = 0, 1, 2, 3, 4, 5

# struct sw_config, field for field (C layout; mutable so that ccall passes a
# pointer to it and sw_config_default can fill it)
Base.@kwdef mutable struct SWConfig
    abi_version::Int32 = SW_ABI_VERSION; model::Int32 = 0; stepper::Int32 = 0
    nx::Int32 = 128; ny::Int32 = 128
    Lx::Float64 = 2π; Ly::Float64 = 2π; aliased_fraction::Float64 = 1/3; dt::Float64 = 5e-2
    f::Float64 = 1.0; Cg::Float64 = 1.0; nu::Float64 = 1e-16; nnu::Int32 = 4
    U::Float64 = 0.5; mu::Float64 = 1e-2; F::Float64 = 90.0
    use_filter::Int32 = 0; filter_order::Int32 = 4
    filter_innerK::Float64 = 0.65; filter_outerK::Float64 = 1.0; filter_tol::Float64 = 1e-15
    device::Int32 = 0; check_nan::Int32 = 1; nop_calcN::Int32 = 0; unfused::Int32 = 0
    nranks::Int32 = 1; rank::Int32 = 0; local_slabs::Int32 = 1
    comm_unique_id::Ptr{Cvoid} = C_NULL
    exchange::Ptr{Cvoid} = C_NULL; exchange_user::Ptr{Cvoid} = C_NULL
    Ro::Float64 = 0.2                                   # ThomasYamada
    f0::Float64 = 1.0; beta::Float64 = 0.0              # MultiLayerQG (2 layers)
    H::NTuple{2,Float64} = (0.5, 0.5); b::NTuple{2,Float64} = (1.0, 0.0)
    Ulayer::NTuple{2,Float64} = (0.0, 0.0)
    precision::Int32 = SW_PREC_F64                      # the reference's T
    aliased_state::Int32 = 0                            # 1: full-array prob.sol (include/sw.h)
end

# struct sw_energy_record
struct SWEnergyRecord
    step::Int64; t::Float64; ke::Float64; ke2::Float64; pe::Float64; wg::NTuple{4,Float64}
end

# ------------------------------------------------ physical fields of prob.vars
# The reference's calcN! writes vars' physical fields at every step
# (rsw/RotatingShallowWater.jl:147-149: u, v, η of the calcN input), and the
# drivers scan one of them for NaN right after stepforward!(prob, diags, n)
# (rsw/RSWDriver.jl:213 vars.η, swqg/TwoLayerDriver.jl:106 vars.q).  Here the
# steps of that block may still be counted only (the per-step seam below).
# So the physical fields of a libsw problem's vars are SWFields: host Arrays
# whose first read runs the counted steps (flush!: one sw_step, no state
# download) and, after SW_E_NAN, holds NaN (blowup!) — the driver's scan then
# throws on the frame where the state went non-finite, and no NaN snapshot
# is written.  Between updatevars! calls they hold the last updatevars!'s
# fields (the reference's: the last calcN input), which no driver reads.
mutable struct Owner
    prob::Any          # the Problem these fields belong to (set once it is built)
end

struct SWField{T,N} <: AbstractArray{T,N}
    data::Array{T,N}
    owner::Owner
end

# run the problem's counted steps, if any, before the field is read
function settle!(a::SWField)
    prob = a.owner.prob
    prob === nothing || prob.timestepper.pending == 0 || flush!(prob)
    return a
end
Base.parent(a::SWField) = a.data
Base.size(a::SWField) = size(a.data)
Base.IndexStyle(::Type{<:SWField}) = IndexLinear()
Base.@propagate_inbounds Base.getindex(a::SWField, i::Int) = (settle!(a); a.data[i])
Base.@propagate_inbounds Base.setindex!(a::SWField, x, i::Int) = (a.data[i] = x; a)
Base.similar(a::SWField, ::Type{S}, dims::Dims) where {S} = similar(a.data, S, dims)
Base.fill!(a::SWField, x) = (fill!(a.data, x); a)
# isnan.(vars.η), abs.(vars.u), @views … read the settled host array
Base.Broadcast.broadcastable(a::SWField) = parent(settle!(a))
# deepcopy(vars.u) before FFTW's mul! (rsw/RotatingShallowWater.jl:128-130,
# swqg/TwoLayerQG.jl:147-148): a plain Array, which FFTW's plans accept
Base.deepcopy_internal(a::SWField, d::IdDict) = Base.deepcopy_internal(parent(settle!(a)), d)
host(a::SWField) = parent(a)
host(a::Array) = a

# the model's own Vars (rsw/RotatingShallowWater.jl:25-34, swqg/TwoLayerQG.jl:32-43,
# thomasyamada/ThomasYamada.jl:26-43: Vars{Aphys, Atrans}) with every physical
# (real) field an SWField of the same host array
function device_vars(vars, owner::Owner)
    V = typeof(vars).name.wrapper
    wrap(x) = x isa Array && eltype(x) <: Real ? SWField(x, owner) : x
    return V((wrap(getfield(vars, k)) for k in fieldnames(typeof(vars)))...)
end

# FourierFlows.Problem with the vars' owner set
function owned_problem(owner::Owner, sol, clock, equation, grid, vars, params, ts)
    prob = FourierFlows.Problem(sol, clock, equation, grid, vars, params, ts)
    owner.prob = prob
    return prob
end

# ------------------------------------------------------------- the time stepper
# The TimeStepper a libsw problem holds.  FourierFlows types Problem's
# timestepper field as AbstractTimeStepper{A}, A the type of prob.sol
# (utils/IFMAB3.jl:13 subtypes it the same way).
mutable struct SWStepper{A<:AbstractArray, Tf} <: AbstractTimeStepper{A}
    ctx::Ptr{Cvoid}
    filter::Tf             # FF makefilter(equation; kw...) or ones: drivers read it
                           # (simulation/TwoLayerSimulation.jl:44)
    model::Int32
    pending::Int           # steps FF's loop has taken that the device has not run yet
    synced::Bool           # prob.sol (host) holds the device state
    rec::SWEnergyRecord    # energies after the last device step (or of the set state)
    rec_step::Int          # clock.step of `rec` (-1: none)
    blewup::Bool           # the last device step returned SW_E_NAN
    uid::Vector{UInt8}     # keeps the RCCL unique id alive with the context
end

is_sw(prob) = prob.timestepper isa SWStepper

lasterror(ctx) = unsafe_string(ccall((:sw_last_error, libsw), Cstring, (Ptr{Cvoid},), ctx))
check(ctx::Ptr{Cvoid}, rc, what) = rc == 0 || error("libsw ", what, ": ", lasterror(ctx), " (code ", rc, ")")
check(ts::SWStepper, rc, what) = check(ts.ctx, rc, what)

# one slab per process (DESIGN.md §6): the launcher (e.g. under MPI.jl) sets
# this before building the problem; rank 0's sw_comm_unique_id bytes are
# broadcast to every rank
const DECOMPOSITION = Ref{Any}(nothing)   # (nranks, rank, uid::Vector{UInt8}, device)
function set_decomposition!(nranks, rank, uid::Vector{UInt8}; device=rank)
    DECOMPOSITION[] = (Int32(nranks), Int32(rank), uid, Int32(device))
end
function comm_unique_id()
    buf = zeros(UInt8, 128)
    rc = ccall((:sw_comm_unique_id, libsw), Cint, (Ptr{UInt8},), buf)
    rc == 0 || error("sw_comm_unique_id failed (code $rc)")
    return buf
end

function config(model, stepper::AbstractString; nx, ny, Lx, Ly, aliased_fraction, dt, T)
    haskey(STEPPERS, stepper) || error("libsw: stepper \"$stepper\" is not built (",
                                       join(keys(STEPPERS), ", "), ")")
    T in (Float32, Float64) || error("libsw: T must be Float32 or Float64, got $T")
    cfg = SWConfig()
    ccall((:sw_config_default, libsw), Cvoid, (Ref{SWConfig},), cfg)
    cfg.model, cfg.stepper = model, STEPPERS[stepper]
    cfg.nx, cfg.ny, cfg.Lx, cfg.Ly = nx, ny, Lx, Ly
    # dt as the Problem holds it (Clock{T}; utils/IFMAB3.jl:69 rounds it to T)
    cfg.aliased_fraction, cfg.dt = aliased_fraction, T(dt)
    cfg.precision = T == Float32 ? SW_PREC_F32 : SW_PREC_F64
    cfg.device = parse(Int32, get(ENV, "LIBSW_DEVICE", "0"))
    # LIBSW_ALIASED_STATE=1: RotatingShallowWater's / TwoLayerQG's / ThomasYamada's /
    # MultiLayerQG's prob.sol, calcN! and energies on the full array, the modes
    # dealias! removes included (include/sw.h)
    model in (SW_MODEL_RSW, SW_MODEL_QG2, SW_MODEL_TY, SW_MODEL_MLQG) &&
        (cfg.aliased_state = get(ENV, "LIBSW_ALIASED_STATE", "0") == "1" ? 1 : 0)
    return cfg
end

# FF makefilter kwargs (utils/IFMAB3.jl:80-84; FilteredAB3 / FilteredRK4)
function set_filter!(cfg, use_filter; order=4, innerK=0.65, outerK=1.0, tol=1e-15, diagonal=false)
    cfg.use_filter = use_filter ? 1 : 0
    cfg.filter_order, cfg.filter_innerK, cfg.filter_outerK, cfg.filter_tol = order, innerK, outerK, tol
    return (; order, innerK, outerK, tol)
end

function SWStepper(cfg::SWConfig, equation, filter)
    uid = UInt8[]
    if DECOMPOSITION[] !== nothing
        cfg.nranks, cfg.rank, uid, cfg.device = DECOMPOSITION[]
        cfg.local_slabs = 1
        cfg.comm_unique_id = pointer(uid)
    end
    h = Ref{Ptr{Cvoid}}(C_NULL)
    rc = GC.@preserve uid ccall((:sw_create, libsw), Cint, (Ref{Ptr{Cvoid}}, Ref{SWConfig}), h, cfg)
    if rc != 0
        msg = h[] == C_NULL ? "sw_create failed" : lasterror(h[])
        ccall((:sw_destroy, libsw), Cvoid, (Ptr{Cvoid},), h[])
        error("libsw sw_create: ", msg, " (code ", rc, ")")
    end
    A = Array{equation.T, length(equation.dims)}
    rec0 = SWEnergyRecord(0, 0.0, 0.0, 0.0, 0.0, (0.0, 0.0, 0.0, 0.0))
    ts = SWStepper{A, typeof(filter)}(h[], filter, cfg.model, 0, true, rec0, -1, false, uid)
    finalizer(t -> ccall((:sw_destroy, libsw), Cvoid, (Ptr{Cvoid},), t.ctx), ts)
    return ts
end

# the filter array the reference's stepper would hold
stepper_filter(equation, filters::Bool, fkw) =
    filters ? FourierFlows.makefilter(equation; fkw...) : ones(real(equation.T), equation.dims)

# --------------------------------------------------------------- state traffic
# prob.sol (Julia (nkr, nl, nf) Complex{T}) <-> the device state; T = Float32
# (rsw/RSWDriver.jl:164, swqg/TwoLayerDriver.jl:63) crosses as it is
# (cfg.precision), libsw computes in Float64 either way
upload!(ts::SWStepper, sol::Array) =
    check(ts, ccall((:sw_set_state, libsw), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t), ts.ctx, sol, sizeof(sol)),
          "sw_set_state")
download!(sol::Array, ts::SWStepper) =
    check(ts, ccall((:sw_get_state, libsw), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Csize_t), ts.ctx, sol, sizeof(sol)),
          "sw_get_state")
push_clock!(ts::SWStepper, clock) =
    check(ts, ccall((:sw_set_clock, libsw), Cint, (Ptr{Cvoid}, Float64, Int64), ts.ctx, clock.t, clock.step),
          "sw_set_clock")

# set_solution! of a libsw problem: the host copy is uploaded (libsw
# dealiases, as the next calcN! would), prob.sol refreshed from the device,
# the clock pushed (TYdriver.jl:190 sets prob.clock.t before set_solution!)
function load_solution!(prob)
    ts = prob.timestepper
    ts.pending = 0                 # steps counted before a new state are void
    upload!(ts, prob.sol)
    download!(prob.sol, ts)
    push_clock!(ts, prob.clock)
    ts.synced, ts.rec_step, ts.blewup = true, -1, false
    return nothing
end

# one physical field (updatevars!) into a host array (or SWField) or a layer of one
function physical!(dst::AbstractArray, ts::SWStepper, id::Integer)
    a = host(dst)
    check(ts, ccall((:sw_get_physical, libsw), Cint, (Ptr{Cvoid}, Int32, Ptr{Cvoid}, Csize_t),
                    ts.ctx, id, a, sizeof(a)), "sw_get_physical")
    return dst
end
function physical!(dst::AbstractArray{T,3}, ts::SWStepper, id::Integer, layer::Integer) where {T}
    a = host(dst)
    GC.@preserve a begin
        n = size(a, 1) * size(a, 2)
        p = pointer(a, (layer - 1) * n + 1)
        check(ts, ccall((:sw_get_physical, libsw), Cint, (Ptr{Cvoid}, Int32, Ptr{Cvoid}, Csize_t),
                        ts.ctx, id, p, n * sizeof(T)), "sw_get_physical")
    end
    return dst
end

# ------------------------------------------------------- stepping and records
# FF's per-step seam (the method utils/IFMAB3.jl:157 defines for its own
# stepper; FF's stepforward!(prob) and stepforward!(prob, diags, n) loops call
# it once per step).  Here it only counts the step and advances the clock in
# the Problem's own arithmetic (clock.t += clock.dt, utils/IFMAB3.jl:162-163):
# no C call, no host copy.  The counted steps run when the host next needs
# the device state (sync!, device_energy).
function FourierFlows.stepforward!(sol, clock, ts::SWStepper, equation, vars, params, grid)
    ts.pending += 1
    ts.synced = false
    clock.t += clock.dt
    clock.step += 1
    return nothing
end

# run the counted steps on the device (one sw_step)
function flush!(prob)
    ts = prob.timestepper
    ts.pending > 0 || return nothing
    n, ts.pending = ts.pending, 0
    rc = ccall((:sw_step, libsw), Cint, (Ptr{Cvoid}, Int64), ts.ctx, n)
    ts.blewup = rc == SW_E_NAN
    ts.blewup || check(ts, rc, "sw_step")
    ts.blewup && blowup!(prob)
    return nothing
end

# prob.sol current on the host (device -> host, dealiased; NaN after a blow-up)
function sync!(prob)
    ts = prob.timestepper
    flush!(prob)
    ts.synced || download!(prob.sol, ts)
    ts.synced = true
    return nothing
end

# The value FF's increment! stores for an energy Diagnostic (after every step
# of stepforward!(prob, diags, n), at clock.step % freq == 0): the counted
# steps run with the energies of the last one recorded on the device
# (sw_step_record: RSW's vars.uh/vh/ηh = the last calcN's input, 2LQG's
# prob.sol, …); several Diagnostics at one step share that record.  With no
# step since the state was set (Diagnostic's own first call), sw_diag of the
# state itself.
function device_energy(prob, pick)
    ts = prob.timestepper
    if ts.pending > 0
        n, ts.pending = ts.pending, 0
        r = Ref{SWEnergyRecord}()
        rc = ccall((:sw_step_record, libsw), Cint, (Ptr{Cvoid}, Int64, Ref{SWEnergyRecord}), ts.ctx, n, r)
        ts.blewup = rc == SW_E_NAN
        ts.blewup || check(ts, rc, "sw_step_record")
        ts.rec, ts.rec_step = r[], prob.clock.step
        ts.blewup && blowup!(prob)
    elseif ts.rec_step != prob.clock.step
        ts.rec, ts.rec_step = diag_record(ts, prob.clock), prob.clock.step
    end
    return as_T(real(eltype(prob.sol)), pick(ts.rec))
end
as_T(T, x::Real) = T(x)
as_T(T, x::Tuple) = map(y -> as_T(T, y), x)
as_T(T, x::AbstractVector) = T.(x)

function diag_record(ts, clock)
    d(id) = (x = Ref{Float64}(0.0);
             check(ts, ccall((:sw_diag, libsw), Cint, (Ptr{Cvoid}, Int32, Ref{Float64}), ts.ctx, id, x), "sw_diag");
             x[])
    ts.model == SW_MODEL_TY &&
        return SWEnergyRecord(clock.step, clock.t, d(SW_DIAG_KE), d(SW_DIAG_BT), d(SW_DIAG_PE),
                              ntuple(i -> d(SW_DIAG_WAVE_KE + Int32(i - 1)), 4))
    return SWEnergyRecord(clock.step, clock.t, d(SW_DIAG_KE1), d(SW_DIAG_KE2), d(SW_DIAG_PE), (0.0, 0.0, 0.0, 0.0))
end

# FF Diagnostic calc -> the record entry it returns (rsw/RSWDriver.jl:193-196,
# swqg/TwoLayerDriver.jl:86-89, TYdriver.jl:152-153,194-195,
# TwoLayerSimulation.jl:52)
const RECORD = IdDict{Any,Function}()

# After SW_E_NAN the drivers' own test finds the NaN and throws "Solution is
# NaN" (rsw/RSWDriver.jl:213-218 tests vars.η, swqg/TwoLayerDriver.jl:106-111
# vars.q: in the reference calcN! leaves them NaN); prob.sol holds the
# non-finite state.  The test's read of vars.η / vars.q itself runs the
# block's counted steps (SWField), so it sees the blow-up of that block.
function blowup!(prob)
    for name in (:η, :q, :u, :v)
        hasproperty(prob.vars, name) && fill!(getproperty(prob.vars, name), NaN)
    end
end

# ------------------------------------------------------------------- models
# Each builder takes the reference Problem's keywords with its defaults
# (cited), builds the host objects the reference builds on CPU(), and returns
# FourierFlows.Problem(sol, clock, equation, grid, vars, params, ts) as the
# reference's IFMAB3 branch does (rsw/RotatingShallowWater.jl:95).

# rsw/RotatingShallowWater.jl:70-99
function rsw_problem(M::Module; nx=128, ny=nx, Lx=2π, Ly=Lx, ν=1.0e-16, nν=4, f=1.0, Cg=1.0,
                     stepper="IFMAB3", dt=5e-2, calcF! = nothing, aliased_fraction=1/3, T=Float64,
                     use_filter=false, stepper_kwargs...)
    (calcF! === nothing || calcF! === M.nothingfunction) ||
        error("libsw: the stochastic forcing calcF! is not on the libsw path")
    grid = TwoDGrid(CPU(); nx, Lx, ny, Ly, aliased_fraction, T)
    params = M.Params{T}(ν, nν, f, Cg^2)
    owner = Owner(nothing)
    vars = device_vars(M.Vars(grid), owner)
    equation = M.Equation(params, grid)         # host L (populate_L!, CPU method :262-274)
    cfg = config(SW_MODEL_RSW, stepper; nx, ny, Lx, Ly, aliased_fraction, dt, T)
    cfg.f, cfg.Cg, cfg.nu, cfg.nnu = params.f, Cg, params.ν, nν   # libsw squares Cg as :88 does
    # FF FilteredAB3 filters always; IFMAB3 / IFMRK4 when use_filter (utils/IFMAB3.jl:80-85)
    filters = stepper in ("FilteredAB3", "FilteredRK4") || use_filter
    fkw = set_filter!(cfg, use_filter; stepper_kwargs...)
    ts = SWStepper(cfg, equation, stepper_filter(equation, filters, fkw))
    clock = FourierFlows.Clock{T}(dt, 0, 0)
    sol = zeros(CPU(), equation.T, equation.dims)
    return owned_problem(owner, sol, clock, equation, grid, vars, params, ts)
end

# swqg/TwoLayerQG.jl:55-90
function qg2_problem(M::Module; nx=128, ny=nx, Lx=2π, Ly=Lx, U=0.5, μ=1e-2, ν=1e-6, nν=4, f0=3.0, Cg=1.0,
                     δρρ0=0.2, stepper="IFMAB3", dt=5e-2, aliased_fraction=1/3, T=Float32, use_filter=false,
                     stepper_kwargs...)
    grid = TwoDGrid(CPU(); nx, Lx, ny, Ly, aliased_fraction, T)
    plan = FourierFlows.plan_flows_rfft(Array{T,3}(undef, grid.nx, grid.ny, 2), [1, 2])
    params = M.Params(T(U), T(μ), T(ν), nν, T(2 * f0^2 / Cg^2 / δρρ0), plan)
    owner = Owner(nothing)
    vars = device_vars(M.Vars(grid), owner)
    equation = M.Equation(params, grid)         # host L (KernelAbstractions CPU backend)
    cfg = config(SW_MODEL_QG2, stepper; nx, ny, Lx, Ly, aliased_fraction, dt, T)
    # libsw rounds F, U, μ exactly as params holds them (T), and reproduces the
    # Complex{Float32} literals of L_kernel! (swqg/TwoLayerQG.jl:189-193)
    cfg.U, cfg.mu, cfg.nu, cfg.nnu, cfg.F = params.U, params.μ, params.ν, nν, params.F
    filters = stepper in ("FilteredAB3", "FilteredRK4") || use_filter
    fkw = set_filter!(cfg, use_filter; stepper_kwargs...)
    ts = SWStepper(cfg, equation, stepper_filter(equation, filters, fkw))
    clock = FourierFlows.Clock{T}(dt, 0, 0)
    sol = zeros(CPU(), equation.T, equation.dims)
    return owned_problem(owner, sol, clock, equation, grid, vars, params, ts)
end

# thomasyamada/ThomasYamada.jl:55-74 (FF's ETDRK4 by default, :63)
function ty_problem(M::Module; nx=128, ny=nx, Lx=2π, Ly=Lx, ν=3.5e-25, nν=8, Ro=0.2, stepper="ETDRK4",
                    dt=5e-2, aliased_fraction=1/3, T=Float64)
    stepper == "ETDRK4" || error("libsw: ThomasYamada steps with ETDRK4 (its diagonal L)")
    grid = TwoDGrid(CPU(); nx, Lx, ny, Ly, aliased_fraction, T)
    params = M.Params{T}(ν, nν, Ro)
    owner = Owner(nothing)
    vars = device_vars(M.Vars(grid), owner)
    equation = M.Equation(params, grid)
    cfg = config(SW_MODEL_TY, stepper; nx, ny, Lx, Ly, aliased_fraction, dt, T)
    cfg.nu, cfg.nnu, cfg.Ro = params.ν, nν, params.Ro
    ts = SWStepper(cfg, equation, stepper_filter(equation, false, (;)))
    clock = FourierFlows.Clock{T}(dt, 0, 0)
    sol = zeros(CPU(), equation.T, equation.dims)
    return owned_problem(owner, sol, clock, equation, grid, vars, params, ts)
end

# GeophysicalFlows MultiLayerQG.Problem(nlayers, dev; nx, Lx, f₀, H, b, U, μ, β,
# dt, stepper, aliased_fraction) as simulation/TwoLayerSimulation.jl:37-38
# builds it: GF's own CPU problem supplies grid, params, vars, equation and
# FilteredRK4's filter; libsw takes over the state and the stepping
function mlqg_problem(M::Module, nlayers::Int; stepper="FilteredRK4", T=Float64, kw...)
    nlayers == 2 || error("libsw: MultiLayerQG with 2 layers")
    # GF's own method (not the CPU() method attach! adds)
    host = invoke(M.Problem, Tuple{Int,FourierFlows.Device}, nlayers, CPU(); stepper, T, kw...)
    g, p = host.grid, host.params
    cfg = config(SW_MODEL_MLQG, stepper; nx=g.nx, ny=g.ny, Lx=g.Lx, Ly=g.Ly,
                 aliased_fraction=get(kw, :aliased_fraction, 1/3), dt=host.clock.dt, T)
    cfg.f0, cfg.beta = get(kw, :f₀, 1.0), get(kw, :β, 0.0)
    cfg.H, cfg.b, cfg.Ulayer = Tuple(Float64.(get(kw, :H, (0.5, 0.5)))), Tuple(Float64.(get(kw, :b, (1.0, 0.0)))),
                               Tuple(Float64.(vec(get(kw, :U, (0.0, 0.0)))))
    cfg.mu, cfg.nu, cfg.nnu = get(kw, :μ, 0.0), get(kw, :ν, 0.0), get(kw, :nν, 1)
    filters = stepper in ("FilteredAB3", "FilteredRK4")
    set_filter!(cfg, filters)
    filt = hasproperty(host.timestepper, :filter) ? host.timestepper.filter :
           stepper_filter(host.eqn, filters, (;))
    ts = SWStepper(cfg, host.eqn, filt)
    return FourierFlows.Problem(host.sol, host.clock, host.eqn, host.grid, host.vars, host.params, ts)
end

# --------------------------------------------------- updatevars! on the device
# rsw/RotatingShallowWater.jl:101-116: spectral vars from the (dealiased,
# current) host sol, the four physical fields by libsw's c2r
function rsw_updatevars!(prob)
    vars, grid, sol, ts = prob.vars, prob.grid, prob.sol, prob.timestepper
    sync!(prob)
    FourierFlows.dealias!(sol, grid)   # :104 (the device's copy is dealiased by sw_get_physical)
    ts.rec_step = -1                   # energies read the updated vars.uh … from here (sw_diag)
    @. vars.uh = @view sol[:, :, 1]
    @. vars.vh = @view sol[:, :, 2]
    @. vars.ηh = @view sol[:, :, 3]
    @. vars.ζh = 1im * grid.kr * vars.vh - 1im * grid.l * vars.uh - prob.params.f * vars.ηh
    physical!(vars.u, ts, PHYS_U); physical!(vars.v, ts, PHYS_V)
    physical!(vars.η, ts, PHYS_ETA); physical!(vars.ζ, ts, PHYS_ZETA)
    return nothing
end

# swqg/TwoLayerQG.jl:113-129
function qg2_updatevars!(M, prob)
    vars, grid, sol, params, ts = prob.vars, prob.grid, prob.sol, prob.params, prob.timestepper
    sync!(prob)
    FourierFlows.dealias!(sol, grid)   # :115 (the device's copy is dealiased by sw_get_physical)
    ts.rec_step = -1
    @. vars.qh = sol
    M.streamfunctionfrompv!(vars.ψh, vars.qh, grid, params)
    @. vars.ζh = -grid.Krsq * vars.ψh
    @. vars.uh = -1im * grid.l * vars.ψh
    @. vars.vh = 1im * grid.kr * vars.ψh
    for layer in 1:2, (field, id) in ((vars.q, PHYS_Q), (vars.ψ, PHYS_PSI), (vars.ζ, PHYS_ZETA),
                                      (vars.u, PHYS_U), (vars.v, PHYS_V))
        physical!(field, ts, 8 * (layer - 1) + id, layer)
    end
    return nothing
end

# thomasyamada/ThomasYamada.jl:76-101 (all = true) and enforce_reality_condition!
# :103-123 (all = false: its mul! into the copies sol[:,:,k] leave sol as it is);
# both dealias sol in place first (:79, :106)
function ty_updatevars!(prob; all=true)
    vars, grid, sol, ts = prob.vars, prob.grid, prob.sol, prob.timestepper
    sync!(prob)
    FourierFlows.dealias!(sol, grid)   # :79 / :106 (the device's copy is dealiased by sw_get_physical)
    ts.rec_step = -1
    @. vars.ζth = sol[:, :, 1]; @. vars.uch = sol[:, :, 2]
    @. vars.vch = sol[:, :, 3]; @. vars.pch = sol[:, :, 4]
    physical!(vars.ζt, ts, 3); physical!(vars.uc, ts, 0); physical!(vars.vc, ts, 1); physical!(vars.pc, ts, 2)
    all || return nothing
    @. vars.ψth = -vars.ζth * grid.invKrsq
    @. vars.uth = -im * grid.l * vars.ψth
    @. vars.vth = im * grid.kr * vars.ψth
    @. vars.qch = im * grid.kr * vars.vch - im * grid.l * vars.uch - vars.pch
    physical!(vars.ut, ts, 8); physical!(vars.vt, ts, 9); physical!(vars.qc, ts, 4)
    return nothing
end

# GeophysicalFlows MultiLayerQG.updatevars!: dealias!(sol), qh = sol, ψh = S⁻¹ qh,
# uh, vh, then q, ψ, u, v per layer
function mlqg_updatevars!(M, prob)
    vars, grid, sol, params, ts = prob.vars, prob.grid, prob.sol, prob.params, prob.timestepper
    sync!(prob)
    FourierFlows.dealias!(sol, grid)   # (the device's copy is dealiased by sw_get_physical)
    ts.rec_step = -1
    @. vars.qh = sol
    M.streamfunctionfrompv!(vars.ψh, vars.qh, params, grid)
    @. vars.uh = -im * grid.l * vars.ψh
    @. vars.vh = im * grid.kr * vars.ψh
    for layer in 1:2, (field, id) in ((vars.q, PHYS_Q), (vars.ψ, PHYS_PSI), (vars.u, PHYS_U), (vars.v, PHYS_V))
        physical!(field, ts, 8 * (layer - 1) + id, layer)
    end
    return nothing
end

# ------------------------------------------------------------------ attach!
# The model's energy functions FF's Diagnostics call (kinetic_energy(prob) …,
# rsw/RotatingShallowWater.jl:326,332, swqg/TwoLayerQG.jl:242,252,
# thomasyamada/ThomasYamada.jl:340-354, GF MultiLayerQG.energies): for a libsw
# problem the device's value (device_energy), else the reference's (invoke).
function energy_methods!(M::Module, picks::Pair{Symbol,<:Function}...)
    for (name, pick) in picks
        RECORD[getfield(M, name)] = pick
        @eval M $name(prob::FourierFlows.Problem) =
            $is_sw(prob) ? $device_energy(prob, $pick) : invoke($name, Tuple{Any}, prob)
    end
    return nothing
end

use_libsw(::CPU) = get(ENV, "LIBSW_CPU", "0") == "1"

"""
    SWLib.attach!(Model)

Give the reference model module `Model` (RotatingShallowWater, TwoLayerQG,
ThomasYamada, GeophysicalFlows.MultiLayerQG) libsw methods.  Each new
method is more specific than the reference's (a typed first argument) and
falls back to it with `invoke` for problems libsw does not hold.
"""
function attach!(M::Module)
    name = nameof(M)
    if name === :RotatingShallowWater
        @eval M begin
            Problem(dev::FourierFlows.GPU; kw...) = $rsw_problem($M; kw...)
            Problem(dev::FourierFlows.CPU; kw...) =
                $use_libsw(dev) ? $rsw_problem($M; kw...) : invoke(Problem, Tuple{FourierFlows.Device}, dev; kw...)
            function set_solution!(prob::FourierFlows.Problem, u0h, v0h, η0h)
                $is_sw(prob) || return invoke(set_solution!, Tuple{Any,Any,Any,Any}, prob, u0h, v0h, η0h)
                prob.sol[:, :, 1] .= u0h; prob.sol[:, :, 2] .= v0h; prob.sol[:, :, 3] .= η0h
                $load_solution!(prob)
                updatevars!(prob)
            end
            updatevars!(prob::FourierFlows.Problem) =
                $is_sw(prob) ? $rsw_updatevars!(prob) : invoke(updatevars!, Tuple{Any}, prob)
        end
        energy_methods!(M, :kinetic_energy => r -> r.ke, :potential_energy => r -> r.pe)
    elseif name === :TwoLayerQG
        @eval M begin
            Problem(dev::FourierFlows.GPU; kw...) = $qg2_problem($M; kw...)
            Problem(dev::FourierFlows.CPU; kw...) =
                $use_libsw(dev) ? $qg2_problem($M; kw...) : invoke(Problem, Tuple{FourierFlows.Device}, dev; kw...)
            function set_solution!(prob::FourierFlows.Problem, q0h)
                $is_sw(prob) || return invoke(set_solution!, Tuple{Any,Any}, prob, q0h)
                prob.sol .= q0h
                $load_solution!(prob)
                updatevars!(prob)
            end
            updatevars!(prob::FourierFlows.Problem) =
                $is_sw(prob) ? $qg2_updatevars!($M, prob) : invoke(updatevars!, Tuple{Any}, prob)
        end
        energy_methods!(M, :kinetic_energy => r -> (r.ke, r.ke2), :potential_energy => r -> r.pe)
    elseif name === :ThomasYamada
        @eval M begin
            Problem(dev::FourierFlows.GPU; kw...) = $ty_problem($M; kw...)
            Problem(dev::FourierFlows.CPU; kw...) =
                $use_libsw(dev) ? $ty_problem($M; kw...) : invoke(Problem, Tuple{FourierFlows.Device}, dev; kw...)
            function set_solution!(prob::FourierFlows.Problem, ζ0h, u0h, v0h, p0h)
                $is_sw(prob) || return invoke(set_solution!, Tuple{Any,Any,Any,Any,Any}, prob, ζ0h, u0h, v0h, p0h)
                prob.sol[:, :, 1] .= ζ0h; prob.sol[:, :, 2] .= u0h
                prob.sol[:, :, 3] .= v0h; prob.sol[:, :, 4] .= p0h
                $load_solution!(prob)
                updatevars!(prob)
            end
            updatevars!(prob::FourierFlows.Problem) =
                $is_sw(prob) ? $ty_updatevars!(prob) : invoke(updatevars!, Tuple{Any}, prob)
            enforce_reality_condition!(prob::FourierFlows.Problem) =
                $is_sw(prob) ? $ty_updatevars!(prob; all=false) :
                               invoke(enforce_reality_condition!, Tuple{Any}, prob)
        end
        energy_methods!(M, :barotropic_energy => r -> r.ke2, :baroclinic_energy => r -> (r.ke, r.pe),
                        :wave_geostrophic_energy => r -> ((r.wg[1], r.wg[2]), (r.wg[3], r.wg[4])))
    elseif name === :MultiLayerQG
        @eval M begin
            Problem(nlayers::Int, dev::FourierFlows.GPU; kw...) = $mlqg_problem($M, nlayers; kw...)
            Problem(nlayers::Int, dev::FourierFlows.CPU; kw...) =
                $use_libsw(dev) ? $mlqg_problem($M, nlayers; kw...) :
                                  invoke(Problem, Tuple{Int,FourierFlows.Device}, nlayers, dev; kw...)
            function set_q!(prob::FourierFlows.Problem, q)
                $is_sw(prob) || return invoke(set_q!, Tuple{Any,Any}, prob, q)
                mul!(prob.vars.qh, prob.params.rfftplan, q)   # GF set_q!: q̂ = rfft(q) over dims (1, 2)
                prob.sol .= prob.vars.qh
                $load_solution!(prob)
                updatevars!(prob)
            end
            updatevars!(prob::FourierFlows.Problem) =
                $is_sw(prob) ? $mlqg_updatevars!($M, prob) : invoke(updatevars!, Tuple{Any}, prob)
        end
        # GF's energies(prob): per-layer KE vector, PE vector (nlayers - 1)
        energy_methods!(M, :energies => r -> ([r.ke, r.ke2], [r.pe]))
    else
        error("SWLib.attach!: no libsw model for module $name")
    end
    return M
end

# TwoLayerSimulation.jl:43 and TwoLayerDriver.jl:11 draw their initial PV as
# device_array(dev)(randn(...)) with dev = GPU(): under SWLib the driver's
# arrays live on the host.  This is SWLib's own function, not a method of
# FourierFlows.device_array: the run-directory wrappers of those two drivers
# (integration/julia/swqg/TwoLayerQG.jl, simulation/Parameters.jl) bind it as
# Main.device_array before the driver's `using FourierFlows` /
# `using GeophysicalFlows`, so only those run directories see it.
device_array(::GPU) = Array
device_array(dev) = FourierFlows.device_array(dev)

end # module
