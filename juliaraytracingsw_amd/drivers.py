"""Driver-side setup mirroring rsw/RSWDriver.jl, swqg/TwoLayerDriver.jl and
thomasyamada/TYdriver.jl: parameter formulas, synthetic random-phase initial conditions
and the frame loop.  Setup only — the per-step work is libsw's.
"""
from __future__ import annotations

import math
import time

import numpy as np

from . import _lib
from . import multilayer_qg as MLQG
from . import rotating_shallow_water as RSW
from . import thomas_yamada as TY
from . import two_layer_qg as QG2
from .grid import TwoDGrid

# rsw/RSWParameters.jl
RSW_PARAMETERS = dict(L=2 * np.pi, f=3.0, Cg=1.0, nnu=4, nutune=20.0, cfltune=0.01, filter_order=8,
                      aliased_fraction=1 / 3, Kg=(10, 13), ag=0.2, Kw=(0, 5), aw=0.1)
# swqg/TwoLayerParameters.jl
QG2_PARAMETERS = dict(L=2 * np.pi, background_Cg=1.0, f=3.0, deformation_radius=1 / 6,
                      intervortex_radius=1.0, nnu=4, nutune=40.0, cfltune=0.025,
                      aliased_fraction=1 / 3, ug=0.025)


# thomasyamada/cpu-setup/Parameters.jl (the first of the three setups)
TY_PARAMETERS = dict(Lx=6 * np.pi, nx=512, Ro=1.0, nnu=8, startup_dt=3e-2, dt=5e-3, stepper="ETDRK4",
                     k0w_range=(0.0, 5 / 3), k0g_range=(10 / 3, 13 / 3), at=0.0, ag=0.3, aw=0.1)


def ty_parameters(nx=None, **over):
    """thomasyamada/cpu-setup/Parameters.jl: ν = 5e-34 (Lx/2π)^16, nν = 8."""
    P = dict(TY_PARAMETERS, **over)
    if nx is not None:
        P["nx"] = nx
    P.setdefault("nu", 5.0e-34 * (P["Lx"] / (2 * np.pi)) ** 16)
    return P


# simulation/Parameters.jl (TwoLayerSimulation with GeophysicalFlows MultiLayerQG)
MLQG_PARAMETERS = dict(Lx=2 * np.pi, nx=512, f=1.0, deformation_radius=1 / 15, intervortex_radius=1 / 2,
                       avg_U=0.1, H0=1.0, nnu=8, nu=0.0, stepper="FilteredRK4", b2=1.0, beta=0.0)


def mlqg_parameters(nx=None, **over):
    """simulation/Parameters.jl: compute_parameters (μ, b₁, shear), dt = 0.02 dx/avg_U,
    U = [s, -s], b = [b₁, b₂], H = [H0/2, H0/2], q0_amplitude = 1e-2 avg_U."""
    P = dict(MLQG_PARAMETERS, **over)
    if nx is not None:
        P["nx"] = nx
    c1, c2 = 3.2, 0.36
    l_star = P["intervortex_radius"] / P["deformation_radius"]
    kappa_star = c2 / math.log(l_star / c1)
    s = P["avg_U"] / l_star
    mu = 2 * s * kappa_star / P["deformation_radius"]
    b1 = 4 * P["f"] ** 2 * P["deformation_radius"] ** 2 / P["H0"] + P["b2"]
    dx = P["Lx"] / P["nx"]
    return dict(P, mu=mu, U=[s, -s], b=[b1, P["b2"]], H=[P["H0"] / 2, P["H0"] / 2], dt=0.02 * dx / P["avg_U"],
                q0_amplitude=1e-2 * P["avg_U"])


def _ff_filter(grid, order=4, innerK=0.65, outerK=1.0, tol=1e-15):
    """FF makefilter values on the host (set-up only; libsw's stepper evaluates
    the same formula per mode)."""
    K = np.sqrt((grid.kr[None, :] * grid.dx / np.pi) ** 2 + (grid.l[:, None] * grid.dy / np.pi) ** 2)
    decay = -np.log(tol) / (outerK - innerK) ** order
    return np.where(K < innerK, 1.0, np.exp(-decay * (K - innerK) ** order))


def mlqg_problem(nx=512, seed=1234, device=0, decomposition=None, **over):
    """TwoLayerSimulation.start! set-up (simulation/TwoLayerSimulation.jl:13-53):
    MultiLayerQG.Problem(2, dev; nx, Lx, f₀, H, b, U, μ, β, dt, stepper,
    aliased_fraction = 0), q₀ = q0_amplitude·randn (seeded numpy stream),
    q̂₀ = filter·rfft(q₀), set_q!."""
    P = mlqg_parameters(nx, **over)
    prob = MLQG.Problem(2, "gpu", nx=P["nx"], Lx=P["Lx"], f0=P["f"], H=P["H"], b=P["b"], U=P["U"], mu=P["mu"],
                        beta=P["beta"], nu=P["nu"], nnu=P["nnu"], dt=P["dt"], stepper=P["stepper"],
                        aliased_fraction=0, device=device, decomposition=decomposition)
    rng = np.random.default_rng(seed)
    g = prob.grid
    q0 = P["q0_amplitude"] * rng.standard_normal((2, g.ny, g.nx))
    q0h = _ff_filter(g)[None] * np.fft.rfft2(q0, axes=(-2, -1))
    prob.sol = q0h  # set_q!(prob, irfft(q̂₀)) = upload of q̂₀ (dealiased)
    return prob, P


def rsw_parameters(nx, **over):
    """rsw/RSWDriver.jl:134-148: dt = cfltune/umax·dx, ν = νtune·dx/kmax^(2nν)/dt."""
    P = dict(RSW_PARAMETERS, **over)
    Lx = P["L"]
    dx = Lx / nx
    kmax = (nx / 2 - 1) * Lx / (2 * np.pi) * (1 - P["aliased_fraction"])
    umax = P["ag"] + P["aw"]
    dt = P["cfltune"] / umax * dx
    nu = P["nutune"] * dx / (kmax ** (2 * P["nnu"])) / dt
    return dict(P, dt=dt, nu=nu, Lx=Lx)


def qg2_compute_parameters(deformation_radius, intervortex_radius, avg_eddy_velocity, H, f0):
    """swqg/TwoLayerDriver.jl:17-27."""
    c1, c2 = 3.2, 0.36
    l_star = intervortex_radius / deformation_radius
    kappa_star = c2 / math.log(l_star / c1)
    U = avg_eddy_velocity / l_star
    mu = 2 * U * kappa_star / deformation_radius
    db = 4 * f0 ** 2 * deformation_radius ** 2 / H
    return mu, db, U


def qg2_parameters(nx, **over):
    """swqg/TwoLayerDriver.jl:29-63."""
    P = dict(QG2_PARAMETERS, **over)
    Lx = P["L"]
    dx = Lx / nx
    kmax = (nx / 2 - 1) * (1 - P["aliased_fraction"])
    H = 1.0
    mu, db, U = qg2_compute_parameters(P["deformation_radius"], P["intervortex_radius"], P["ug"], H, P["f"])
    drr0 = db / (P["background_Cg"] / H)
    dt = P["cfltune"] / P["ug"] * dx
    nu = P["nutune"] * 2 * np.pi / nx / (kmax ** (2 * P["nnu"])) / dt
    return dict(P, dt=dt, nu=nu, U=U, mu=mu, drhorho0=drr0, Lx=Lx)


def shafer_spectra(grid: TwoDGrid, Kg, Kw, f, Cg2, rng):
    """rsw/RSWDriver.jl:93-106,118-120: geostrophic and wave spectra with random
    phases on the annuli, before normalisation.  Draw order: phase = 2π·U[0,1)
    then sgn = sign(U[0,1) - 0.5), each over (nkr, nl) column-major."""
    K2 = grid.Krsq
    geo = (Kg[0] ** 2 <= K2) & (K2 <= Kg[1] ** 2) & (K2 > 0)
    wav = (Kw[0] ** 2 <= K2) & (K2 <= Kw[1] ** 2) & (K2 > 0)
    phase = 2 * np.pi * rng.random((grid.nkr, grid.nl)).T
    sgn = np.sign(rng.random((grid.nkr, grid.nl)).T - 0.5)
    shift = np.exp(1j * phase)
    om = np.sqrt(f ** 2 + Cg2 * K2)
    gamp = 1 / om
    wamp = np.sqrt(grid.invKrsq) / (2 * om)
    kr = np.broadcast_to(grid.kr[None, :], K2.shape)
    l = np.broadcast_to(grid.l[:, None], K2.shape)
    z = np.zeros(K2.shape, np.complex128)
    ugh, vgh, egh, uwh, vwh, ewh = (z.copy() for _ in range(6))
    egh[geo] += (gamp * f * shift)[geo]
    ugh[geo] += (-gamp * 1j * Cg2 * l * shift)[geo]
    vgh[geo] += (gamp * 1j * Cg2 * kr * shift)[geo]
    ewh[wav] += (wamp * K2 * shift)[wav]
    uwh[wav] += (wamp * (sgn * kr * om * shift + 1j * f * l * shift))[wav]
    vwh[wav] += (wamp * (sgn * l * om * shift - 1j * f * kr * shift))[wav]
    return (ugh, vgh, egh), (uwh, vwh, ewh)


def _umax(prob, uh, vh):
    """max sqrt(u² + v²) of the c2r of (uh, vh), computed by libsw's own FFTs."""
    z = np.zeros_like(uh)
    RSW.set_solution(prob, uh, vh, z)
    g = prob.grid
    u = prob.ctx.physical(_lib.SW_PHYS_U, g.ny, g.nx)
    v = prob.ctx.physical(_lib.SW_PHYS_V, g.ny, g.nx)
    return float(np.max(np.sqrt(u ** 2 + v ** 2)))


def set_shafer_initial_condition(prob, Kg, Kw, ag, aw, f, Cg2, rng):
    """rsw/RSWDriver.jl:88-132.  The Umax normalisations use libsw's c2r.

    Note: the dealiasing of set_solution! happens before the c2r here, while
    the reference c2r's the raw spectra; the annuli (K <= 13) are far inside the
    live band, so the two agree."""
    (ugh, vgh, egh), (uwh, vwh, ewh) = shafer_spectra(prob.grid, Kg, Kw, f, Cg2, rng)
    s = ag / _umax(prob, ugh, vgh)
    ugh, vgh, egh = ugh * s, vgh * s, egh * s
    s = aw / _umax(prob, uwh, vwh)
    uwh, vwh, ewh = uwh * s, vwh * s, ewh * s
    RSW.set_solution(prob, ugh + uwh, vgh + vwh, egh + ewh)


def set_seed_initial_condition(prob, rng):
    """swqg/TwoLayerDriver.jl:10-15: q0 = 1e-2·randn(nx, ny, 2), rfft over (1,2).
    The forward transform here is numpy's host FFT on the one-off IC (setup)."""
    g = prob.grid
    q0 = 1e-2 * rng.standard_normal((2, g.ny, g.nx))
    QG2.set_solution(prob, np.fft.rfft2(q0, axes=(-2, -1)))


def set_ty_initial_condition(prob, rng, k0w_range=(0, 1), k0g_range=(0, 1), at=0.0, ag=0.0, aw=0.0):
    """thomasyamada/TYdriver.jl:36-87 (set_initial_condition): phases
    θ, θ₀, θ₊, θ₋ = U[0,1) over (nkr, nl) column-major from the seeded ``rng``
    (Julia's stream is not reproducible), projected on the TYUtils bases
    inside the annuli, each part scaled by its physical max — taken with
    libsw's own c2r."""
    g = prob.grid
    K2 = g.kr[None, :] ** 2 + g.l[:, None] ** 2
    wf = (k0w_range[0] ** 2 <= K2) & (K2 <= k0w_range[1] ** 2)
    gf = (k0g_range[0] ** 2 <= K2) & (K2 <= k0g_range[1] ** 2)
    th = [rng.random((g.nkr, g.nl)).T for _ in range(4)]
    ph, ph0, php, phm = [np.exp(2 * np.pi * 1j * t) for t in th]
    P0, Pp, Pm = TY._bases(g)
    psith = ph * gf
    gh = [P0[i] * ph0 * gf for i in range(3)]
    wh = [(Pp[i] * php + Pm[i] * phm) * wf for i in range(3)]
    z = np.zeros_like(psith)

    def absmax(f):  # max |c2r(f)| through field ζ_T (physical id 3)
        TY.set_solution(prob, f, z, z, z)
        return float(np.max(np.abs(prob.ctx.physical(3, g.ny, g.nx))))

    mt, mg, mw = absmax(psith), absmax(gh[0]), absmax(wh[0])
    psith = psith * (at / mt) if mt > 0 else z
    gh = [x * (ag / mg) for x in gh] if mg > 0 else [z] * 3
    wh = [x * (aw / mw) for x in wh] if mw > 0 else [z] * 3
    TY.set_solution(prob, -K2 * psith, wh[0] + gh[0], wh[1] + gh[1], wh[2] + gh[2])


def ty_problem(nx=512, seed=5678, device=0, decomposition=None, **over):
    """TYdriver.start! set-up (:119-149): Problem with the Parameters.jl
    values and the seeded random-phase IC, fp64 on the GPU."""
    P = ty_parameters(nx, **over)
    prob = TY.Problem("gpu", nx=P["nx"], Lx=P["Lx"], nu=P["nu"], nnu=P["nnu"], Ro=P["Ro"], dt=P["dt"],
                      device=device, decomposition=decomposition)
    rng = np.random.default_rng(seed)
    set_ty_initial_condition(prob, rng, k0w_range=P["k0w_range"], k0g_range=P["k0g_range"], at=P["at"],
                             ag=P["ag"], aw=P["aw"])
    return prob, P


def rsw_problem(nx, stepper="FilteredAB3", seed=20261015, device=0, decomposition=None, T=np.float64, **over):
    """RSWDriver.initialize_problem (:134-176) on the GPU (fp64 compute) with the
    named stepper and the shafer random-phase IC; ``T=np.float32`` gives the
    driver's Float32 caller arrays (:164)."""
    P = rsw_parameters(nx, **over)
    kw = {"order": P["filter_order"]} if stepper == "FilteredAB3" else {}
    prob = RSW.Problem("gpu", nx=nx, Lx=P["Lx"], dt=P["dt"], f=P["f"], Cg=P["Cg"], nnu=P["nnu"],
                       nu=P["nu"], aliased_fraction=P["aliased_fraction"], stepper=stepper,
                       use_filter=(P["nutune"] == 0), T=T, device=device, decomposition=decomposition, **kw)
    rng = np.random.default_rng(seed)
    set_shafer_initial_condition(prob, P["Kg"], P["Kw"], P["ag"], P["aw"], P["f"], P["Cg"] ** 2, rng)
    return prob, P


def qg2_problem(nx, stepper="IFMAB3", seed=1234, device=0, decomposition=None, T=np.float64, **over):
    """TwoLayerDriver.initialize_problem (:29-68) on the GPU (fp64 compute;
    ``T=np.float32`` gives the driver's Float32 caller arrays)."""
    P = qg2_parameters(nx, **over)
    prob = QG2.Problem("gpu", nx=nx, Lx=P["Lx"], dt=P["dt"], f0=P["f"], Cg=P["background_Cg"],
                       U=P["U"], drhorho0=P["drhorho0"], nnu=P["nnu"], nu=P["nu"], mu=P["mu"],
                       aliased_fraction=P["aliased_fraction"], stepper=stepper, use_filter=False,
                       T=T, device=device, decomposition=decomposition)
    rng = np.random.default_rng(seed)
    set_seed_initial_condition(prob, rng)
    return prob, P


def run_frames(prob, nframes, output_freq, diags=(), on_frame=None, log_every=100):
    """The drivers' frame loop (rsw/RSWDriver.jl:205-223, swqg/TwoLayerDriver.jl:98-117):
    every log_every frames print step, t and the CFL number (device
    reduction), then stepforward!(prob, diags, output_freq) with the energy
    Diagnostics recorded on the device; a NaN makes sw_step return SW_E_NAN,
    raised as LibSWError("Solution is NaN") (the reference's throw); then the
    optional per-frame callback (updatevars!/output)."""
    from . import problem

    mod = {_lib.SW_MODEL_RSW: RSW, _lib.SW_MODEL_QG2: QG2, _lib.SW_MODEL_TY: TY,
           _lib.SW_MODEL_MLQG: MLQG}[prob.model]
    t0 = time.time()
    for frame in range(nframes):
        if log_every and frame % log_every == 0:
            print(f"step: {prob.clock.step:04d}, t: {prob.clock.t:.2f}, cfl: {mod.cfl(prob):.2e}, "
                  f"time: {(time.time() - t0) / 60:.2f} mins")
        problem.stepforward(prob, list(diags), output_freq)
        if on_frame is not None:
            on_frame(prob, frame)
