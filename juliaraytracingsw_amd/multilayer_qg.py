"""``GeophysicalFlows.MultiLayerQG`` mirror for two layers, as
simulation/TwoLayerSimulation.jl:37-47 builds it.

GeophysicalFlows is not vendored in the reference; libsw restates its
MultiLayerQG (2 layers, no topography) from the package's published
equations: q_j = ∇²ψ_j + stretching with F_j = f₀²/(g′ H_j), g′ = b₁ − b₂,

    ∂t q_j + J(ψ_j, q_j) + U_j ∂x q_j + Qy_j ∂x ψ_j = δ_{j,2} μ K² ψ̂_2 − ν K^(2nν) q̂_j,
    Qy₁ = β − F₁(U₂ − U₁),  Qy₂ = β − F₂(U₁ − U₂),

stepped by FourierFlows' FilteredRK4.  The nonlinear term runs through the
2LQG transform kernels; the mean-flow, background-gradient and drag terms are
added per mode in the column pass.  Parity is against the oracle's
restatement (unpinned against GeophysicalFlows itself), which the analytic
two-layer baroclinic growth rate pins.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .problem import Diagnostic, Problem as _Problem, increment, stepforward  # noqa: F401


def Problem(nlayers=2, dev="gpu", *, nx=128, ny=None, Lx=2 * np.pi, Ly=None, f0=1.0, beta=0.0,
            H=(0.5, 0.5), b=(1.0, 0.0), U=(0.0, 0.0), mu=0.0, nu=0.0, nnu=1, dt=0.01,
            stepper="FilteredRK4", aliased_fraction=1 / 3, T=np.float64, device=0, check_nan=True,
            unfused=False, decomposition=None, aliased_state=False, **stepper_kwargs):
    """``MultiLayerQG.Problem(nlayers, dev; nx, Lx, f₀, H, b, U, μ, β, ν, nν, dt,
    stepper, aliased_fraction)``; nlayers must be 2 (TwoLayerSimulation's).
    ``aliased_state=True`` also carries the modes dealias! removes (with
    aliased_fraction = 0 the Nyquist column and row), as GF's prob.sol holds
    them between steps: calcN! returns N there and the FilteredRK4 update
    writes filter·dt·(N₁/6 + N₂/3 + N₃/3 + N₄/6) into them."""
    if nlayers != 2:
        raise _lib.LibSWError("libsw's MultiLayerQG has nlayers = 2")
    if dev not in ("gpu", "GPU", "GPU()"):
        raise _lib.LibSWError("libsw runs on the GPU only (dev='gpu')")
    ny = nx if ny is None else ny
    Ly = Lx if Ly is None else Ly
    params = dict(f0=float(f0), beta=float(beta), H=list(H), b=list(b), Ulayer=list(U), mu=float(mu),
                  nu=float(nu), nnu=int(nnu))
    prob = _Problem(_lib.SW_MODEL_MLQG, nx=nx, ny=ny, Lx=Lx, Ly=Ly, dt=dt, aliased_fraction=aliased_fraction,
                    stepper=stepper, params=params, filter_kw=stepper_kwargs, device=device,
                    check_nan=check_nan, T=T, unfused=unfused, aliased_state=aliased_state,
                    **(decomposition or {}))
    gp = b[0] - b[1]
    prob.params.update(F1=f0 ** 2 / (gp * H[0]), F2=f0 ** 2 / (gp * H[1]))
    return prob


def set_q(prob, q0):
    """``set_q!(prob, q0)``: q0 physical [2][ny][nx]; the r2c of each layer
    (host numpy, once at set-up) then upload + dealias."""
    prob.sol = np.fft.rfft2(np.asarray(q0, np.float64), axes=(-2, -1))


def pvfromstreamfunction(prob, psih):
    """``pvfromstreamfunction!``: q̂ = S ψ̂ per mode (set-up from a streamfunction)."""
    g = prob.grid
    K2 = g.kr[None, :] ** 2 + g.l[:, None] ** 2
    F1, F2 = prob.params["F1"], prob.params["F2"]
    return np.stack([(-K2 - F1) * psih[0] + F1 * psih[1], F2 * psih[0] + (-K2 - F2) * psih[1]])


def updatevars(prob):
    """``updatevars!(prob)``: q, ψ, u, v (and ζ) per layer, each [2][ny][nx]."""
    g = prob.grid
    out = {}
    for name, fid in (("q", _lib.SW_PHYS_Q), ("psi", _lib.SW_PHYS_PSI), ("zeta", _lib.SW_PHYS_ZETA),
                      ("u", _lib.SW_PHYS_U), ("v", _lib.SW_PHYS_V)):
        out[name] = np.stack([prob.ctx.physical(layer * 8 + fid, g.ny, g.nx) for layer in (0, 1)])
    return out


def energies(prob):
    """``MultiLayerQG.energies(prob)`` -> ((KE₁, KE₂), (PE,)), reduced on the device."""
    return ((prob.ctx.diag(_lib.SW_DIAG_KE1), prob.ctx.diag(_lib.SW_DIAG_KE2)), (prob.ctx.diag(_lib.SW_DIAG_PE),))


def cfl(prob):
    """clock.dt · max(maximum(u)/dx, maximum(v)/dy) over both layers
    (simulation/TwoLayerSimulation.jl:124, signed maxima), on the device."""
    return prob.ctx.diag(_lib.SW_DIAG_CFL)


energies._sw_energy = "mlqg"
