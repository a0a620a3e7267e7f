"""``TwoLayerQG`` module mirror (swqg/TwoLayerQG.jl).

Same names, argument meaning and defaults as the reference's ``Problem``
(:55-72), including F = 2 f0²/Cg²/δρρ0 (:79) and the Complex{Float32} literal
quirk of its linear operator (:189-193), which libsw reproduces bit for bit.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .problem import Diagnostic, Problem as _Problem, increment, stepforward  # noqa: F401


def Problem(dev="gpu", *, nx=128, ny=None, Lx=2 * np.pi, Ly=None, U=0.5, mu=1e-2, nu=1e-6, nnu=4,
            f0=3.0, Cg=1.0, drhorho0=0.2, stepper="IFMAB3", dt=5e-2, aliased_fraction=1 / 3,
            T=np.float32, use_filter=False, device=0, check_nan=True, nop_calcN=False, unfused=False,
            decomposition=None, aliased_state=False, **stepper_kwargs):
    """``TwoLayerQG.Problem(dev; nx, ny, Lx, Ly, U, μ, ν, nν, f0, Cg, δρρ0, stepper,
    dt, aliased_fraction, T, use_filter, stepper_kwargs...)`` (:55-90).

    ``T`` (default Float32, as the reference's :70) is the element type of
    the caller-side arrays (``prob.sol``, ``updatevars``); libsw computes in
    fp64 either way (BASELINE parity precision) and rounds once on output.
    ``aliased_state=True`` also carries the modes the 2/3 rule removes, so
    ``prob.sol``, calcN and the energy diagnostics cover the full array as
    the reference's do (slabs of one process; include/sw.h).
    """
    if dev not in ("gpu", "GPU", "GPU()"):
        raise _lib.LibSWError("libsw runs on the GPU only (dev='gpu')")
    ny = nx if ny is None else ny
    Ly = Lx if Ly is None else Ly
    F = 2 * f0 ** 2 / Cg ** 2 / drhorho0
    params = dict(U=float(U), mu=float(mu), nu=float(nu), nnu=int(nnu), F=float(F))
    prob = _Problem(_lib.SW_MODEL_QG2, nx=nx, ny=ny, Lx=Lx, Ly=Ly, dt=dt,
                    aliased_fraction=aliased_fraction, stepper=stepper, params=params,
                    use_filter=use_filter, filter_kw=stepper_kwargs, device=device,
                    check_nan=check_nan, T=T, nop_calcN=nop_calcN, unfused=unfused,
                    aliased_state=aliased_state, **(decomposition or {}))
    return prob


def set_solution(prob, q0h):
    """``set_solution!(prob, q0h)`` (:220-228): upload + dealias."""
    prob.sol = np.asarray(q0h)


def updatevars(prob):
    """``updatevars!(prob)`` (:113-129): q, ψ, ζ, u, v per layer, shape [2][ny][nx]."""
    g = prob.grid
    out = {}
    for name, fid in (("q", _lib.SW_PHYS_Q), ("psi", _lib.SW_PHYS_PSI), ("zeta", _lib.SW_PHYS_ZETA),
                      ("u", _lib.SW_PHYS_U), ("v", _lib.SW_PHYS_V)):
        out[name] = np.stack([prob.ctx.physical(layer * 8 + fid, g.ny, g.nx) for layer in (0, 1)])
    return out


def kinetic_energy(prob):
    """``kinetic_energy(prob)`` (:230-240): the tuple (KE_1, KE_2) of the layers."""
    return (prob.ctx.diag(_lib.SW_DIAG_KE1), prob.ctx.diag(_lib.SW_DIAG_KE2))


def potential_energy(prob):
    """``potential_energy(prob)`` (:244-250)."""
    return prob.ctx.diag(_lib.SW_DIAG_PE)


def cfl(prob):
    """clock.dt · max(max|u|/dx, max|v|/dy) over both layers
    (swqg/TwoLayerDriver.jl:100-101), reduced on the device."""
    return prob.ctx.diag(_lib.SW_DIAG_CFL)


kinetic_energy._sw_energy = "ke12"
potential_energy._sw_energy = "pe"
