"""``RotatingShallowWater`` module mirror (rsw/RotatingShallowWater.jl).

Same names, argument meaning and defaults as the reference's ``Problem`` (:70-85);
the stepping, calcN and the linear operator all run in libsw on the GPU.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .problem import Diagnostic, Problem as _Problem, increment, stepforward  # noqa: F401


def Problem(dev="gpu", *, nx=128, ny=None, Lx=2 * np.pi, Ly=None, nu=1.0e-16, nnu=4, f=1.0, Cg=1.0,
            stepper="IFMAB3", dt=5e-2, aliased_fraction=1 / 3, T=np.float64, use_filter=False,
            device=0, check_nan=True, nop_calcN=False, unfused=False,
            decomposition=None, aliased_state=False, **stepper_kwargs):
    """``RotatingShallowWater.Problem(dev; nx, ny, Lx, Ly, ν, nν, f, Cg, stepper,
    dt, aliased_fraction, T, use_filter, stepper_kwargs...)`` (:70-99).

    ``stepper``: "IFMAB3" (reference default), "FilteredAB3" (FF, with the
    per-mode matvec L·sol of SURVEY §3.2, filter kwargs forwarded as keywords —
    the reference's positional splat at :97 is its BUG 1), or "IFMRK4".
    """
    if dev not in ("gpu", "GPU", "GPU()"):
        raise _lib.LibSWError("libsw runs on the GPU only (dev='gpu')")
    ny = nx if ny is None else ny
    Ly = Lx if Ly is None else Ly
    params = dict(nu=float(nu), nnu=int(nnu), f=float(f), Cg=float(Cg))
    prob = _Problem(_lib.SW_MODEL_RSW, nx=nx, ny=ny, Lx=Lx, Ly=Ly, dt=dt,
                    aliased_fraction=aliased_fraction, stepper=stepper, params=params,
                    use_filter=use_filter, filter_kw=stepper_kwargs, device=device,
                    check_nan=check_nan, T=T, nop_calcN=nop_calcN, unfused=unfused,
                    **(decomposition or {}), aliased_state=aliased_state)
    prob.params["Cg2"] = float(Cg) ** 2
    return prob


def set_solution(prob, u0h, v0h, eta0h):
    """``set_solution!(prob, u0h, v0h, η0h)`` (:309-321): upload + dealias."""
    prob.sol = np.stack([np.asarray(u0h), np.asarray(v0h), np.asarray(eta0h)])


def updatevars(prob):
    """``updatevars!(prob)`` (:101-116): physical u, v, η, ζ of the dealiased state."""
    g = prob.grid
    return {name: prob.ctx.physical(fid, g.ny, g.nx)
            for name, fid in (("u", _lib.SW_PHYS_U), ("v", _lib.SW_PHYS_V),
                              ("eta", _lib.SW_PHYS_ETA), ("zeta", _lib.SW_PHYS_ZETA))}


def kinetic_energy(prob):
    """``kinetic_energy(prob)`` (:323-327) of the dealiased state."""
    return prob.ctx.diag(_lib.SW_DIAG_KE)


def potential_energy(prob):
    """``potential_energy(prob)`` (:329-333)."""
    return prob.ctx.diag(_lib.SW_DIAG_PE)


def energy(prob):
    return kinetic_energy(prob) + potential_energy(prob)


def cfl(prob):
    """The drivers' CFL number clock.dt · max(max|u|/dx, max|v|/dy)
    (rsw/RSWDriver.jl:207-208), reduced on the device."""
    return prob.ctx.diag(_lib.SW_DIAG_CFL)


kinetic_energy._sw_energy = "ke"
potential_energy._sw_energy = "pe"
