"""``ThomasYamada`` module mirror (thomasyamada/ThomasYamada.jl).

Same names, argument meaning and defaults as the reference's ``Problem``
(:55-74): fields (ζ_T, u_c, v_c, p_c), a real diagonal L = -ν K^(2nν) on all
four fields (:265-277), stepped by FourierFlows' ``ETDRK4`` (the default
``stepper``).  calcN (:129-262), the ETDRK4 coefficient table and every stage
run in libsw on the GPU.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .problem import Diagnostic, Problem as _Problem, increment, stepforward  # noqa: F401


def Problem(dev="gpu", *, nx=128, ny=None, Lx=2 * np.pi, Ly=None, nu=3.5e-25, nnu=8, Ro=0.2,
            stepper="ETDRK4", dt=5e-2, aliased_fraction=1 / 3, T=np.float64, device=0,
            check_nan=True, unfused=False, decomposition=None, aliased_state=False):
    """``ThomasYamada.Problem(dev; nx, ny, Lx, Ly, ν, nν, Ro, stepper, dt,
    aliased_fraction, T)`` (:55-74).  ``stepper`` must be "ETDRK4" (the only
    stepper the reference runs this model with, cpu-setup/Parameters.jl:12).

    ``aliased_state=True`` also carries the modes the 2/3 rule removes, as
    the reference's prob.sol holds them between steps: calcN! dealiases its
    input in place (:130) but returns N on every mode, and the ETDRK4 update
    writes α N₁ + 2β (N₂ + N₃) + Γ N₄ there (the energies, :333-360, count
    them; the next calcN!/updatevars! discards them).  Off by default: the
    modes never reach a dealiased quantity."""
    if dev not in ("gpu", "GPU", "GPU()"):
        raise _lib.LibSWError("libsw runs on the GPU only (dev='gpu')")
    if stepper != "ETDRK4":
        raise _lib.LibSWError("the Thomas-Yamada model is stepped with ETDRK4")
    ny = nx if ny is None else ny
    Ly = Lx if Ly is None else Ly
    params = dict(nu=float(nu), nnu=int(nnu), Ro=float(Ro))
    return _Problem(_lib.SW_MODEL_TY, nx=nx, ny=ny, Lx=Lx, Ly=Ly, dt=dt,
                    aliased_fraction=aliased_fraction, stepper=stepper, params=params,
                    device=device, check_nan=check_nan, T=T, unfused=unfused,
                    aliased_state=aliased_state, **(decomposition or {}))


def set_solution(prob, zeta0h, u0h, v0h, p0h):
    """``set_solution!(prob, ζ0h, u0h, v0h, p0h)`` (:279-306): upload + dealias."""
    prob.sol = np.stack([np.asarray(zeta0h), np.asarray(u0h), np.asarray(v0h), np.asarray(p0h)])


def updatevars(prob):
    """``updatevars!(prob)`` (:67-92): physical ζ_T, u_c, v_c, p_c, u_T, v_T,
    q_c (and ψ_T) of the dealiased state, each [ny][nx]."""
    g = prob.grid
    ids = (("zt", 3), ("uc", 0), ("vc", 1), ("pc", 2), ("ut", 8), ("vt", 9), ("qc", 4), ("psit", 5))
    return {name: prob.ctx.physical(fid, g.ny, g.nx) for name, fid in ids}


def enforce_reality_condition(prob):
    """``enforce_reality_condition!(prob)`` (:103-123): ``dealias!(sol)``, the
    spectral and physical vars, then ``mul!(sol[:,:,k], grid.rfftplan, …)``
    for each field.  In Julia ``sol[:,:,k]`` (no ``@views``) is a copy, so
    those r2c's write into temporaries and the state is left as it is: the
    function amounts to ``dealias!`` + ``updatevars!`` — which is what this
    does (libsw's updatevars! dealiases an aliased_state problem's state
    first).  Returns the physical vars."""
    return updatevars(prob)


def baroclinic_energy(prob):
    """``baroclinic_energy(prob)`` (:333-342): (|u_c|² + |v_c|², |p_c|²) by
    parsevalsum2, reduced on the device."""
    return (prob.ctx.diag(_lib.SW_DIAG_KE), prob.ctx.diag(_lib.SW_DIAG_PE))


def barotropic_energy(prob):
    """``barotropic_energy(prob)`` (:344-351): parsevalsum2(K⁻¹ ζ_T)."""
    return prob.ctx.diag(_lib.SW_DIAG_BT)


def _bases(grid):
    """thomasyamada/TYUtils.jl:10-38: Φ₀, Φ₊, Φ₋ per mode, each [3][nl][nkr]
    (host set-up of the driver's initial condition)."""
    kr = grid.kr[None, :]
    l = grid.l[:, None]
    K2 = kr ** 2 + l ** 2
    om = np.sqrt(1 + K2)
    with np.errstate(divide="ignore"):
        iK2 = np.where(K2 == 0, 0.0, 1.0 / K2)
    s = np.sqrt(iK2 / 2) / om
    one = np.ones_like(K2)
    P0 = np.stack([1j * l / om * one, -1j * kr / om * one, -1 / om + 0j])
    Pp = np.stack([(om * kr + 1j * l) * s, (om * l - 1j * kr) * s, (om ** 2 - 1) * s + 0j])
    Pm = np.stack([(-om * kr + 1j * l) * s, (-om * l - 1j * kr) * s, (om ** 2 - 1) * s + 0j])
    P0[:, 0, 0] = [0, 0, 1]
    Pp[:, 0, 0] = np.array([1j, 1, 0]) / np.sqrt(2)
    Pm[:, 0, 0] = np.array([1j, -1, 0]) / np.sqrt(2)
    return P0, Pp, Pm


def wave_geostrophic_energy(prob):
    """``wave_geostrophic_energy(prob)`` (:353-367) via
    ``decompose_balanced_wave`` (thomasyamada/TYUtils.jl:40-51): ((wave KE,
    wave PE), (geostrophic KE, geostrophic PE)), the per-mode projection on
    Φ₀, Φ₊, Φ₋ and its Parseval sums reduced on the device (k_energy_cols)."""
    d = prob.ctx.diag
    return ((d(_lib.SW_DIAG_WAVE_KE), d(_lib.SW_DIAG_WAVE_PE)),
            (d(_lib.SW_DIAG_GEO_KE), d(_lib.SW_DIAG_GEO_PE)))


def cfl(prob):
    """clock.dt · max(maximum(u_c)/dx, maximum(v_c)/dy, maximum(u_T)/dx,
    maximum(v_T)/dy) (thomasyamada/TYdriver.jl:150-151: signed maxima),
    reduced on the device."""
    return prob.ctx.diag(_lib.SW_DIAG_CFL)


baroclinic_energy._sw_energy = "bc"
barotropic_energy._sw_energy = "bt"
wave_geostrophic_energy._sw_energy = "wg"
