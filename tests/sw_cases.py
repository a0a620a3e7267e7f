"""Parity case definitions shared by the golden generator and the tests.

Each case = (model, stepper, grid size, parameters, IC).  Parameters follow the
reference drivers (rsw/RSWDriver.jl:134-148, swqg/TwoLayerDriver.jl:29-63);
small grids use a larger CFL and an annulus moved inside the live band so the
nonlinear terms are exercised within a few steps.
"""
from __future__ import annotations

import numpy as np

import sw_oracle as O

CASES = ["rsw_fab3", "rsw_ifmab3", "rsw_ifmrk4", "qg2_ifmab3", "qg2_ifmrk4", "qg2_fab3"]
# Thomas–Yamada (thomasyamada/ThomasYamada.jl) stepped by FF ETDRK4
TY_CASES = ["ty_etdrk4"]
# GeophysicalFlows MultiLayerQG (2 layers, aliased_fraction = 0) stepped by
# FF FilteredRK4, as simulation/TwoLayerSimulation.jl runs it
MLQG_CASES = ["mlqg_frk4"]
ALL_CASES = CASES + TY_CASES + MLQG_CASES


def case_params(name, n):
    model, st = name.split("_", 1)
    stepper = {"fab3": "FilteredAB3", "ifmab3": "IFMAB3", "ifmrk4": "IFMRK4", "etdrk4": "ETDRK4",
               "frk4": "FilteredRK4"}[st]
    if model == "mlqg":
        # simulation/Parameters.jl (f = 1, rd = 1/15, ℓ = 1/2, avg_U = 0.1, H =
        # [1/2, 1/2], nν = 8, ν = 0, dt = 0.02 dx/avg_U), aliased_fraction = 0;
        # small grids: a larger PV amplitude so J(ψ, q) matters within steps
        P = O.mlqg_simulation_params(n)
        return dict(model="mlqg", stepper=stepper, n=n, af=0.0, dt=P["dt"], f0=P["f0"], H=P["H"], b=P["b"],
                    U=P["U"], mu=P["mu"], beta=P["beta"], nu=P["nu"], nnu=P["nnu"],
                    amp=0.5 if n <= 256 else P["q0_amplitude"], seed=1234)
    if model == "ty":
        # thomasyamada/cpu-setup/Parameters.jl: Lx = 6π, ν = 5e-34 (Lx/2π)^16,
        # nν = 8, Ro = 1, dt = 5e-3; annuli k0g = (10/3, 13/3), k0w = (0, 5/3).
        # Small grids: larger dt and (32²) annuli inside the live band; a
        # small barotropic amplitude so every term of calcN is active at once.
        Lx = 6 * np.pi
        kg, kw = ((4 / 3, 2.0), (0.0, 1.0)) if n <= 32 else ((10 / 3, 13 / 3), (0.0, 5 / 3))
        return dict(model="ty", stepper=stepper, n=n, Lx=Lx, dt=2e-2 if n <= 256 else 5e-3,
                    nu=5.0e-34 * (Lx / (2 * np.pi)) ** 16, nnu=8, Ro=1.0, k0g=kg, k0w=kw,
                    at=0.1, ag=0.3, aw=0.1, seed=5678)
    if model == "rsw":
        cfl = 0.05 if n <= 256 else 0.01
        nut = 20.0
        if stepper == "FilteredAB3" and n < 2048:
            # explicit steppers treat ν·K^8 explicitly: keep dt·ν·kmax^8 (= νtune·dx)
            # well below its 2048² driver value on the coarse test grids
            nut, cfl = 20.0 * n / 2048 * 0.25, cfl * 0.5
        dt, nu = O.rsw_driver_params(n, cfltune=cfl, nutune=nut)
        Kg, Kw = ((4, 6), (0, 3)) if n <= 64 else ((10, 13), (0, 5))
        return dict(model="rsw", stepper=stepper, n=n, dt=dt, nu=nu, nnu=4, f=3.0, Cg=1.0,
                    Kg=Kg, Kw=Kw, ag=0.2, aw=0.1, order=8, seed=20261015)
    if stepper == "FilteredAB3" and n < 2048:
        P = O.qg2_driver_params(n, nutune=40.0 * n / 2048 * 0.25, cfltune=0.0125)
    else:
        P = O.qg2_driver_params(n)
    return dict(model="qg2", stepper=stepper, n=n, dt=P["dt"], nu=P["nu"], nnu=4, U=P["U"], mu=P["mu"],
                F=P["F"], f0=3.0, Cg=1.0, drhorho0=P["drhorho0"], amp=0.5 if n <= 256 else 1e-2,
                order=8, seed=1234)


def oracle_problem(p, expm="scipy"):
    """the oracle Problem of a case; expm: its integrating factors' matrix
    exponential (sw_oracle.expm_modes: scipy's expm, or "closed")"""
    if p["model"] == "mlqg":
        params = O.MLQGParams(p["f0"], p["H"], p["b"], p["U"], p["mu"], p["beta"], p["nu"], p["nnu"])
        return O.Problem("mlqg", p["stepper"], p["n"], p["dt"], aliased_fraction=p["af"], params=params)
    if p["model"] == "ty":
        return O.Problem("ty", "ETDRK4", p["n"], p["dt"], Lx=p["Lx"],
                         params=O.TYParams(p["nu"], p["nnu"], p["Ro"]))
    if p["model"] == "rsw":
        params = O.RSWParams(p["nu"], p["nnu"], p["f"], p["Cg"])
    else:
        params = O.QG2Params(p["U"], p["mu"], p["nu"], p["nnu"], F=p["F"])
    fk = dict(order=p["order"]) if p["stepper"] == "FilteredAB3" else {}
    return O.Problem(p["model"], p["stepper"], p["n"], p["dt"], params=params, expm=expm, **fk)


def initial_condition(p, grid):
    rng = np.random.default_rng(p["seed"])
    if p["model"] == "mlqg":
        # simulation/TwoLayerSimulation.jl:50-53: q₀ = a·randn, q̂₀ = filter·rfft(q₀)
        q0 = p["amp"] * rng.standard_normal((2, grid.ny, grid.nx))
        return O.makefilter(grid)[None] * grid.rfft(q0)
    if p["model"] == "ty":
        return O.ty_initial_condition(grid, rng, k0w_range=p["k0w"], k0g_range=p["k0g"],
                                      at=p["at"], ag=p["ag"], aw=p["aw"])
    if p["model"] == "rsw":
        return O.shafer_ic(grid, p["Kg"], p["Kw"], p["ag"], p["aw"], p["f"], p["Cg"] ** 2, rng)
    q0 = p["amp"] * rng.standard_normal((2, grid.ny, grid.nx))
    return grid.rfft(q0)


def libsw_problem(p, **kw):
    """The GPU problem for the same case, through the package's public mirror."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW, thomas_yamada as TY, two_layer_qg as QG2

    if p["model"] == "mlqg":
        from juliaraytracingsw_amd import multilayer_qg as MLQG

        return MLQG.Problem(2, "gpu", nx=p["n"], f0=p["f0"], H=p["H"], b=p["b"], U=p["U"], mu=p["mu"],
                            beta=p["beta"], nu=p["nu"], nnu=p["nnu"], dt=p["dt"], stepper=p["stepper"],
                            aliased_fraction=p["af"], **kw)
    if p["model"] == "ty":
        return TY.Problem("gpu", nx=p["n"], Lx=p["Lx"], dt=p["dt"], nu=p["nu"], nnu=p["nnu"], Ro=p["Ro"], **kw)
    fk = dict(order=p["order"]) if p["stepper"] == "FilteredAB3" else {}
    if p["model"] == "rsw":
        return RSW.Problem("gpu", nx=p["n"], dt=p["dt"], nu=p["nu"], nnu=p["nnu"], f=p["f"], Cg=p["Cg"],
                           stepper=p["stepper"], **fk, **kw)
    return QG2.Problem("gpu", nx=p["n"], dt=p["dt"], nu=p["nu"], nnu=p["nnu"], U=p["U"], mu=p["mu"],
                       f0=p["f0"], Cg=p["Cg"], drhorho0=p["drhorho0"], stepper=p["stepper"],
                       T=kw.pop("T", np.float64), **fk, **kw)
