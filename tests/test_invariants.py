"""The oracle's nonlinear terms against the Galerkin invariants of the
equations (tests/invariants.py): an oracle-independent pin of the restated
calcN (rsw/RotatingShallowWater.jl:140-230, swqg/TwoLayerQG.jl:152-182),
and a check that the identities fail loudly on a perturbed N."""
import numpy as np
import pytest

import invariants as I
import sw_cases
import sw_oracle as O

TOL = 1e-13


@pytest.mark.parametrize("n", [64, 128])
def test_oracle_rsw_invariants(n):
    p = sw_cases.case_params("rsw_fab3", n)
    grid = O.TwoDGrid(n)
    sol = I.rsw_state(grid, seed=11)
    N = O.rsw_calcN(sol.copy(), grid, O.RSWParams(p["nu"], p["nnu"], p["f"], p["Cg"]))
    r = I.rsw_residuals(grid, sol, N)
    assert max(r.values()) < TOL, r
    # the identities are not vacuous (roundoff leaves ~1e-17): a 0.1 % error
    # in N_u breaks the vorticity one (~1e-6), N_u without its v ∂y u term
    # (:193-197) too (~1e-3), and N_η without its ∂y(vη) term (:224-226) the η one
    bad = N.copy()
    bad[0] *= 1.001
    assert I.rsw_residuals(grid, sol, bad)["vorticity"] > 1e-8
    l = grid.l[:, None]
    bad = N.copy()
    bad[0] += grid.rfft(grid.irfft(1j * l * sol[0]) * grid.irfft(sol[1]))
    assert I.rsw_residuals(grid, sol, bad)["vorticity"] > 1e-5
    bad = N.copy()
    bad[2] += 1j * l * grid.rfft(grid.irfft(sol[1]) * grid.irfft(sol[2]))
    assert I.rsw_residuals(grid, sol, bad)["eta"] > 1e-5


@pytest.mark.parametrize("n", [64, 128])
def test_oracle_qg2_invariants(n):
    p = sw_cases.case_params("qg2_ifmrk4", n)
    grid = O.TwoDGrid(n)
    q = I.random_real_spectrum(grid, 2, seed=12)
    params = O.QG2Params(p["U"], p["mu"], p["nu"], p["nnu"], F=p["F"])
    psi = O.qg2_streamfunction(q, grid, params)
    N = O.qg2_calcN(q.copy(), grid, params)
    r = I.qg2_residuals(grid, q, psi, N)
    assert max(r.values()) < TOL, r
    # an x-derivative with the wrong sign on one term is caught
    kr, l = grid.kr[None, :], grid.l[:, None]
    psixq = grid.irfft(1j * kr * psi) * grid.irfft(q)
    bad = N + 2j * l * grid.rfft(psixq)  # flips the sign of the ψx q term
    assert min(I.qg2_residuals(grid, q, psi, bad).values()) > 1e-5


@pytest.mark.parametrize("n", [64, 128])
def test_oracle_ty_invariants(n):
    p = sw_cases.case_params("ty_etdrk4", n)
    grid = O.TwoDGrid(n, Lx=p["Lx"])
    sol = I.random_real_spectrum(grid, 4, seed=13)
    N = O.ty_calcN(sol.copy(), grid, O.TYParams(p["nu"], p["nnu"], p["Ro"]))
    r = I.ty_residuals(grid, sol, N)
    assert r["energy"] < TOL, r
    bad = N.copy()
    bad[3] *= 1.001  # 0.1 % on the pressure tendency
    assert I.ty_residuals(grid, sol, bad)["energy"] > 1e-8


@pytest.mark.parametrize("n", [64, 128])
def test_oracle_mlqg_invariants(n):
    """MultiLayerQG with U = β = μ = 0 (no background PV gradient, no drag)
    and the 2/3 rule: N_j = -J(ψ_j, q_j) per layer, as TwoLayerQG's."""
    p = sw_cases.case_params("mlqg_frk4", n)
    grid = O.TwoDGrid(n)
    params = O.MLQGParams(p["f0"], p["H"], p["b"], [0.0, 0.0], 0.0, 0.0, p["nu"], p["nnu"])
    q = I.random_real_spectrum(grid, 2, seed=14)
    N = O.mlqg_calcN(q.copy(), grid, params)
    r = I.qg2_residuals(grid, q, O.mlqg_streamfunction(q, grid, params), N)
    assert max(r.values()) < TOL, r


def test_divergence_free_state():
    grid = O.TwoDGrid(64)
    s = I.rsw_state(grid, seed=3)
    kr, l = grid.kr[None, :], grid.l[:, None]
    div = 1j * kr * s[0] + 1j * l * s[1]
    assert np.max(np.abs(div)) <= 1e-12 * np.max(np.abs(s[0]))
