"""libsw's nonlinear terms at the BASELINE sizes against the Galerkin
invariants of the equations (tests/invariants.py): oracle-independent pins of
the whole nonlinear transform chain (column inverse, row products, column
forward) on the full arrays, one slab and several.

* RotatingShallowWater (rsw/RotatingShallowWater.jl:140-230) at 2048²
  (the metric) and 4096² (config 4), divergence-free velocity, any η:
  ⟨u, N_u⟩ = ⟨v, N_v⟩ = ⟨ζ, ∂x N_v - ∂y N_u⟩ = ⟨η, N_η⟩ = 0;
* TwoLayerQG (swqg/TwoLayerQG.jl:152-182) at 2048² (config 3) and 8192²
  (config 5): ⟨q_j, N_j⟩ = ⟨ψ_j, N_j⟩ = 0 per layer, for white-noise q and
  for the stepped state of the parity case;
* MultiLayerQG (GeophysicalFlows calcN_advection!, two layers) with
  U = β = μ = 0 and the 2/3 rule at 512² (TwoLayerSimulation's grid) and
  2048²: the TwoLayerQG identities per layer;
* ThomasYamada (thomasyamada/ThomasYamada.jl:129-262) at 512² (its
  production size, thomasyamada/cpu-setup/Parameters.jl) and 2048²: the
  total-energy budget of N.

The oracle's residuals are ~1e-17 (tests/test_invariants.py); a 0.1 % error
in one term shows at ~1e-6."""
import numpy as np
import pytest

import invariants as I
import sw_cases
import sw_oracle as O

pytestmark = pytest.mark.gpu
# roundoff leaves 1e-22..1e-17 on the RSW/2LQG identities (oracle and GPU);
# the TY budget, normalised by terms that cancel, 1e-16..1e-15.  RSW's η
# budget: the row transforms η + iζ as one complex line, whose split leaves η
# an absolute error ~ eps |ζ| — on white noise |ζ| ~ 1e5 |η|, and the budget
# reads 5e-14..9e-14 on the GPU (1e-19 on the oracle, which transforms η alone)
TOL = 1e-15
TOL_ETA = 1e-12
TOL_TY = 1e-13


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


@pytest.fixture(autouse=True)
def _fft_workers():
    import os

    O.set_fft_workers(min(16, len(os.sched_getaffinity(0))))
    yield
    O.set_fft_workers(None)


def _calcN(p, sol, **kw):
    prob = sw_cases.libsw_problem(p, **kw)
    try:
        return prob.calcN(sol)
    finally:
        prob.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,slabs", [(2048, 1), (4096, 1), (4096, 4)])
def test_rsw_invariants(n, slabs):
    p = sw_cases.case_params("rsw_fab3", n)
    grid = O.TwoDGrid(n)
    sol = I.rsw_state(grid, seed=n + 1)
    kw = dict(decomposition=dict(nranks=slabs, local_slabs=slabs)) if slabs > 1 else {}
    N = _calcN(p, sol, **kw)
    r = I.rsw_residuals(grid, sol, N)
    print(f"rsw {n}² slabs={slabs}: {r}")
    assert max(r["u"], r["v"], r["vorticity"]) < TOL, r
    assert r["eta"] < TOL_ETA, r
    assert np.max(np.abs(N)) > 0


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,slabs", [(2048, 1), (8192, 1), (8192, 8)])
def test_qg2_invariants(n, slabs):
    p = sw_cases.case_params("qg2_ifmrk4", n)
    grid = O.TwoDGrid(n)
    params = O.QG2Params(p["U"], p["mu"], p["nu"], p["nnu"], F=p["F"])
    kw = dict(decomposition=dict(nranks=slabs, local_slabs=slabs)) if slabs > 1 else {}
    q = I.random_real_spectrum(grid, 2, seed=n + 2)
    N = _calcN(p, q, **kw)
    r = I.qg2_residuals(grid, q, O.qg2_streamfunction(q, grid, params), N)
    print(f"qg2 {n}² slabs={slabs} white noise: {r}")
    assert max(r.values()) < TOL, r
    if slabs == 1:
        # a stepped state: the parity case's initial condition after 2 steps
        prob = sw_cases.libsw_problem(p)
        try:
            prob.sol = sw_cases.initial_condition(p, grid)
            prob.stepforward(2)
            q = prob.sol
            N = prob.calcN(q)
        finally:
            prob.close()
        grid.dealias(q)
        r = I.qg2_residuals(grid, q, O.qg2_streamfunction(q, grid, params), N)
        print(f"qg2 {n}² stepped: {r}")
        assert max(r.values()) < TOL, r


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,slabs", [(512, 1), (2048, 1), (2048, 2)])
def test_ty_invariants(n, slabs):
    p = sw_cases.case_params("ty_etdrk4", n)
    grid = O.TwoDGrid(n, Lx=p["Lx"])
    sol = I.random_real_spectrum(grid, 4, seed=n + 3)
    kw = dict(decomposition=dict(nranks=slabs, local_slabs=slabs)) if slabs > 1 else {}
    N = _calcN(p, sol, **kw)
    r = I.ty_residuals(grid, sol, N)
    print(f"ty {n}² slabs={slabs}: {r}")
    assert r["energy"] < TOL_TY, r


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n,slabs", [(512, 1), (2048, 1), (2048, 2)])
def test_mlqg_invariants(n, slabs):
    p = dict(sw_cases.case_params("mlqg_frk4", n), U=[0.0, 0.0], beta=0.0, mu=0.0, af=1 / 3)
    grid = O.TwoDGrid(n)
    params = O.MLQGParams(p["f0"], p["H"], p["b"], p["U"], p["mu"], p["beta"], p["nu"], p["nnu"])
    q = I.random_real_spectrum(grid, 2, seed=n + 4)
    kw = dict(decomposition=dict(nranks=slabs, local_slabs=slabs)) if slabs > 1 else {}
    N = _calcN(p, q, **kw)
    r = I.qg2_residuals(grid, q, O.mlqg_streamfunction(q, grid, params), N)
    print(f"mlqg {n}² slabs={slabs}: {r}")
    assert max(r.values()) < TOL, r
