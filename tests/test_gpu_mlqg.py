"""GPU parity of GeophysicalFlows' MultiLayerQG (2 layers, aliased_fraction =
0) stepped by FourierFlows' FilteredRK4, as simulation/TwoLayerSimulation.jl
runs it, against the oracle's restatement through the C
ABI.  GeophysicalFlows is not vendored: parity is UNPINNED against GF itself;
the restatement is pinned by the analytic Phillips growth rate
(tests/test_oracle.py).  Tolerance: max|a−b|/max|b| over live modes ≤ 1e-10."""
import numpy as np
import pytest

import sw_cases
import sw_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _pair(name, n, **over):
    p = dict(sw_cases.case_params(name, n), **over)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    return p, pr, prob


@pytest.mark.parametrize("n", [64, 128, 256])
def test_mlqg_calcN_and_steps(n):
    p, pr, prob = _pair("mlqg_frk4", n)
    N_gpu = prob.calcN(pr.sol)
    N_cpu = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    assert O.parity_error(N_gpu, N_cpu, pr.grid) < RTOL
    for nsteps in (1, 3, 6):
        pr.stepforward(nsteps)
        prob.stepforward(nsteps)
        e = O.parity_error(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (nsteps, e)
    prob.close()


def test_mlqg_simulation_config():
    """simulation/Parameters.jl: 512², aliased_fraction = 0, amplitude 1e-3."""
    p, pr, prob = _pair("mlqg_frk4", 512)
    pr.stepforward(3)
    prob.stepforward(3)
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


def test_mlqg_unequal_layers_beta_drag_viscosity():
    """Every term of the restated equations at once: H₁ ≠ H₂ (F₁ ≠ F₂), β,
    bottom drag, hyperviscosity, dealiased grid."""
    p, pr, prob = _pair("mlqg_frk4", 128, H=[0.3, 0.7], beta=2.0, mu=0.05, nu=1e-12, nnu=4, af=1 / 3)
    N_gpu = prob.calcN(pr.sol)
    assert O.parity_error(N_gpu, pr.calcN(pr.sol.copy(), pr.grid, pr.params), pr.grid) < RTOL
    pr.stepforward(5)
    prob.stepforward(5)
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


def test_mlqg_filtered_ab3():
    """simulation/FreelyEvolvingSimulation.jl:38-39 steps MultiLayerQG with
    FreelyEvolvingParameters.jl:7's FilteredAB3 (aliased_fraction = 0):
    forward Euler for clock.step < 3, AB3 after, filter after each update;
    L = −νK^(2nν) per layer added to N (addlinearterm!)."""
    p, pr, prob = _pair("mlqg_frk4", 128, stepper="FilteredAB3", nu=1e-16, nnu=4)
    for nsteps in (1, 2, 4):
        pr.stepforward(nsteps)
        prob.stepforward(nsteps)
        e = O.parity_error(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (nsteps, e)
    prob.close()


@pytest.mark.parametrize("name", ["rsw_fab3", "qg2_ifmab3"])
def test_filtered_rk4_other_models(name):
    """FF FilteredRK4 is generic: RSW (3×3 L matvec) and 2LQG (2×2, with the
    Float32 literal quirk) step with it too."""
    p = dict(sw_cases.case_params(name, 128), stepper="FilteredRK4")
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    pr.stepforward(4)
    prob.stepforward(4)
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


def test_mlqg_physical_energy_cfl_diagnostics():
    from juliaraytracingsw_amd import multilayer_qg as MLQG

    p, pr, prob = _pair("mlqg_frk4", 128)
    E = MLQG.Diagnostic(MLQG.energies, prob, freq=2, nsteps=4)
    expected = [O.mlqg_energies(pr.sol, pr.grid, pr.params)]
    for s in range(1, 5):
        pr.stepforward(1)
        if s % 2 == 0:
            expected.append(O.mlqg_energies(pr.grid.dealias(pr.sol.copy()), pr.grid, pr.params))
    MLQG.stepforward(prob, [E], 4)
    assert E.i == 3
    for i, ((k1, k2), pe) in enumerate(expected):
        (a, b), (c,) = E.data[i]
        np.testing.assert_allclose([a, b, c], [k1, k2, pe], rtol=RTOL)
    g = pr.grid
    sol = g.dealias(pr.sol.copy())
    psih = O.mlqg_streamfunction(sol, g, pr.params)
    got = MLQG.updatevars(prob)
    for name, ref in (("q", g.irfft(sol)), ("psi", g.irfft(psih)), ("u", g.irfft(-1j * g.l[:, None] * psih)),
                      ("v", g.irfft(1j * g.kr[None, :] * psih))):
        assert np.max(np.abs(got[name] - ref)) < 1e-10 * np.max(np.abs(ref)), name
    u, v = g.irfft(-1j * g.l[:, None] * psih), g.irfft(1j * g.kr[None, :] * psih)
    exp = p["dt"] * max(u.max() / g.dx, v.max() / g.dy)
    assert abs(MLQG.cfl(prob) / exp - 1) < 1e-10
    prob.close()


@pytest.mark.parametrize("nx,ny", [(256, 64), (64, 256)])
@pytest.mark.parametrize("model", ["mlqg", "ty"])
def test_rectangular_ty_mlqg(model, nx, ny):
    """Rectangular grids (Lx ≠ Ly too) for the Thomas–Yamada and MultiLayerQG
    paths: separate x and y wavenumber spacings everywhere (k_row's ik,
    k_col_inv's il, the per-mode linear terms, the ETDRK4 table, the filter)."""
    from juliaraytracingsw_amd import multilayer_qg as MLQG, thomas_yamada as TY

    rng = np.random.default_rng(11)
    Lx, Ly = 2 * np.pi * nx / 128, 2 * np.pi * ny / 128
    if model == "mlqg":
        P = O.mlqg_simulation_params(128)
        params = O.MLQGParams(P["f0"], P["H"], P["b"], P["U"], P["mu"], 0.5, 1e-14, 4)
        pr = O.Problem("mlqg", "FilteredRK4", nx, 0.01, Lx=Lx, ny=ny, Ly=Ly, aliased_fraction=0, params=params)
        prob = MLQG.Problem(2, "gpu", nx=nx, ny=ny, Lx=Lx, Ly=Ly, f0=P["f0"], H=P["H"], b=P["b"], U=P["U"],
                            mu=P["mu"], beta=0.5, nu=1e-14, nnu=4, dt=0.01, aliased_fraction=0)
        nf = 2
    else:
        params = O.TYParams(1e-12, 4, 1.0)
        pr = O.Problem("ty", "ETDRK4", nx, 0.02, Lx=Lx, ny=ny, Ly=Ly, params=params)
        prob = TY.Problem("gpu", nx=nx, ny=ny, Lx=Lx, Ly=Ly, nu=1e-12, nnu=4, Ro=1.0, dt=0.02)
        nf = 4
    g = pr.grid
    spec = g.rfft(rng.standard_normal((nf, ny, nx)))
    spec *= np.exp(-g.Krsq / (0.02 * (g.kc ** 2 + (g.ny / 3) ** 2)))
    spec *= 0.3 / np.abs(g.irfft(spec)).max()
    pr.set_solution(spec)
    prob.sol = pr.sol
    assert O.parity_error(prob.calcN(pr.sol), pr.calcN(pr.sol.copy(), g, pr.params), g) < RTOL
    pr.stepforward(3)
    prob.stepforward(3)
    assert O.parity_error(prob.sol, pr.sol, g) < RTOL
    prob.close()


def test_mlqg_driver_setup():
    """TwoLayerSimulation set-up: parameters and the filtered randn IC."""
    from juliaraytracingsw_amd import drivers

    prob, P = drivers.mlqg_problem(128)
    assert P["dt"] == 0.02 * (2 * np.pi / 128) / 0.1
    s = prob.sol
    assert np.all(s[:, :, -1] == 0) and np.all(s[:, 64, :] == 0)  # Nyquist column and row dealiased
    prob.stepforward(3)
    assert np.isfinite(prob.sol).all()
    prob.close()
