"""Grids that are not powers of two (VERDICT r05 missing #4): libsw's generic
engine (csrc/sw_generic.hip) runs GeophysicalFlows' MultiLayerQG with FF's
FilteredRK4 — TwoLayerSimulation, whose simulation/MattParameters.jl:8 sets
nx = 384 = 3·2⁷ — on even grids of 2^a·3^b·5^c points per side, through the
same C ABI.  Parity against the oracle's restatement (oracle/sw_oracle.py
mlqg_calcN, FilteredRK4; unpinned against GF itself, as tests/test_gpu_mlqg.py)
at max|a−b|/max|b| over live modes ≤ 1e-10; slabs in one process bitwise
equal to one slab; diagnostics, checkpoints and the NaN check as on the
power-of-two path."""
import numpy as np
import pytest

import sw_cases
import sw_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _pair(n):
    p = sw_cases.case_params("mlqg_frk4", n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    return p, pr, prob


@pytest.mark.parametrize("n", [96, 120, 384])
def test_generic_calcN_and_steps(n):
    """96 = 2⁵·3, 120 = 2³·3·5, 384 = 2⁷·3 (MattParameters.jl:8)."""
    p, pr, prob = _pair(n)
    N_gpu = prob.calcN(pr.sol)
    N_cpu = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    assert O.parity_error(N_gpu, N_cpu, pr.grid) < RTOL
    for nsteps in (1, 4, 10):
        pr.stepforward(nsteps)
        prob.stepforward(nsteps)
        e = O.parity_error(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (nsteps, e)
    prob.close()


@pytest.mark.parametrize("n", [120, 384])
def test_generic_separate_passes(n, monkeypatch):
    """SW_GEN_FUSED=0: the separate-pass stages (k_prep … k_frk4, the path of
    grids above 1024) against the oracle, and the fused stages (k_gcol_inv,
    k_grow, k_gcol_fwd) against them."""
    p, pr, prob = _pair(n)
    monkeypatch.setenv("SW_GEN_FUSED", "0")
    sep = sw_cases.libsw_problem(p)
    monkeypatch.delenv("SW_GEN_FUSED")
    sep.sol = pr.sol
    pr.stepforward(5)
    prob.stepforward(5)
    sep.stepforward(5)
    assert O.parity_error(sep.sol, pr.sol, pr.grid) < RTOL
    assert O.parity_error(prob.sol, sep.sol, pr.grid) < 1e-12
    prob.close()
    sep.close()


@pytest.mark.parametrize("n", [96, 384])
def test_generic_compile_time_lines_bitwise(n, monkeypatch):
    """The fused kernels compiled for the 3·2^k line lengths (k_gcol_inv /
    k_grow / k_gcol_fwd<N, B, NTH>) against their runtime forms (SW_GEN_CT=0):
    the same butterflies in the same order, bitwise the same state."""
    p, pr, prob = _pair(n)
    monkeypatch.setenv("SW_GEN_CT", "0")
    rt = sw_cases.libsw_problem(p)
    monkeypatch.delenv("SW_GEN_CT")
    rt.sol = pr.sol
    prob.stepforward(6)
    rt.stepforward(6)
    assert np.array_equal(prob.sol, rt.sol)
    prob.close()
    rt.close()


def test_generic_every_term_rectangular():
    """H₁ ≠ H₂, β, drag, hyperviscosity, the 2/3 rule, and nx ≠ ny (96 × 48)."""
    from juliaraytracingsw_amd import multilayer_qg as MLQG

    params = O.MLQGParams(1.0, [0.3, 0.7], [2.0, 1.0], [0.2, -0.1], 0.05, beta=2.0, nu=1e-10, nnu=4)
    dt = 0.002
    pr = O.Problem("mlqg", "FilteredRK4", 96, dt, ny=48, aliased_fraction=1 / 3, params=params)
    rng = np.random.default_rng(7)
    pr.set_solution(pr.grid.rfft(0.5 * rng.standard_normal((2, 48, 96))))
    prob = MLQG.Problem(2, "gpu", nx=96, ny=48, f0=1.0, H=[0.3, 0.7], b=[2.0, 1.0], U=[0.2, -0.1], mu=0.05,
                        beta=2.0, nu=1e-10, nnu=4, dt=dt, aliased_fraction=1 / 3)
    prob.sol = pr.sol
    assert O.parity_error(prob.calcN(pr.sol), pr.calcN(pr.sol.copy(), pr.grid, pr.params), pr.grid) < RTOL
    pr.stepforward(8)
    prob.stepforward(8)
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


def test_generic_matt_parameters():
    """simulation/MattParameters.jl as TwoLayerSimulation builds it: nx = 384,
    Lx = 25·2π·Ld (+1e-5), f = 1e-4, H = [2000, 2000], b₁ = 4f²Ld²/H₀ + 1,
    U = [2U₀, 0], μ = 2U₀κ*/Ld, ν = 0, nν = 8, dt = 1200 s, FilteredRK4,
    aliased_fraction = 0; q₀ = 1e-3 U₀ · randn, filtered (TwoLayerSimulation.jl:50-53)."""
    from juliaraytracingsw_amd import multilayer_qg as MLQG

    Ld, f, H0, U0 = 15e3, 1e-4, 4000.0, 0.01
    Lx = 25 * 2 * np.pi * Ld + 1e-5
    b = [4 * f ** 2 * Ld ** 2 / H0 + 1, 1.0]
    U, mu, dt = [2 * U0, 0.0], 2 * U0 / Ld * 0.1, 60 * 20.0
    params = O.MLQGParams(f, [H0 / 2, H0 / 2], b, U, mu, beta=0.0, nu=0.0, nnu=8)
    pr = O.Problem("mlqg", "FilteredRK4", 384, dt, Lx=Lx, aliased_fraction=0, params=params)
    rng = np.random.default_rng(2024)
    q0 = 1e-3 * U0 * rng.standard_normal((2, 384, 384))
    pr.set_solution(O.makefilter(pr.grid)[None] * pr.grid.rfft(q0))
    prob = MLQG.Problem(2, "gpu", nx=384, Lx=Lx, f0=f, H=[H0 / 2, H0 / 2], b=b, U=U, mu=mu, beta=0.0, nu=0.0,
                        nnu=8, dt=dt, aliased_fraction=0)
    prob.sol = pr.sol
    for nsteps in (1, 5, 20):
        pr.stepforward(nsteps)
        prob.stepforward(nsteps)
        e = O.parity_error(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (nsteps, e)
    # the driver's diagnostics on the device: energies, physical fields, CFL
    (k1, k2), (pe,) = MLQG.energies(prob)
    (K1, K2), PE = O.mlqg_energies(pr.grid.dealias(pr.sol.copy()), pr.grid, params)
    assert abs(k1 / K1 - 1) < 1e-12 and abs(k2 / K2 - 1) < 1e-12 and abs(pe / PE - 1) < 1e-12
    ph = MLQG.updatevars(prob)
    sol = pr.grid.dealias(pr.sol.copy())
    psih = O.mlqg_streamfunction(sol, pr.grid, params)
    for name, spec in (("q", sol), ("psi", psih), ("u", -1j * pr.grid.l[:, None] * psih),
                       ("v", 1j * pr.grid.kr[None, :] * psih)):
        ref = pr.grid.irfft(spec)
        assert np.max(np.abs(ph[name] - ref)) <= 1e-12 * np.max(np.abs(ref)), name
    u = pr.grid.irfft(-1j * pr.grid.l[:, None] * psih)
    v = pr.grid.irfft(1j * pr.grid.kr[None, :] * psih)
    cfl = dt * max(u.max() / pr.grid.dx, v.max() / pr.grid.dy)  # TwoLayerSimulation.jl:124 (signed maxima)
    assert MLQG.cfl(prob) == pytest.approx(cfl, rel=1e-12)
    prob.close()


@pytest.mark.parametrize("P", [2, 4])
def test_generic_slabs_in_one_process_bitwise(P):
    """local_slabs = nranks: the generic engine holds the whole grid, so every
    decomposition returns the undecomposed run's state bitwise."""
    p = sw_cases.case_params("mlqg_frk4", 96)
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    a = sw_cases.libsw_problem(p)
    b = sw_cases.libsw_problem(p, decomposition=dict(nranks=P, local_slabs=P))
    a.sol = ic
    b.sol = ic
    a.stepforward(6)
    b.stepforward(6)
    assert np.array_equal(a.sol, b.sol)
    a.close()
    b.close()


def test_generic_checkpoint_records_and_nan():
    from juliaraytracingsw_amd import LibSWError

    p, pr, prob = _pair(96)
    prob.ctx.set_energy_diagnostics(2, 16)
    prob.stepforward(4)
    blob = prob.ctx.get_checkpoint().copy()
    prob.stepforward(6)
    want = prob.sol
    recs = prob.ctx.energy_diagnostics()
    assert [r[0] for r in recs] == [2, 4, 6, 8, 10]
    q = sw_cases.libsw_problem(p)
    q.ctx.set_checkpoint(blob)
    assert q.ctx.get_clock()[1] == 4
    q.stepforward(6)
    assert np.array_equal(q.sol, want)  # bitwise continuation
    # the records are the energies of prob.sol after each recorded step
    pr.stepforward(10)
    (K1, K2), PE = O.mlqg_energies(pr.grid.dealias(pr.sol.copy()), pr.grid, pr.params)
    assert recs[-1][2] == pytest.approx(K1, rel=1e-10) and recs[-1][4] == pytest.approx(PE, rel=1e-10)
    rec = prob.ctx.step_record(1)
    assert rec[0] == 11
    bad = np.zeros_like(want)
    bad[0, 2, 3] = np.nan
    q.sol = bad
    with pytest.raises(LibSWError) as ei:
        q.stepforward(1)
    assert ei.value.code == -5
    q.close()
    prob.close()


@pytest.mark.parametrize("case", [
    dict(nx=98),                                   # 2·7²: no radix-7 stage
    dict(nx=384, model="qg2"),                     # TwoLayerQG: power-of-two grids only
    dict(nx=384, stepper="FilteredAB3"),           # MultiLayerQG + FilteredAB3: power-of-two grids only
    dict(nx=384, aliased_state=True),
    dict(nx=8192 * 3 // 4),                        # 6144 > 4096
])
def test_generic_refusals(case):
    from juliaraytracingsw_amd import LibSWError, multilayer_qg as MLQG, two_layer_qg as QG2

    nx = case["nx"]
    with pytest.raises(LibSWError) as ei:
        if case.get("model") == "qg2":
            QG2.Problem("gpu", nx=nx, stepper="IFMAB3")
        else:
            MLQG.Problem(2, "gpu", nx=nx, H=[0.5, 0.5], b=[2.0, 1.0], stepper=case.get("stepper", "FilteredRK4"),
                         aliased_state=case.get("aliased_state", False))
    assert ei.value.code == -1
