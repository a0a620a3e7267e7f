"""GPU parity of the Thomas–Yamada model stepped by ETDRK4
(thomasyamada/ThomasYamada.jl, FF ETDRK4TimeStepper)
against the CPU oracle, through the C ABI.  Tolerance as every other parity
test: max|a−b|/max|b| over the dealias-masked state ≤ 1e-10 (fp64)."""
import numpy as np
import pytest

import sw_cases
import sw_oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _pair(n, **over):
    p = dict(sw_cases.case_params("ty_etdrk4", n), **over)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    return p, pr, prob


@pytest.mark.parametrize("n", [64, 128, 256])
def test_ty_calcN_and_steps(n):
    p, pr, prob = _pair(n)
    N_gpu = prob.calcN(pr.sol)
    N_cpu = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    assert O.parity_error(N_gpu, N_cpu, pr.grid) < RTOL
    for nsteps in (1, 3, 6):
        pr.stepforward(nsteps)
        prob.stepforward(nsteps)
        e = O.parity_error(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (nsteps, e)
    assert prob.clock.step == 10
    prob.close()


def test_ty_production_config():
    """thomasyamada/cpu-setup/Parameters.jl: 512², Lx = 6π, Ro = 1, dt = 5e-3."""
    p, pr, prob = _pair(512)
    pr.stepforward(3)
    prob.stepforward(3)
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


def test_ty_stiff_hyperviscosity():
    """Coefficient table over a wide range of dt·L (down to ≈ -900 at the
    highest live K): libsw's device getetdcoeffs equals the oracle's."""
    p, pr, prob = _pair(128, nu=1e-16, nnu=8)
    kmax2 = pr.grid.Krsq[pr.grid.live].max()
    assert p["dt"] * 1e-16 * kmax2 ** 8 > 100
    pr.stepforward(5)
    prob.stepforward(5)
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


def test_ty_linear_exactness():
    """N ≡ 0 (the NOPcalcN! hook): ETDRK4 steps give e^{L t}·sol0."""
    from juliaraytracingsw_amd import _lib
    from juliaraytracingsw_amd.problem import Problem

    n, dt = 64, 0.05
    g = O.TwoDGrid(n, 6 * np.pi)
    rng = np.random.default_rng(3)
    ic = g.dealias(rng.standard_normal((4, n, n // 2 + 1)) + 1j * rng.standard_normal((4, n, n // 2 + 1)))
    prob = Problem(_lib.SW_MODEL_TY, nx=n, ny=n, Lx=6 * np.pi, Ly=6 * np.pi, dt=dt, aliased_fraction=1 / 3,
                   stepper="ETDRK4", params=dict(nu=1e-4, nnu=2, Ro=1.0), nop_calcN=True)
    prob.sol = ic
    prob.stepforward(6)
    exact = np.exp(6 * dt * O.ty_L(g, O.TYParams(1e-4, 2, 1.0))) * ic
    assert O.parity_error(prob.sol, exact, g) < 1e-13
    prob.close()


def test_ty_physical_energy_cfl():
    """updatevars! (:67-92), baroclinic/barotropic energies (:333-351), the
    wave/geostrophic split (TYUtils.jl:40-51) and the driver CFL with signed
    maxima (TYdriver.jl:150-151)."""
    from juliaraytracingsw_amd import thomas_yamada as TY

    p, pr, prob = _pair(128)
    pr.stepforward(2)
    prob.stepforward(2)
    sol = pr.grid.dealias(pr.sol.copy())
    ref = O.ty_updatevars(sol.copy(), pr.grid, pr.params)
    got = TY.updatevars(prob)
    for k in ("zt", "uc", "vc", "pc", "ut", "vt", "qc"):
        assert np.max(np.abs(got[k] - ref[k])) < 1e-10 * np.max(np.abs(ref[k])), k
    bt, (bk, bp), ((wk, wp), (gk, gp)) = O.ty_energies(sol, pr.grid)
    assert abs(TY.barotropic_energy(prob) / bt - 1) < 1e-10
    k2, p2 = TY.baroclinic_energy(prob)
    assert abs(k2 / bk - 1) < 1e-10 and abs(p2 / bp - 1) < 1e-10
    (a, b), (c, d) = TY.wave_geostrophic_energy(prob)
    np.testing.assert_allclose([a, b, c, d], [wk, wp, gk, gp], rtol=1e-10)
    g = pr.grid
    exp = p["dt"] * max(ref["uc"].max() / g.dx, ref["vc"].max() / g.dy, ref["ut"].max() / g.dx,
                        ref["vt"].max() / g.dy)
    assert abs(TY.cfl(prob) / exp - 1) < 1e-10
    # the K = 0 mode's special bases (TYUtils.jl:18, 35-36): a mean flow and
    # a mean p_c only
    s0 = np.zeros_like(sol)
    s0[1:4, 0, 0] = [3.0 + 1.0j, -2.0 + 0.5j, 0.7]
    prob.sol = s0
    (a, b), (c, d) = TY.wave_geostrophic_energy(prob)
    _, _, ((wk, wp), (gk, gp)) = O.ty_energies(s0, pr.grid)
    np.testing.assert_allclose([a, b, c, d], [wk, wp, gk, gp], rtol=1e-12, atol=1e-300)
    prob.close()


def test_ty_energy_diagnostics_recorded():
    """FF Diagnostic(barotropic_energy / baroclinic_energy; freq)
    (thomasyamada/TYdriver.jl:146-147) recorded on the device after every
    freq-th step, of the post-step state (live modes)."""
    from juliaraytracingsw_amd import thomas_yamada as TY

    p, pr, prob = _pair(64)
    freq, nsteps = 2, 6
    BT = TY.Diagnostic(TY.barotropic_energy, prob, freq=freq, nsteps=nsteps)
    BC = TY.Diagnostic(TY.baroclinic_energy, prob, freq=freq, nsteps=nsteps)
    WG = TY.Diagnostic(TY.wave_geostrophic_energy, prob, freq=freq, nsteps=nsteps)
    expected = [(0, O.ty_energies(pr.sol, pr.grid))]
    for s in range(1, nsteps + 1):
        pr.stepforward(1)
        if s % freq == 0:
            expected.append((s, O.ty_energies(pr.grid.dealias(pr.sol.copy()), pr.grid)))
    TY.stepforward(prob, [BT, BC, WG], nsteps)
    assert BT.i == BC.i == WG.i == len(expected) == 4
    for i, (s, (bt, bc, wg)) in enumerate(expected):
        assert BT.steps[i] == s
        assert abs(BT.data[i] / bt - 1) < RTOL
        np.testing.assert_allclose(BC.data[i], bc, rtol=RTOL)
        np.testing.assert_allclose(np.ravel(WG.data[i]), np.ravel(wg), rtol=RTOL)
    prob.close()


def test_ty_enforce_reality_condition():
    """enforce_reality_condition! (:103-123) leaves the (dealiased) state as
    it is — its ``mul!(sol[:,:,k], …)`` write into copies — and fills the
    physical vars as updatevars! does."""
    from juliaraytracingsw_amd import thomas_yamada as TY

    p, pr, prob = _pair(64)
    s0 = prob.sol
    v = TY.enforce_reality_condition(prob)
    assert np.array_equal(prob.sol, s0)
    ref = O.ty_updatevars(pr.sol.copy(), pr.grid, pr.params)
    for k in ("zt", "uc", "vc", "pc"):
        assert np.max(np.abs(v[k] - ref[k])) <= 1e-12 * np.max(np.abs(ref[k])), k
    prob.close()


def test_ty_invalid_combinations():
    from juliaraytracingsw_amd import LibSWError, rotating_shallow_water as RSW, thomas_yamada as TY

    with pytest.raises(LibSWError):
        TY.Problem("gpu", nx=64, stepper="IFMAB3")
    with pytest.raises(LibSWError):
        RSW.Problem("gpu", nx=64, stepper="ETDRK4")


def test_ty_snapshot_restart(tmp_path):
    """Output/saveoutput of prob.sol then a restart from the file (state and
    clock): the single-step ETDRK4 continues bitwise."""
    from juliaraytracingsw_amd import output

    p, pr, a = _pair(64)
    fn = str(tmp_path / "ty.jld2")
    out = output.Output(a, fn)
    output.saveproblem(out)
    a.stepforward(4)
    output.saveoutput(out)
    a.stepforward(3)
    b = sw_cases.libsw_problem(p)
    assert output.restart(b, fn) == 4
    b.stepforward(3)
    assert np.array_equal(a.sol, b.sol) and b.clock.step == 7
    a.close()
    b.close()
