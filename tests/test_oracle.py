"""CPU tests: pin the oracle restatement to every known answer the reference
holds for this path plus analytic known answers, and check
the committed golden fixtures against it."""
import glob
import json
import os
import sys

import numpy as np
import pytest

import sw_cases
import sw_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# --- known answers from the reference's own notebooks -----------------------
def test_expm_known_answer():
    """rsw/Notebooks/MatrixExponentialTest.ipynb:64 (Lop) and :197-199 (printed exp)."""
    k = l = 1
    Lop = np.array([[0, 1, 1j * k], [-1, 0, 1j * l], [-1j * k, -1j * l, 0]])
    E = O.expm_batched(Lop[None])[0]
    ref = np.array([
        [1.0, 1.7182818284590455, 1.7182818284590453j],
        [-0.6321205588285577, 1.0, 0.6321205588285577j],
        [-0.6321205588285578j, -1.7182818284590453j, 2.0861612696304874],
    ])
    assert np.max(np.abs(E - ref)) <= 4 * np.finfo(float).eps


def test_mvmul_assertion():
    """MatrixExponentialTest.ipynb:498: A[1,1,:,:]*orig_x[1,1,:] ≈ x[1,1,:] after
    the in-place per-mode matvec (utils/IFMAB3.jl:90-100)."""
    rng = np.random.default_rng(0)
    A = rng.random((4, 5, 3, 3)) + 1j * rng.random((4, 5, 3, 3))
    x = rng.random((3, 4, 5)) + 1j * rng.random((3, 4, 5))
    y = O.mvmul(A, x)
    np.testing.assert_allclose(y[:, 0, 0], A[0, 0] @ x[:, 0, 0], rtol=1e-14)


def test_grid_display():
    """MatrixExponentialTest.ipynb:17-20: TwoDGrid(Lx=2π, nx=128) display."""
    g = O.TwoDGrid(128)
    assert g.dx == 0.04908738521234052
    assert g.x[0] == -3.141592653589793
    assert abs(g.x[-1] - 3.0925052683774528) <= 4e-16
    assert g.aliased_fraction == 0.3333333333333333


def test_driver_dt_nu_known_answer():
    """rsw/Notebooks/RSW_Test.ipynb:206 formulas, printed at :228-229."""
    nx, Lx = 512, 2 * np.pi
    dx = Lx / nx
    kmax = nx / 2 - 1
    cfltune, umax = 0.1, 0.3
    nutune = 1 / cfltune
    dt = cfltune / umax * dx
    nu = nutune * 2 * np.pi / nx / (kmax ** (2 * 4)) / dt
    assert nu == 1.6780303489894543e-18
    assert dt == 0.00409061543436171


def test_rsw_driver_params_2048():
    """rsw/RSWDriver.jl:134-148 at the BASELINE sizes."""
    dt, nu = O.rsw_driver_params(2048)
    assert dt == 1.0226538585904273e-4
    assert abs(nu / 1.281965e-20 - 1) < 1e-6
    dt, nu = O.rsw_driver_params(1024)
    assert dt == 2.0453077171808545e-4
    assert abs(nu / 3.307609e-18 - 1) < 1e-6


def test_qg2_driver_params():
    """swqg/TwoLayerDriver.jl:17-63 (U=0.0041667, μ=0.0286347, F=18, dt=2π/N)."""
    P = O.qg2_driver_params(2048)
    assert abs(P["U"] - 0.0041667) < 1e-7
    assert abs(P["mu"] - 0.0286347) < 1e-7
    assert P["F"] == 18.0
    assert abs(P["dt"] - 2 * np.pi / 2048) < 1e-18
    assert abs(P["nu"] / 8.546e-22 - 1) < 1e-3


def test_dealias_ranges():
    """FF getaliasedwavenumbers: N=2048 -> kralias 683:1025, lalias 683:1366."""
    g = O.TwoDGrid(2048)
    assert g.kralias == (682, 1025) and g.lalias == (682, 1366)
    assert g.kc == 682 and len(g.live_rows) == 1364
    assert g.live.sum() == 682 * 1364


def test_qg2_L_float32_quirk():
    """swqg/TwoLayerQG.jl:189-193: PV/drag/Sinv literals are Complex{Float32}."""
    g = O.TwoDGrid(64)
    p = O.QG2Params(0.0041666, 0.02863, 1e-10, 4, F=18.0)
    L = O.qg2_L(g, p)
    k, l = 5, 7
    K2 = k * k + l * l
    pv2 = float(np.float32(((2.0 * k) * p.F) * p.U))
    a = float(np.float32(-K2 - p.F))
    S11 = (a / (K2 + 2 * p.F)) * (1 / K2)
    D = -p.nu * K2 ** 4
    drag = float(np.float32(p.mu * K2))
    assert L[l, k, 1, 1] == complex(drag * S11 + D, pv2 * S11 + k * p.U)
    # the quirk is visible at the 1e-9 level against an all-fp64 evaluation
    S11_64 = (-K2 - p.F) / (K2 + 2 * p.F) / K2
    assert abs(pv2 * S11 - (2 * k * p.F * p.U) * S11_64) > 0


# --- analytic known answers --------------------------------------------------
def _rsw_linear_problem(stepper, n=32, nu=0.0, dt=0.01):
    params = O.RSWParams(nu, 4, 3.0, 1.0)
    pr = O.Problem("rsw", stepper, n, dt, params=params, calcN=O.rsw_NOPcalcN)
    rng = np.random.default_rng(3)
    ic = rng.standard_normal(pr.sol.shape) + 1j * rng.standard_normal(pr.sol.shape)
    pr.set_solution(ic)
    return pr


def test_ifmab3_linear_exactness():
    """NOPcalcN! hook (rsw/RotatingShallowWater.jl:135-138): IFMAB3 gives exp(L t)·sol0."""
    pr = _rsw_linear_problem("IFMAB3", nu=1e-6)
    sol0 = pr.sol.copy()
    pr.stepforward(7)
    exact = O.mvmul(O.expm_batched(pr.L * (7 * pr.clock.dt)), sol0)
    assert O.parity_error(pr.sol, exact, pr.grid) < 1e-12


def test_linear_energy_conservation():
    """diag(1,1,Cg²)·L is anti-Hermitian at ν=0, so KE+PE is conserved by exp(L t)."""
    pr = _rsw_linear_problem("IFMRK4", nu=0.0, dt=0.05)
    e0 = sum(O.rsw_energies(pr.sol, pr.grid, pr.params))
    pr.stepforward(50)
    e1 = sum(O.rsw_energies(pr.sol, pr.grid, pr.params))
    assert abs(e1 / e0 - 1) < 1e-12


def test_fab3_linear_third_order():
    """FilteredAB3 on the linear problem converges at third order to exp(L t)."""
    errs = []
    for dt in (0.02, 0.01):
        params = O.RSWParams(0.0, 4, 3.0, 1.0)
        pr = O.Problem("rsw", "FilteredAB3", 32, dt, params=params, calcN=O.rsw_NOPcalcN,
                       innerK=10.0, outerK=11.0)  # filter ≡ 1
        rng = np.random.default_rng(3)
        ic = np.zeros(pr.sol.shape, complex)
        ic[:, 1:4, 1:4] = rng.standard_normal((3, 3, 3))
        pr.set_solution(ic)
        sol0 = pr.sol.copy()
        nsteps = int(round(0.4 / dt))
        pr.stepforward(nsteps)
        exact = O.mvmul(O.expm_batched(pr.L * (nsteps * dt)), sol0)
        errs.append(np.max(np.abs(pr.sol - exact)))
    # Euler start-up steps are first order per step but only 3 of them: the
    # global error is dominated by O(dt²) from them; check ≥ 2nd order
    assert errs[0] / errs[1] > 3.5


def test_ifmrk4_fourth_order():
    """Lawson IF-RK4 converges at fourth order on the nonlinear RSW
    step (ν = 0, live modes; aliased modes are dead)."""
    p = dict(sw_cases.case_params("rsw_ifmrk4", 32), nu=0.0)
    sols = {}
    for dt in (0.02, 0.01, 0.0025):
        p2 = dict(p, dt=dt)
        pr = sw_cases.oracle_problem(p2)
        pr.set_solution(sw_cases.initial_condition(p2, pr.grid))
        pr.stepforward(int(round(0.16 / dt)))
        sols[dt] = pr.grid.dealias(pr.sol.copy())
    e1 = np.max(np.abs(sols[0.02] - sols[0.0025]))
    e2 = np.max(np.abs(sols[0.01] - sols[0.0025]))
    assert e1 / e2 > 12  # 4th order: (16·(1 - 1/512)/(1 - 1/16)) ≈ 17


def test_kr0_column_hermitian_part_preserved():
    """The physical fields depend only on the Hermitian part of the kr=0 column
    (numpy c2r rule); N is Hermitian there."""
    p = sw_cases.case_params("rsw_fab3", 32)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    N = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    col = N[:, :, 0]
    l = np.arange(32)
    live = pr.grid.live[:, 0] & pr.grid.live[(-l) % 32, 0]
    herm = np.conj(col[:, (-l) % 32])
    assert np.max(np.abs((col - herm)[:, live])) < 1e-12 * np.max(np.abs(col))


# --- Thomas–Yamada + ETDRK4 ------------------------------------------------------
def test_ty_decomposition_known_answers():
    """thomasyamada/Notebooks/TestDecomposition.ipynb cells 2-3 and 7: a
    purely geostrophic IC has no wave part (max|Wh| ~ 1e-13 there), and the
    balanced + wave parts rebuild (u_c, v_c, p_c) (max|Gh + Wh - sol| ~ 5e-13)
    — the TYUtils bases are orthonormal per mode."""
    g = O.TwoDGrid(64, 6 * np.pi)
    rng = np.random.default_rng(5678)
    ic = O.ty_initial_condition(g, rng, at=0.5, ag=0.5, aw=0.0)
    G, W = O.ty_decompose(ic, g)
    assert np.max(np.abs(W)) < 1e-13 * np.max(np.abs(ic))
    assert O.parsevalsum2(W[0], g) + O.parsevalsum2(W[1], g) + O.parsevalsum2(W[2], g) < 1e-24
    rng = np.random.default_rng(1)
    b = rng.standard_normal((4, g.nl, g.nkr)) + 1j * rng.standard_normal((4, g.nl, g.nkr))
    G, W = O.ty_decompose(b, g)
    assert np.max(np.abs(G + W - b[1:4])) < 1e-13 * np.max(np.abs(b))


def test_ty_linear_modes():
    """The TYUtils bases are the eigenvectors of the linear part of calcN!
    (thomasyamada/ThomasYamada.jl:142-145): Φ₀ is balanced (eigenvalue 0)
    and Φ± oscillate at ∓iω, ω = sqrt(1 + K²)."""
    g = O.TwoDGrid(32, 6 * np.pi)
    p = O.TYParams(0.0, 8, 0.0)  # Ro = 0: calcN is the linear part alone
    P0 = O.ty_balanced_basis(g)
    Pp, Pm = O.ty_wave_bases(g)
    om = np.sqrt(1 + g.Krsq)
    m = g.live.copy()
    m[0, 0] = False
    for P, lam in ((P0, 0 * om), (Pp, -1j * om), (Pm, 1j * om)):
        sol = np.concatenate([np.zeros((1,) + P.shape[1:], complex), P])
        N = O.ty_calcN(sol, g, p)
        assert np.max(np.abs(N[1:4] - lam * g.dealias(P.copy()))[:, m]) < 1e-12 * np.max(om[m])
        assert np.max(np.abs(N[0])) == 0


def test_etdrk4_coefficients():
    """getetdcoeffs' contour means equal the Cox–Matthews functions: the
    z → 0 limits (ζ, α, β, Γ)/dt → (1/2, 1/6, 1/6, 1/6) and the closed forms
    at moderate and stiff z (where the contour avoids their cancellation)."""
    dt = 0.1
    z = np.array([0.0, -1e-8, -0.5, -3.0, -40.0, -900.0])
    ze, al, be, ga = O.etdrk4_coeffs(dt, z / dt)
    np.testing.assert_allclose([ze[0] / dt, al[0] / dt, be[0] / dt, ga[0] / dt], [0.5, 1 / 6, 1 / 6, 1 / 6],
                               rtol=1e-14)
    zz = z[2:]
    ez = np.exp(zz)
    np.testing.assert_allclose(ze[2:], dt * (np.exp(zz / 2) - 1) / zz, rtol=1e-12)
    np.testing.assert_allclose(al[2:], dt * (-4 - zz + ez * (4 - 3 * zz + zz ** 2)) / zz ** 3, rtol=1e-12)
    np.testing.assert_allclose(be[2:], dt * (2 + zz + ez * (-2 + zz)) / zz ** 3, rtol=1e-12)
    np.testing.assert_allclose(ga[2:], dt * (-4 - 3 * zz - zz ** 2 + ez * (4 - zz)) / zz ** 3, rtol=1e-12)


def test_etdrk4_linear_exactness():
    """With N ≡ 0, ETDRK4 is exp(L t)·sol0 exactly (E = e^{dt L} per mode)."""
    g = O.TwoDGrid(32, 6 * np.pi)
    p = O.TYParams(1e-4, 2, 1.0)
    pr = O.Problem("ty", "ETDRK4", 32, 0.05, Lx=6 * np.pi, params=p, calcN=lambda s, g, p: np.zeros_like(s))
    rng = np.random.default_rng(3)
    pr.set_solution(rng.standard_normal(pr.sol.shape) + 1j * rng.standard_normal(pr.sol.shape))
    s0 = pr.sol.copy()
    pr.stepforward(6)
    assert O.parity_error(pr.sol, np.exp(6 * 0.05 * O.ty_L(g, p)) * s0, g) < 1e-14


def test_etdrk4_fourth_order():
    """ETDRK4 converges at fourth order on the nonlinear TY step, also with a
    stiff hyperviscosity (ν K⁴ up to ≈ 320, dt·L down to ≈ -26)."""
    for nu in (0.0, 1.0):
        p = dict(sw_cases.case_params("ty_etdrk4", 32), nu=nu, nnu=2)
        sols = {}
        for dt in (0.08, 0.04, 0.01):
            p2 = dict(p, dt=dt)
            pr = sw_cases.oracle_problem(p2)
            pr.set_solution(sw_cases.initial_condition(p2, pr.grid))
            pr.stepforward(int(round(1.6 / dt)))
            sols[dt] = pr.grid.dealias(pr.sol.copy())
        e1 = np.max(np.abs(sols[0.08] - sols[0.01]))
        e2 = np.max(np.abs(sols[0.04] - sols[0.01]))
        assert e1 / e2 > 12, (nu, e1 / e2)


# --- GeophysicalFlows MultiLayerQG + FilteredRK4 ---------------------------------
def _mlqg_params(**over):
    P = O.mlqg_simulation_params(64)
    P.update(over)
    return O.MLQGParams(P["f0"], P["H"], P["b"], P["U"], P["mu"], P["beta"], P["nu"], P["nnu"])


def test_mlqg_phillips_growth_rate():
    """Analytic known answer pinning the restated MultiLayerQG (parity unpinned
    against GeophysicalFlows itself): the two-layer Phillips problem (β = 0,
    μ = 0, ν = 0, equal depths, U₁ = -U₂ = U) grows at
    σ = k U sqrt((2F − K²)/(2F + K²)) for K² < 2F and is neutral otherwise —
    the largest real part of the eigenvalues of the per-mode linear operator
    (L plus the linear part of calcN!)."""
    g = O.TwoDGrid(64, aliased_fraction=0)
    p = _mlqg_params(mu=0.0)
    assert p.F1 == p.F2
    A = O.mlqg_linear_operator(g, p)
    got = np.linalg.eigvals(A).real.max(-1)
    k = g.kr[None, :] * np.ones_like(g.Krsq)
    F, U, K2 = p.F1, p.U[0], g.Krsq
    exp = np.where(K2 < 2 * F, k * U * np.sqrt(np.clip((2 * F - K2) / (2 * F + K2), 0, None)), 0.0)
    m = g.live & (np.abs(K2 - 2 * F) > 1.0)  # away from the double root at K² = 2F
    assert np.max(np.abs(got - exp)[m]) < 1e-12
    assert exp[m].max() > 0.05  # unstable band resolved


def test_mlqg_calcN_linear_part():
    """calcN!'s linear part (mean flow, background PV gradient, bottom drag)
    is the linear operator minus L: calcN(ε q)/ε → (A − L) q as ε → 0."""
    g = O.TwoDGrid(32, aliased_fraction=0)
    p = _mlqg_params(nu=1e-3, nnu=2, beta=0.7)
    rng = np.random.default_rng(2)
    q = g.dealias(rng.standard_normal((2, 32, 17)) + 1j * rng.standard_normal((2, 32, 17)))
    eps = 1e-7
    lin = O.mlqg_calcN(eps * q, g, p) / eps
    exp = O.mvmul(O.mlqg_linear_operator(g, p), q) - O.mlqg_L(g, p) * q
    assert O.parity_error(lin, exp, g) < 1e-6


def test_mlqg_energies_and_inversion():
    """pvfromstreamfunction! ∘ streamfunctionfrompv! is the identity (K ≠ 0),
    and the energies are positive quadratic forms of ψ."""
    g = O.TwoDGrid(32, aliased_fraction=0)
    p = _mlqg_params()
    rng = np.random.default_rng(4)
    q = g.dealias(rng.standard_normal((2, 32, 17)) + 1j * rng.standard_normal((2, 32, 17)))
    q[:, 0, 0] = 0
    back = O.mlqg_pvfromstreamfunction(O.mlqg_streamfunction(q, g, p), g, p)
    assert O.parity_error(back, q, g) < 1e-13
    (k1, k2), pe = O.mlqg_energies(q, g, p)
    assert k1 > 0 and k2 > 0 and pe > 0


def test_filtered_rk4_fourth_order():
    """FF FilteredRK4 converges at fourth order (filter ≡ 1 here, innerK > 1)
    on the nonlinear MultiLayerQG step."""
    p = sw_cases.case_params("mlqg_frk4", 32)
    sols = {}
    for dt in (0.04, 0.02, 0.005):
        params = O.MLQGParams(p["f0"], p["H"], p["b"], p["U"], p["mu"], p["beta"], p["nu"], p["nnu"])
        pr = O.Problem("mlqg", "FilteredRK4", 32, dt, aliased_fraction=0, params=params, innerK=10.0, outerK=11.0)
        pr.set_solution(sw_cases.initial_condition(p, pr.grid))
        pr.stepforward(int(round(2.0 / dt)))
        sols[dt] = pr.grid.dealias(pr.sol.copy())
    e1 = np.max(np.abs(sols[0.04] - sols[0.005]))
    e2 = np.max(np.abs(sols[0.02] - sols[0.005]))
    assert e1 / e2 > 12, e1 / e2


def test_aliased_fraction_zero_grid():
    """FF TwoDGrid(aliased_fraction = 0): dealias! zeroes only the Nyquist
    column and row (the reference's MultiLayerQG set-up,
    simulation/TwoLayerSimulation.jl:38)."""
    g = O.TwoDGrid(64, aliased_fraction=0)
    assert g.kc == 32 and g.kralias == (32, 33) and g.lalias == (32, 33)
    assert g.live.sum() == 32 * 63


def test_config1_fab3_at_driver_nutune_is_unstable():
    """BASELINE config 1 (RSWDriver at 128², FilteredAB3) with the driver's own
    νtune = 20: the explicit hyperviscous rate at kmax is dt·ν·kmax⁸ = νtune·dx
    ≈ 0.98, outside AB3's real-axis stability interval (6/11), so the run
    blows up within 50 steps — as the reference's FilteredAB3 would.  The
    parity cases therefore scale νtune with the grid (tests/sw_cases.py)."""
    n = 128
    dt, nu = O.rsw_driver_params(n)
    assert abs(dt * nu * ((n / 2 - 1) * (2 / 3)) ** 8 - 20 * 2 * np.pi / n) < 1e-12
    pr = O.Problem("rsw", "FilteredAB3", n, dt, params=O.RSWParams(nu, 4, 3.0, 1.0), order=8)
    pr.set_solution(O.shafer_ic(pr.grid, (10, 13), (0, 5), 0.2, 0.1, 3.0, 1.0, np.random.default_rng(1)))
    with np.errstate(all="ignore"):
        pr.stepforward(60)
    assert not np.isfinite(pr.sol).all() or np.abs(pr.sol).max() > 1e6


@pytest.mark.parametrize("n,unstable", [(128, True), (512, True), (1024, True), (2048, False)])
def test_fab3_driver_params_stability_boundary(n, unstable):
    """RSW FilteredAB3 at the RSWDriver parameters (νtune = 20, cfltune =
    0.01, filter order 8; rsw/RSWDriver.jl:134-148): the linear scheme's
    amplification over the live modes.  Below 2048² the explicit
    hyperviscosity of the corner modes (dt·ν·K⁸ up to ≈ 100 at 512²) outruns
    the order-8 filter, so BASELINE configs 1 (128²) and 2 (1024²) blow up
    at the driver's own νtune; from 2048² on the filter wins (|z| = 1 at
    K = 0)."""
    dt, nu = O.rsw_driver_params(n)
    z = O.fab3_linear_growth(O.TwoDGrid(n), O.RSWParams(nu, 4, 3.0, 1.0), dt, order=8)
    if unstable:
        assert z > 1.2
    else:
        assert z <= 1 + 1e-12


# --- golden fixtures -----------------------------------------------------------
GOLDEN_FILES = sorted(f for f in glob.glob(os.path.join(GOLDEN, "*.npz")) if not f.endswith("_rows.npz"))


def test_golden_present():
    assert len(GOLDEN_FILES) == 2 * len(sw_cases.ALL_CASES)


@pytest.mark.parametrize("fn", GOLDEN_FILES, ids=[os.path.basename(f) for f in GOLDEN_FILES])
def test_oracle_reproduces_golden(fn):
    d = np.load(fn)  # allow_pickle=False (data only)
    p = json.loads(str(d["params"]))
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    pr.set_solution(ic)
    assert np.array_equal(pr.sol, d["ic"])
    N0 = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    assert O.parity_error(N0, d["N0"], pr.grid) < 1e-13
    done = 0
    for key in sorted((k for k in d.files if k.startswith("sol")), key=lambda k: int(k[3:])):
        s = int(key[3:])
        pr.stepforward(s - done)
        done = s
        assert O.parity_error(pr.sol, d[key], pr.grid) < 1e-12, key


# --- closed-form 2×2 integrating factors (the 8192² oracle) -------------------
@pytest.mark.parametrize("model", ["qg2", "mlqg"])
@pytest.mark.parametrize("tau", [1e-4, 0.05, 0.5, 5.0])
def test_expm_2x2_matches_scipy(model, tau):
    """sw_oracle.expm_2x2 (cosh/sinh of the traceless part) equals scipy's
    expm mode by mode (≤ 1e-11 of each mode's matrix norm), for the 2LQG
    (with its Float32 literals) and MultiLayerQG operators."""
    g = O.TwoDGrid(64, aliased_fraction=0.0 if model == "mlqg" else 1 / 3)
    if model == "qg2":
        L = O.qg2_L(g, O.QG2Params(0.5, 1e-2, 1e-6, 4))
    else:
        P = O.mlqg_simulation_params(64)
        L = O.mlqg_L(g, O.MLQGParams(P["f0"], P["H"], P["b"], P["U"], P["mu"], P["beta"], 1e-6, 4))
        if L.ndim == 3:  # a diagonal operator: promote
            L = np.stack([np.stack([L[0], 0 * L[0]], -1), np.stack([0 * L[1], L[1]], -1)], -2)
    a, b = O.expm_batched(L * tau), O.expm_2x2(L * tau)
    na = np.linalg.norm(a, axis=(-2, -1))
    # worst modes: the strongly damped ones (norms ~1e-100, where the
    # scaling-and-squaring of expm loses digits) and, at dt·L ~ 200i, the
    # cancellation in δ² = p² + bc (≈ 1e4·eps); the median mode to < 1e-14
    r = np.linalg.norm(a - b, axis=(-2, -1)) / np.maximum(na, 1e-300)  # (underflowed modes: both 0)
    assert np.max(r) < 1e-11
    assert np.median(r) < 1e-14


@pytest.mark.parametrize("case,n,taus", [
    ("qg2_ifmab3", 2048, (1, 2)),    # BASELINE config 3: E = exp(dt L), E2 = exp(2 dt L) (utils/IFMAB3.jl:26-30)
    ("qg2_ifmrk4", 8192, (1, 0.5)),  # config 5: E, H = exp(dt L / 2), on the fixture's 24 rows
])
def test_expm_2x2_pinned_at_the_config_operators(case, n, taus):
    """the closed-form 2×2 exponential (the device's ExpOf<2>
    formula, sw_oracle.expm_2x2) against scipy's expm (Padé scaling and
    squaring, no 2×2 special case) on the actual BASELINE operators — config
    3 on every live mode of 2048², config 5 on every live kr of the config-5
    fixture's 24 l rows of 8192² — ≤ 1e-13 of each mode's norm.  (The
    oracle's stepped parity runs on scipy's expm by default; this pins the
    closed form the device evaluates, at the parameters it runs.)"""
    p = sw_cases.case_params(case, n)
    g = O.TwoDGrid(n)
    L = O.qg2_L(g, O.QG2Params(p["U"], p["mu"], p["nu"], p["nnu"], F=p["F"]))
    if n == 8192:
        fx = np.load(os.path.join(GOLDEN, "qg2_ifmrk4_8192_rows.npz"))
        L = L[fx["rows"]][:, :int(fx["kc"])].reshape(-1, 2, 2)
    else:
        L = L[O.live_mask(g)]
    worst = []
    for tau in taus:
        A = L * (tau * p["dt"])
        a = np.concatenate([O.expm_batched(A[i:i + 250_000]) for i in range(0, len(A), 250_000)])
        b = O.expm_2x2(A)
        na = np.linalg.norm(a, axis=(-2, -1))
        r = np.linalg.norm(a - b, axis=(-2, -1)) / na
        worst.append(float(r.max()))
        assert np.all(na > 0)
        assert r.max() <= 1e-13, (tau, r.max(), A[np.argmax(r)].ravel())
        assert np.median(r) < 1e-15
    print(f"{case} {n}²: {len(L)} modes, worst relative mode error {worst}")


def test_config5_fixture_ic_is_the_seeded_driver_ic():
    """tests/golden/qg2_ifmrk4_8192_rows.npz was generated from the seeded
    driver IC that the GPU test regenerates (numpy PCG64 + pocketfft)."""
    fx = np.load(os.path.join(GOLDEN, "qg2_ifmrk4_8192_rows.npz"))
    p = sw_cases.case_params("qg2_ifmrk4", 8192)
    assert json.loads(str(fx["params"])) == json.loads(json.dumps(p))
    g = O.TwoDGrid(8192)
    ic = g.dealias(sw_cases.initial_condition(p, g))
    sys.path.insert(0, GOLDEN)
    import make_qg2_8192 as M

    rows, kc = fx["rows"], int(fx["kc"])
    assert np.allclose(M.ic_check(ic[:, rows, :kc]), fx["ic_check"], rtol=1e-12, atol=0)
