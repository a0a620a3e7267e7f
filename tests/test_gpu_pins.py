"""Stepped states at BASELINE sizes pinned independently of the oracle
(VERDICT r02), through the production kernels.

A state whose Fourier modes all lie on one line through the origin,
K_m = m·(k0, l0), depends on x only through s = K̂·x.  Then

* RSW (rsw/RotatingShallowWater.jl:140-230): with every velocity amplitude
  perpendicular to K̂ (geostrophic: f v̂ = ik Cg² η̂, f û = −il Cg² η̂),
  u·∇u = (u·K̂) ∂s u = 0 and ∇·(u η) = ∂s((u·K̂) η) = 0, so calcN ≡ 0; and
  the RSW operator (:242-260) acts on a geostrophic mode as its diagonal,
  L·sol = D·sol, D = −ν K^(2nν);
* 2LQG (swqg/TwoLayerQG.jl:152-182): ψ_j and q_j are functions of s, so
  J(ψ_j, q_j) ≡ 0 and calcN ≡ 0.

The 2/3 rule sends every alias of the products onto dead modes, so the
pseudo-spectral calcN vanishes on the live modes up to rounding.  Each
step then has a closed form per mode:

* FilteredAB3 (FF): the scalar recurrence x ← F (x + dt R),
  R = D x, Euler for steps 0-2, then 23/12 R − 16/12 R₋₁ + 5/12 R₋₂;
* IFMAB3 / IFMRK4 (utils/IFMAB3.jl:129-160): x ← E x with the
  per-mode 2×2 E = exp(dt L) (scipy expm of the reference's L, including
  its Complex{Float32} literals, A11), so x_n = Eⁿ x₀.

None of this uses the oracle's stepping code: the expected states come from
the closed forms, evaluated here.  Sizes: the metric grid (RSW 2048²),
config 4's grid (RSW 4096², one slab and four), config 5 (2LQG 8192² IFMRK4,
one slab and eight)."""
import numpy as np
import pytest

import sw_oracle as O
from juliaraytracingsw_amd import rotating_shallow_water as RSW, two_layer_qg as QG2

pytestmark = pytest.mark.gpu
TOL = 1e-12


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _modes(n, k0, l0, ms):
    """(kr index, l row) of m·(k0, l0) in the rfft2 layout"""
    return [(m * k0, (m * l0) % n) for m in ms]


def _filter(n, k, l, order=8, innerK=0.65, outerK=1.0, tol=1e-15):
    """FF makefilter at one mode, Lx = Ly = 2π"""
    dx = 2 * np.pi / n
    K = np.sqrt((k * dx / np.pi) ** 2 + (l * dx / np.pi) ** 2)
    if K < innerK:
        return 1.0
    return float(np.exp(-(-np.log(tol) / (outerK - innerK) ** order) * (K - innerK) ** order))


def _fab3_closed_form(x0, D, F, dt, nsteps):
    """FF FilteredAB3 (filter after the update) on x' = D x, scalar per mode"""
    x, R = x0, []
    for n in range(nsteps):
        R.append(D * x)
        if n < 3:
            x = F * (x + dt * R[-1])
        else:
            x = F * (x + dt * (23 / 12 * R[-1] - 16 / 12 * R[-2] + 5 / 12 * R[-3]))
    return x


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,slabs", [(2048, 1), (2048, 8), (4096, 1), (4096, 4)])
def test_rsw_geostrophic_line_fab3_closed_form(n, slabs):
    """RSW FilteredAB3 at the RSWDriver's parameters (the metric
    configuration and config 4), fused column step (k_col_step_fab3_rsw):
    40 steps of a geostrophic state on the line m·(1, 1), from the largest
    scales to the filtered band next to the 2/3 cut-off."""
    dt, nu = O.rsw_driver_params(n)
    f, Cg2 = 3.0, 1.0
    kc = n // 3  # live kr < kc (2/3 rule)
    ms = [1, 2, 7, 40, n // 8, n // 4, kc - 80, kc - 40, kc - 2]
    rng = np.random.default_rng(7)
    sol = np.zeros((3, n, n // 2 + 1), np.complex128)
    amp = 0.02 * n * n  # physical amplitude ~1e-2 per mode (c2r divides by n²)
    expect = np.zeros_like(sol)
    steps = 40
    for (k, lr), m in zip(_modes(n, 1, 1, ms), ms):
        l = m  # positive l row
        eta = amp * (rng.standard_normal() + 1j * rng.standard_normal())
        u, v = -1j * l * Cg2 * eta / f, 1j * k * Cg2 * eta / f  # geostrophic balance
        D = -nu * float(k * k + l * l) ** 4
        F = _filter(n, k, l)
        for fld, x in enumerate((u, v, eta)):
            sol[fld, lr, k] = x
            expect[fld, lr, k] = _fab3_closed_form(x, D, F, dt, steps)
    dec = dict(nranks=slabs, local_slabs=slabs) if slabs > 1 else None
    prob = RSW.Problem("gpu", nx=n, dt=dt, nu=nu, nnu=4, f=f, Cg=1.0, stepper="FilteredAB3", order=8,
                       decomposition=dec)
    prob.sol = sol
    prob.stepforward(steps)
    got = prob.sol
    prob.close()
    scale = np.max(np.abs(expect))
    err = np.max(np.abs(got - expect)) / scale
    print(f"[pin] RSW FilteredAB3 {n}² P={slabs}: {steps} steps, max|libsw - closed form| / max = {err:.2e}")
    assert err < TOL, err
    # the filtered modes did decay (the closed form is not the identity there)
    k, lr = _modes(n, 1, 1, [kc - 2])[0]
    assert abs(expect[2, lr, k]) < 0.9 * abs(sol[2, lr, k])


def _qg2_E(n, k, l, p, dt):
    """exp(dt L) of the 2LQG operator at one mode (swqg/TwoLayerQG.jl:184-198,
    Complex{Float32} literals included), by scipy's expm"""
    from scipy.linalg import expm

    g = O.TwoDGrid.__new__(O.TwoDGrid)  # a one-mode "grid" for qg2_L
    g.kr, g.l = np.array([float(k)]), np.array([float(l)])
    g.Krsq = g.kr[None, :] ** 2 + g.l[:, None] ** 2
    L = O.qg2_L(g, p)[0, 0]
    return expm(dt * L)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("n,stepper,slabs,steps", [(2048, "IFMAB3", 1, 40), (8192, "IFMRK4", 1, 40),
                                                   (8192, "IFMRK4", 8, 40)])
def test_qg2_line_closed_form(n, stepper, slabs, steps):
    """2LQG at the TwoLayerDriver's parameters: BASELINE config 3 (2048²
    IFMAB3) and config 5 (8192² IFMRK4, one slab and eight): a two-layer PV
    state on the line m·(2, 1) steps as x_n = Eⁿ x₀ per mode."""
    P = O.qg2_driver_params(n)
    params = O.QG2Params(P["U"], P["mu"], P["nu"], 4, F=P["F"])
    kc = n // 3
    ms = [1, 3, 20, n // 16, n // 8, kc // 2 - 3]  # 2m < kc
    rng = np.random.default_rng(11)
    amp = 1e-2 * n * n
    sol = np.zeros((2, n, n // 2 + 1), np.complex128)
    expect = np.zeros_like(sol)
    for (k, lr), m in zip(_modes(n, 2, 1, ms), ms):
        x0 = amp * (rng.standard_normal(2) + 1j * rng.standard_normal(2))
        E = _qg2_E(n, k, m, params, P["dt"])
        sol[:, lr, k] = x0
        expect[:, lr, k] = np.linalg.matrix_power(E, steps) @ x0
    dec = dict(nranks=slabs, local_slabs=slabs) if slabs > 1 else None
    prob = QG2.Problem("gpu", nx=n, dt=P["dt"], f0=P["f0"], Cg=P["Cg"], U=P["U"], drhorho0=P["drhorho0"], nnu=4,
                       nu=P["nu"], mu=P["mu"], stepper=stepper, T=np.float64, decomposition=dec)
    prob.sol = sol
    del sol
    prob.stepforward(steps)
    got = prob.sol
    prob.close()
    err = np.max(np.abs(got - expect)) / np.max(np.abs(expect))
    print(f"[pin] 2LQG {stepper} {n}² P={slabs}: {steps} steps, max|libsw - E^n x0| / max = {err:.2e}")
    assert err < TOL, err
