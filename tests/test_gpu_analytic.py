"""The HIP calcN (sw_calcN through the C ABI) against closed-form nonlinear
terms of few-mode states (tests/analytic.py) — pinned independently of the
oracle: RSW (rsw/RotatingShallowWater.jl:140-230) and 2LQG
(swqg/TwoLayerQG.jl:152-182) triads, the 2LQG same-shell state whose
Jacobian vanishes identically, Thomas–Yamada (thomasyamada/ThomasYamada.jl
:129-262) and MultiLayerQG few-mode states, on one slab and on in-process
slabs."""
import numpy as np
import pytest

import analytic as A
import sw_cases

pytestmark = pytest.mark.gpu
TOL = 1e-12


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.mark.parametrize("P", [1, 2])
@pytest.mark.parametrize("n", [64, 256])
def test_rsw_calcN_triad(n, P):
    p = sw_cases.case_params("rsw_ifmab3", n)
    dec = dict(nranks=P, local_slabs=P) if P > 1 else None
    prob = sw_cases.libsw_problem(p, decomposition=dec)
    got = prob.calcN(A.state(A.rsw_triad(), n))
    assert _rel(got, A.state(A.rsw_N(*A.rsw_triad()), n)) < TOL
    prob.close()


@pytest.mark.parametrize("n", [64, 256])
def test_qg2_calcN_triad(n):
    p = sw_cases.case_params("qg2_ifmab3", n)
    prob = sw_cases.libsw_problem(p)
    q1, q2 = A.qg2_triad()
    got = prob.calcN(A.state((q1, q2), n))
    assert _rel(got, A.state(A.qg2_N(q1, q2, p["F"]), n)) < TOL
    prob.close()


def test_qg2_calcN_shell_vanishes():
    p = sw_cases.case_params("qg2_ifmab3", 128)
    prob = sw_cases.libsw_problem(p)
    q1, q2 = A.qg2_shell()
    got = prob.calcN(A.state((q1, q2), 128))
    ref = np.abs(A.state((A.mul(A.dx(q1, 0), A.dx(q1, 1)),), 128)).max()
    assert np.abs(got).max() / ref < TOL
    prob.close()


@pytest.mark.parametrize("P", [1, 2])
@pytest.mark.parametrize("n", [64, 128])
def test_ty_calcN_quad(n, P):
    from juliaraytracingsw_amd import thomas_yamada as TY

    dec = dict(nranks=P, local_slabs=P) if P > 1 else None
    prob = TY.Problem("gpu", nx=n, Lx=2 * np.pi, dt=1e-3, nu=1e-30, nnu=8, Ro=0.7, decomposition=dec)
    flds = A.ty_quad()
    got = prob.calcN(A.state(flds, n))
    want = A.state(A.ty_N(*flds, 0.7), n)
    for f in range(4):
        assert _rel(got[f], want[f]) < TOL, f
    prob.close()


@pytest.mark.parametrize("n", [64, 128])
def test_mlqg_calcN_pair(n):
    from juliaraytracingsw_amd import multilayer_qg as MLQG
    import sw_oracle as O

    kw = dict(f0=1.0, H=[0.3, 0.7], b=[1.0, 0.8], U=[0.15, -0.05], mu=0.02, beta=0.4)
    prob = MLQG.Problem(2, "gpu", nx=n, nu=0.0, nnu=8, dt=1e-3, stepper="FilteredRK4", aliased_fraction=0.0, **kw)
    p = O.MLQGParams(kw["f0"], kw["H"], kw["b"], kw["U"], kw["mu"], beta=kw["beta"])
    q1, q2 = A.mlqg_pair()
    got = prob.calcN(A.state((q1, q2), n))
    want = A.state(A.mlqg_N(q1, q2, p.F1, p.F2, p.U, p.Qy, p.mu), n)
    for f in range(2):
        assert _rel(got[f], want[f]) < TOL, f
    prob.close()
