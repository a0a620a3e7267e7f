"""The HIP calcN (sw_calcN through the C ABI) against closed-form nonlinear
terms of few-mode states (tests/analytic.py) — pinned independently of the
oracle: RSW (rsw/RotatingShallowWater.jl:140-230) and 2LQG
(swqg/TwoLayerQG.jl:152-182) triads, and the 2LQG same-shell state whose
Jacobian vanishes identically, on one slab and on in-process slabs."""
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
