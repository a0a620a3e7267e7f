"""The oracle's calcN against closed-form nonlinear terms (tests/analytic.py):
an independent pin of the restatement beyond the set-up known answers the
reference holds.  CPU only; the HIP calcN is checked against the
same closed forms in tests/test_gpu_analytic.py."""
import numpy as np
import pytest

import analytic as A
import sw_oracle as O

N = 64
TOL = 1e-12


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


def test_trig_algebra_matches_sampled_fields():
    """The closed-form spectra equal the rfft2 of the sampled trig fields."""
    x = 2 * np.pi * np.arange(N) / N
    X, Y = np.meshgrid(x, x)
    u, v, eta = A.rsw_triad()

    def sample(f):
        return sum(a * (np.cos if k == "c" else np.sin)(m[0] * X + m[1] * Y) for a, k, m in f)

    for f in (u, v, eta, A.mul(u, v), A.dx(A.mul(v, eta), 1)):
        assert _rel(A.spectrum(f, N, N), np.fft.rfft2(sample(f))) < 1e-13


def test_rsw_calcN_triad():
    g = O.TwoDGrid(N)
    sol = A.state(A.rsw_triad(), N)
    want = A.state(A.rsw_N(*A.rsw_triad()), N)
    got = O.rsw_calcN(sol.copy(), g, O.RSWParams(1e-16, 4, 3.0, 1.0))
    assert _rel(got, want) < TOL


@pytest.mark.parametrize("F", [18.0, 0.5])
def test_qg2_calcN_triad(F):
    g = O.TwoDGrid(N)
    q1, q2 = A.qg2_triad()
    got = O.qg2_calcN(A.state((q1, q2), N), g, O.QG2Params(0.01, 0.03, 1e-20, 4, F=F))
    assert _rel(got, A.state(A.qg2_N(q1, q2, F), N)) < TOL


def test_qg2_calcN_shell_vanishes():
    """J(ψ, q) = 0 for q2 = c·q1 on one |K| shell (each product is O(1))."""
    g = O.TwoDGrid(N)
    q1, q2 = A.qg2_shell()
    sol = A.state((q1, q2), N)
    got = O.qg2_calcN(sol, g, O.QG2Params(0.01, 0.03, 1e-20, 4, F=18.0))
    ref = np.abs(A.state((A.mul(A.dx(q1, 0), A.dx(q1, 1)),), N)).max()  # an O(1) product's scale
    assert np.abs(got).max() / ref < TOL


def test_ty_calcN_quad():
    """Thomas–Yamada: every term of calcN! (advection of ζ_T, the baroclinic
    and pressure products, the linear terms) on a four-field few-mode state."""
    g = O.TwoDGrid(N)
    flds = A.ty_quad()
    got = O.ty_calcN(A.state(flds, N), g, O.TYParams(1e-30, 8, 0.7))
    want = A.state(A.ty_N(*flds, 0.7), N)
    for f in range(4):
        assert _rel(got[f], want[f]) < TOL, f


def test_mlqg_calcN_pair():
    """MultiLayerQG (aliased_fraction = 0): advection by U + u, the β/shear
    background gradient and the bottom drag, unequal layer depths."""
    g = O.TwoDGrid(N, aliased_fraction=0.0)
    p = O.MLQGParams(1.0, [0.3, 0.7], [1.0, 0.8], [0.15, -0.05], 0.02, beta=0.4)
    q1, q2 = A.mlqg_pair()
    got = O.mlqg_calcN(A.state((q1, q2), N), g, p)
    want = A.state(A.mlqg_N(q1, q2, p.F1, p.F2, p.U, p.Qy, p.mu), N)
    for f in range(2):
        assert _rel(got[f], want[f]) < TOL, f
