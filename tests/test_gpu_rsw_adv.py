"""RSW with aliased_fraction = 0 (missing #5): the reference's
Problem accepts any aliased_fraction (rsw/RotatingShallowWater.jl:82), while
libsw's vorticity-form calcN is exact only on the live modes of the 2/3 rule.
Without a dealiased band libsw runs the reference's calcN as written — the
advective form (:140-230: u ux, v uy, u vx, v vy, (uη)_x, (vη)_y), kernel
family sw::MODEL_RSWA — compared here with the oracle on every mode of the
full array (FF with aliased_fraction = 0 zeroes only the Nyquist column and
row), and with the vorticity form where both apply (SW_RSW_ADV=1 at the
default 1/3).
"""
import numpy as np
import pytest

import sw_cases
import sw_oracle as O
from juliaraytracingsw_amd import rotating_shallow_water as RSW

pytestmark = pytest.mark.gpu
RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _pair(stepper, n=64, af=0.0, **kw):
    p = sw_cases.case_params(f"rsw_{ {'FilteredAB3': 'fab3', 'IFMAB3': 'ifmab3', 'IFMRK4': 'ifmrk4'}[stepper]}", n)
    params = O.RSWParams(p["nu"], p["nnu"], p["f"], p["Cg"])
    fk = dict(order=p["order"]) if stepper == "FilteredAB3" else {}
    pr = O.Problem("rsw", stepper, n, p["dt"], aliased_fraction=af, params=params, **fk)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = RSW.Problem("gpu", nx=n, dt=p["dt"], nu=p["nu"], nnu=p["nnu"], f=p["f"], Cg=p["Cg"], stepper=stepper,
                       aliased_fraction=af, **fk, **kw)
    prob.sol = pr.sol
    return pr, prob


def _err(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


@pytest.mark.parametrize("stepper", ["FilteredAB3", "IFMAB3", "IFMRK4"])
def test_af0_full_array_parity(stepper):
    """20 steps at aliased_fraction = 0 against the oracle, every mode (the
    Nyquist column and row the update writes are dt·N-small here)."""
    pr, prob = _pair(stepper)
    for s in range(4):
        pr.stepforward(5)
        prob.stepforward(5)
        assert _err(prob.sol, pr.sol) < RTOL, (s, _err(prob.sol, pr.sol))
    # no 2/3 band: the modes between kc(1/3) and Nyquist are live and nonzero
    g13 = O.TwoDGrid(64)
    band = g13.dealias(np.ones((1, g13.nl, g13.nkr), np.complex128))[0] == 0
    band[:, -1] = False
    band[g13.nl // 2, :] = False
    assert np.max(np.abs(pr.sol[:, band])) > 1e-8 * np.max(np.abs(pr.sol))
    prob.close()


def test_af0_calcN_every_live_mode():
    """calcN at aliased_fraction = 0 on every mode but the Nyquist column and
    row — there FF's dealias! still zeroes the state, so they are the aliased
    modes of this grid (the reference's N holds values there that the next
    calcN! discards; full-array tracking: 2LQG only, tests/test_gpu_aliased.py)."""
    pr, prob = _pair("IFMAB3", n=128)
    pr.stepforward(3)
    x = pr.sol.copy()
    ref = pr.calcN(x.copy(), pr.grid, pr.params)
    got = prob.calcN(x)
    assert np.max(np.abs(ref[:, :, -1])) > 0  # the Nyquist column
    assert _err(got, pr.grid.dealias(ref.copy())) < RTOL
    prob.close()


def test_advective_equals_vorticity_form_on_live_modes(monkeypatch):
    """At aliased_fraction = 1/3 both forms are exact on the live modes: the
    advective kernels (SW_RSW_ADV=1) and the default vorticity form give the
    same calcN and the same states there (to rounding), both the oracle's."""
    pr, vort = _pair("IFMAB3", n=128, af=1 / 3)
    monkeypatch.setenv("SW_RSW_ADV", "1")
    adv = RSW.Problem("gpu", nx=128, dt=pr.clock.dt, nu=pr.params.nu, nnu=pr.params.nnu, f=pr.params.f,
                      Cg=np.sqrt(pr.params.Cg2), stepper="IFMAB3")
    monkeypatch.delenv("SW_RSW_ADV")
    adv.sol = vort.sol
    x = vort.sol
    na, nv = adv.calcN(x), vort.calcN(x)
    ref = pr.grid.dealias(pr.calcN(x.copy(), pr.grid, pr.params))
    assert _err(na, ref) < RTOL and _err(nv, ref) < RTOL
    assert _err(na, nv) < 1e-12
    for _ in range(3):
        pr.stepforward(4)
        adv.stepforward(4)
        vort.stepforward(4)
        assert _err(adv.sol, pr.grid.dealias(pr.sol.copy())) < RTOL
        assert _err(adv.sol, vort.sol) < 1e-12
    adv.close()
    vort.close()


@pytest.mark.parametrize("stepper", ["FilteredAB3", "IFMRK4"])
def test_af0_slabs_bitwise(stepper, monkeypatch):
    """Two and four in-process slabs (pipelined with row chunks, and
    sequential) bitwise equal to one slab at aliased_fraction = 0."""
    pr, one = _pair(stepper, n=256)
    one.stepforward(6)
    want = one.sol
    one.close()
    for P, ov in ((2, "1"), (4, "0")):
        monkeypatch.setenv("SW_OVERLAP", ov)
        monkeypatch.setenv("SW_ROW_CHUNKS", "2")
        _, sl = _pair(stepper, n=256, decomposition=dict(nranks=P, local_slabs=P))
        sl.stepforward(6)
        assert np.array_equal(sl.sol, want), (P, ov)
        sl.close()
