"""BASELINE configurations 4 and 5 at full size on one GPU (-m gpu):

* config 4 — RSW 4096² FilteredAB3 at the RSWDriver parameters
  (rsw/RSWDriver.jl:134-176): the 4-slab decomposition (every slab in this
  process, transposes as device copies with exactly the block pattern of the
  RCCL all-to-all) is bitwise equal to one slab for 5 steps, pipelined and
  sequential, for 20 steps, and the state matches the CPU oracle to 1e-10
  after 4 and after 20 steps (tests/test_gpu_pins.py adds 40-step
  closed-form pins at this size, one slab and four);
* config 5 — TwoLayerQG 8192² IFMRK4 at the TwoLayerDriver parameters
  (swqg/TwoLayerDriver.jl:29-68, stepper utils/IFMRK4.jl as the build defines
  it): the 8-slab decomposition is bitwise equal to one slab for 2 steps,
  calcN at 8192² matches the oracle to 1e-10, and the state after 2 steps
  matches tests/golden/qg2_ifmrk4_8192_rows.npz (24 l rows of an oracle run
  whose integrating factors are scipy's expm on every live mode, forked over
  8 processes: round 5, independent of the device's closed form; the IFMRK4
  update is also checked on 8192-point lines by
  test_gpu_parity.py::test_rectangular_long_lines).

What the RCCL transport itself adds (the same blocks moved by grouped
ncclSend/ncclRecv between processes) runs on the driver's multi-GPU node."""
import json
import os
import sys

import numpy as np
import pytest

import sw_cases
import sw_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


@pytest.fixture(autouse=True)
def _fft_workers():
    import os

    O.set_fft_workers(min(16, len(os.sched_getaffinity(0))))
    yield
    O.set_fft_workers(None)


@pytest.mark.timeout(900)
def test_config4_rsw4096_fab3(monkeypatch):
    """20 steps (3 Euler + 17 AB3) against the oracle, one slab and four
    (pipelined and sequential schedules bitwise equal to one slab)."""
    p = sw_cases.case_params("rsw_fab3", 4096)
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    a = sw_cases.libsw_problem(p)
    a.sol = ic
    a.stepforward(4)
    s4 = a.sol
    a.stepforward(16)
    s20 = a.sol
    a.close()
    for overlap in ("1", "0"):
        monkeypatch.setenv("SW_OVERLAP", overlap)
        b = sw_cases.libsw_problem(p, decomposition=dict(nranks=4, local_slabs=4))
        monkeypatch.delenv("SW_OVERLAP", raising=False)
        b.sol = ic
        b.stepforward(4)
        assert np.array_equal(b.sol, s4), overlap
        b.stepforward(16)
        assert np.array_equal(b.sol, s20), overlap
        b.close()
    pr.set_solution(ic)
    pr.stepforward(4)
    e = O.parity_error(s4, pr.sol, pr.grid)
    assert e < RTOL, e
    pr.stepforward(16)
    e = O.parity_error(s20, pr.sol, pr.grid)
    assert e < RTOL, e


@pytest.mark.timeout(600)
def test_config5_qg2_8192_ifmrk4():
    p = sw_cases.case_params("qg2_ifmrk4", 8192)
    g = O.TwoDGrid(8192)
    ic = sw_cases.initial_condition(p, g)
    a = sw_cases.libsw_problem(p)
    b = sw_cases.libsw_problem(p, decomposition=dict(nranks=8, local_slabs=8))
    a.sol = ic
    b.sol = ic
    Na, Nb = a.calcN(ic), b.calcN(ic)
    assert np.array_equal(Na, Nb)
    params = O.QG2Params(p["U"], p["mu"], p["nu"], p["nnu"], F=p["F"])
    Nc = O.qg2_calcN(g.dealias(ic.copy()), g, params)
    e = O.parity_error(Na, Nc, g)
    assert e < RTOL, e
    del Nb, Nc
    for n in (1, 1):
        a.stepforward(n)
        b.stepforward(n)
        assert np.array_equal(a.sol, b.sol)
    assert np.isfinite(a.sol).all()
    a.close()
    b.close()


@pytest.mark.timeout(600)
def test_config5_stepped_state_matches_the_oracle():
    """BASELINE config 5 at full size, nonlinear: TwoLayerQG
    8192² IFMRK4 from the seeded driver IC, two full steps, libsw on one slab
    and on eight (in-process) against the oracle's two steps
    (tests/golden/make_qg2_8192.py; its fixture keeps 24 l rows of the
    state, every live kr, both layers).  Within 1e-10 of the sample's
    magnitude, where the nonlinear part of the sample is far larger; the
    eight-slab state bitwise the one-slab state; the full per-layer sums of
    |q̂|² within 1e-12."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_qg2_8192 as M

    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "qg2_ifmrk4_8192_rows.npz"))
    rows, kc, steps = fx["rows"], int(fx["kc"]), int(fx["steps"])
    p = sw_cases.case_params("qg2_ifmrk4", 8192)
    assert json.loads(str(fx["params"])) == json.loads(json.dumps(p))
    g = O.TwoDGrid(8192)
    ic = g.dealias(sw_cases.initial_condition(p, g))
    # the box's seeded IC is the generator's (numpy's PCG64 + pocketfft)
    assert np.allclose(M.ic_check(ic[:, rows, :kc]), fx["ic_check"], rtol=1e-12, atol=0)
    ref = fx["sol_rows"]
    scale = np.max(np.abs(ref))
    nonlinear = float(fx["nonlinear_part"])
    assert nonlinear > 1e-6  # the nonlinear term moved the sample (2.0e-5 of it), 1e5 x the tolerance
    got = {}
    for P in (1, 8):
        kw = {} if P == 1 else dict(decomposition=dict(nranks=8, local_slabs=8))
        a = sw_cases.libsw_problem(p, **kw)
        a.sol = ic
        a.stepforward(steps)
        got[P] = a.sol
        a.close()
    assert np.array_equal(got[1], got[8])
    e = np.max(np.abs(got[1][:, rows, :kc] - ref)) / scale
    print(f"[config5] 8192² IFMRK4, {steps} steps: sample error {e:.2e} of its max; nonlinear part {nonlinear:.2e}")
    assert e < 1e-10, e
    ss = np.array([np.sum(np.abs(got[1][f]) ** 2) for f in range(2)])
    assert np.allclose(ss, fx["sumsq"], rtol=1e-12, atol=0), (ss, fx["sumsq"])
