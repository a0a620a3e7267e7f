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
  it): the 8-slab decomposition is bitwise equal to one slab for 2 steps, and
  calcN at 8192² matches the oracle to 1e-10 (the oracle's per-mode scipy
  expm of 33.5 M 2×2 operators is too slow for a stepped 8192² oracle run; the
  IFMRK4 update is checked against the oracle on 8192-point lines by
  test_gpu_parity.py::test_rectangular_long_lines).

What the RCCL transport itself adds (the same blocks moved by grouped
ncclSend/ncclRecv between processes) runs on the driver's multi-GPU node."""
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
