"""GPU tests of the ABI-6/7 boundary additions (include/sw.h):

* Float32 caller buffers (``sw_config.precision``): the drivers' ``T=Float32``
  (rsw/RSWDriver.jl:164, swqg/TwoLayerDriver.jl:63) through the exact
  ``RSWDriver.initialize_problem`` / ``TwoLayerDriver.initialize_problem``
  parameters.  libsw computes in fp64 and rounds once on the way out, so an
  fp32-buffer problem returns bit for bit the fp32 rounding of the fp64
  problem started from the same (fp32-representable) state.
* stepper history for checkpoint/restart (``sw_get_history`` /
  ``sw_set_history``): a restart from a checkpoint continues bitwise; a
  restart from a snapshot starts AB3 with Euler steps (``sw_reset_history``),
  as the oracle started from that state does.
* MultiLayerQG snapshot output (the r01 KeyError) and restart.
* ``sw_step_alg_bytes`` counts every stage of the RK4-family steppers.
"""
import numpy as np
import pytest

import sw_cases
import sw_oracle as O
from juliaraytracingsw_amd import _lib, drivers, output, rotating_shallow_water as RSW, two_layer_qg as QG2

pytestmark = pytest.mark.gpu
RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


@pytest.mark.parametrize("model,stepper,n", [("rsw", "IFMAB3", 256), ("rsw", "FilteredAB3", 1024),
                                             ("qg2", "IFMAB3", 256)])
def test_float32_driver_buffers(model, stepper, n):
    """RSWDriver / TwoLayerDriver set-up with T=Float32 caller arrays."""
    make = drivers.rsw_problem if model == "rsw" else drivers.qg2_problem
    p32, _ = make(n, stepper, T=np.float32)
    p64, _ = make(n, stepper, T=np.float64)
    s0 = p32.sol
    assert s0.dtype == np.complex64 and s0.shape == p64.ctx.state_shape
    p64.sol = s0.astype(np.complex128)  # the same (fp32-representable) initial state
    assert np.array_equal(p64.sol.astype(np.complex64), s0)
    N32, N64 = p32.calcN(s0), p64.calcN(s0.astype(np.complex128))
    assert N32.dtype == np.complex64 and np.array_equal(N32, N64.astype(np.complex64))
    p32.stepforward(5)
    p64.stepforward(5)
    assert np.array_equal(p32.sol, p64.sol.astype(np.complex64))
    M = RSW if model == "rsw" else QG2
    v32, v64 = M.updatevars(p32), M.updatevars(p64)
    for k in v64:
        assert v32[k].dtype == np.float32 and np.array_equal(v32[k], v64[k].astype(np.float32)), k
    assert M.cfl(p32) == M.cfl(p64)
    with pytest.raises(ValueError):
        p32.ctx.set_state(np.zeros((1, 2, 3), np.complex64))
    p32.close()
    p64.close()


def test_float32_size_checked_by_the_library():
    """A caller buffer of the wrong element size is rejected (SW_E_INVALID)."""
    p32, _ = drivers.rsw_problem(128, "IFMAB3", T=np.float32)
    a = np.zeros(p32.ctx.state_shape, np.complex128)  # fp64 bytes to an fp32 context
    rc = p32.ctx.lib.sw_set_state(p32.ctx._h, a.ctypes.data, a.nbytes)
    assert rc == _lib.SW_E_INVALID
    p32.stepforward(1)  # the context stays usable
    p32.close()


@pytest.mark.parametrize("T", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("name", ["rsw_fab3", "rsw_ifmab3", "qg2_ifmab3", "qg2_ifmrk4", "ty_etdrk4", "mlqg_frk4"])
def test_checkpoint_restart_bitwise(name, T, tmp_path):
    """checkpoint + restart continues bitwise, also for T = Float32 caller
    buffers: the file carries libsw's fp64 blob (state, history, clock), not
    the fp32-rounded arrays."""
    if T == np.float32 and name.startswith(("ty", "mlqg")):
        pytest.skip("T=Float32 is the RSW/2LQG drivers' precision")
    p = sw_cases.case_params(name, 64)
    g = O.TwoDGrid(64, Lx=p.get("Lx", 2 * np.pi), aliased_fraction=p.get("af", 1 / 3))
    a = sw_cases.libsw_problem(p, T=T)
    a.sol = sw_cases.initial_condition(p, g)
    a.stepforward(10)
    fn = str(tmp_path / "ckpt.jld2")
    output.checkpoint(a, fn)
    a.stepforward(7)
    b = sw_cases.libsw_problem(p, T=T)
    assert output.restart(b, fn) == 10
    assert b.ctx.history_slots() == (2 if p["stepper"] in ("FilteredAB3", "IFMAB3") else 0)
    b.stepforward(7)
    assert np.array_equal(a.sol, b.sol)
    assert a.clock.step == b.clock.step == 17 and a.clock.t == b.clock.t
    with np.load(fn) as d:  # the readable copy is in the caller's precision
        assert d["checkpoint/sol"].dtype == (np.complex64 if T == np.float32 else np.complex128)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["rsw_fab3", "qg2_ifmab3"])
def test_snapshot_then_checkpoint_restart_one_context(name, tmp_path):
    """One context restarted from a snapshot (Euler start-up pending) and
    then from a checkpoint: the checkpoint's stepper memory wins — the run
    continues with AB3 exactly as the uninterrupted one (the
    pending Euler steps of the snapshot restart used to survive)."""
    p = sw_cases.case_params(name, 64)
    g = O.TwoDGrid(64, aliased_fraction=p.get("af", 1 / 3))
    a = sw_cases.libsw_problem(p)
    a.sol = sw_cases.initial_condition(p, g)
    a.stepforward(50)
    ck = str(tmp_path / "ckpt.jld2")
    output.checkpoint(a, ck)
    a.stepforward(50)
    sn = str(tmp_path / "snap.jld2")
    out = output.Output(a, sn)
    out.saveproblem()
    out.saveoutput()
    b = sw_cases.libsw_problem(p)
    assert output.restart(b, sn) == 100  # 3 Euler steps pending
    assert output.restart(b, ck) == 50   # ... cancelled by the checkpoint
    c = sw_cases.libsw_problem(p)
    assert output.restart(c, ck) == 50
    b.stepforward(5)
    c.stepforward(5)
    assert np.array_equal(b.sol, c.sol)
    # and the raw history ABI: sw_set_history also cancels a pending reset
    d = sw_cases.libsw_problem(p)
    d.sol = c.sol
    d.clock.set(*c.ctx.get_clock())
    d.ctx.reset_history()
    for k in (1, 2):
        d.ctx.set_history(k, c.ctx.get_history(k))
    c.stepforward(3)
    d.stepforward(3)
    assert np.array_equal(c.sol, d.sol)
    for q in (a, b, c, d):
        q.close()


def test_checkpoint_rejects_another_problem():
    pa = sw_cases.case_params("rsw_fab3", 64)
    pb = sw_cases.case_params("rsw_ifmab3", 64)
    a, b = sw_cases.libsw_problem(pa), sw_cases.libsw_problem(pb)
    blob = a.ctx.get_checkpoint()
    with pytest.raises(_lib.LibSWError):
        b.ctx.set_checkpoint(blob)
    with pytest.raises(_lib.LibSWError):
        a.ctx.set_checkpoint(blob[:-16])
    bad = blob.copy()
    bad[0] ^= 1
    with pytest.raises(_lib.LibSWError):
        a.ctx.set_checkpoint(bad)
    a.ctx.set_checkpoint(blob)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["rsw_fab3", "rsw_ifmab3", "qg2_ifmab3"])
def test_snapshot_restart_starts_with_euler(name, tmp_path):
    """A snapshot holds no history: the AB3 steppers restart with three Euler
    steps (the oracle started from the snapshot state at step 0), not AB3
    with zero history."""
    p = sw_cases.case_params(name, 64)
    a = sw_cases.libsw_problem(p)
    pr = sw_cases.oracle_problem(p)
    a.sol = sw_cases.initial_condition(p, pr.grid)
    a.stepforward(10)
    fn = str(tmp_path / "snap.jld2")
    out = output.Output(a, fn)
    out.saveproblem()
    out.saveoutput()
    b = sw_cases.libsw_problem(p)
    assert output.restart(b, fn) == 10
    b.stepforward(6)
    pr.set_solution(a.sol)
    pr.stepforward(6)
    assert O.parity_error(b.sol, pr.sol, pr.grid) < RTOL
    a.close()
    b.close()


def test_mlqg_snapshot_output(tmp_path):
    p = sw_cases.case_params("mlqg_frk4", 64)
    prob = sw_cases.libsw_problem(p)
    prob.sol = sw_cases.initial_condition(p, O.TwoDGrid(64, aliased_fraction=0.0))
    prob.stepforward(3)
    fn = str(tmp_path / "mlqg.jld2")
    out = output.Output(prob, fn)
    output.saveproblem(out)
    output.saveoutput(out)
    with np.load(fn) as d:
        assert str(d["eqn/model"]) == "MultiLayerQG" and str(d["timestepper/name"]) == "FilteredRK4"
        assert np.array_equal(d["snapshots/sol/3"], prob.sol)
    q = sw_cases.libsw_problem(p)
    assert output.restart(q, fn) == 3
    prob.stepforward(2)
    q.stepforward(2)
    assert np.array_equal(prob.sol, q.sol)  # RK4: no history, restart is exact
    prob.close()
    q.close()


@pytest.mark.parametrize("name", sw_cases.ALL_CASES)
def test_step_alg_bytes_counts_every_stage(name):
    """sw_step_alg_bytes = the algorithmic bytes of every kernel launch of a
    step (the RK4-family steppers run four stages)."""
    p = sw_cases.case_params(name, 64)
    prob = sw_cases.libsw_problem(p)
    prob.sol = sw_cases.initial_condition(p, O.TwoDGrid(64, Lx=p.get("Lx", 2 * np.pi),
                                                        aliased_fraction=p.get("af", 1 / 3)))
    prob.stepforward(4)  # past the Euler start and the fused pipeline's priming
    nst = 6
    stats = prob.ctx.profile(nst)
    per_step = sum(s["alg_bytes"] * s["launches"] for s in stats if s["name"] != "transpose") / nst
    assert prob.ctx.step_alg_bytes() == pytest.approx(per_step, rel=1e-12)
    prob.close()


def test_legacy_checkpoint_file_restarts(tmp_path):
    """A checkpoint file written before the fp64 blob (round-2 layout:
    checkpoint/sol, t, step, history/k) still restarts: state, clock and
    history are set from it, bitwise for fp64 buffers."""
    import zipfile

    p = sw_cases.case_params("rsw_fab3", 64)
    g = O.TwoDGrid(64, aliased_fraction=p.get("af", 1 / 3))
    a = sw_cases.libsw_problem(p)
    a.sol = sw_cases.initial_condition(p, g)
    a.stepforward(9)
    fn = str(tmp_path / "old.jld2")
    t, step = a.ctx.get_clock()
    with zipfile.ZipFile(fn, "w") as zf:
        output._put(zf, "checkpoint/sol", a.ctx.get_state())
        output._put(zf, "checkpoint/t", t)
        output._put(zf, "checkpoint/step", step)
        for k in (1, 2):
            output._put(zf, f"checkpoint/history/{k}", a.ctx.get_history(k))
    a.stepforward(6)
    b = sw_cases.libsw_problem(p)
    assert output.restart(b, fn) == 9
    b.stepforward(6)
    assert np.array_equal(a.sol, b.sol) and b.ctx.get_clock() == a.ctx.get_clock()
    a.close()
    b.close()


def test_checkpoint_aliased_state_must_match():
    """An aliased_state blob carries modes a default context would drop (and
    the reverse lacks them): sw_set_checkpoint refuses the mismatch instead of
    continuing non-bitwise."""
    p = sw_cases.case_params("qg2_ifmab3", 64)
    a = sw_cases.libsw_problem(p, aliased_state=True)
    b = sw_cases.libsw_problem(p)
    a.stepforward(3)
    b.stepforward(3)
    with pytest.raises(_lib.LibSWError, match="aliased_state"):
        b.ctx.set_checkpoint(a.ctx.get_checkpoint())
    with pytest.raises(_lib.LibSWError, match="aliased_state"):
        a.ctx.set_checkpoint(b.ctx.get_checkpoint())
    a.ctx.set_checkpoint(a.ctx.get_checkpoint())
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["rsw_fab3", "rsw_ifmab3", "rsw_ifmrk4", "qg2_ifmab3", "ty_etdrk4", "mlqg_frk4"])
def test_step_record_matches_the_recorded_diagnostics(name):
    """sw_step_record(n) (ABI 9, the lazy Julia seam's energy at a
    Diagnostic step) steps n times and returns exactly the record
    sw_set_energy_diagnostics keeps for that step, on the same state."""
    p = sw_cases.case_params(name, 64)
    g = O.TwoDGrid(64, Lx=p.get("Lx", 2 * np.pi), aliased_fraction=p.get("af", 1 / 3))
    ic = sw_cases.initial_condition(p, g)
    a, b = sw_cases.libsw_problem(p), sw_cases.libsw_problem(p)
    a.sol = ic
    b.sol = ic
    a.ctx.set_energy_diagnostics(5, 10)
    a.ctx.step(15)
    recs = a.ctx.energy_diagnostics()
    got = [b.ctx.step_record(5) for _ in range(3)]
    assert [r[0] for r in got] == [r[0] for r in recs] == [5, 10, 15]
    for r, q in zip(got, recs):
        assert r[1:5] == q[1:5] and r[5] == q[5]  # bitwise: the same reduction
    assert np.array_equal(a.sol, b.sol)
    with pytest.raises(_lib.LibSWError):
        b.ctx.step_record(0)
    a.close()
    b.close()
