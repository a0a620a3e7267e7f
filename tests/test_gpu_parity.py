"""GPU parity tests: libsw (HIP, gfx950) against the CPU oracle and the golden
fixtures, through the C ABI.  Tolerance: SURVEY §8c metric
max|a−b|/max|b| over the dealias-masked state ≤ 1e-10 (fp64)."""
import glob
import json
import os

import numpy as np
import pytest

import sw_cases
import sw_oracle as O
from juliaraytracingsw_amd import _lib

pytestmark = pytest.mark.gpu

RTOL = 1e-10
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _err(a, b, grid):
    return O.parity_error(a, b, grid)


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


# (the config-5 row sample *_rows.npz has its own test: test_gpu_large.py)
@pytest.mark.parametrize("fn", sorted(f for f in glob.glob(os.path.join(GOLDEN, "*.npz")) if not f.endswith("_rows.npz")),
                         ids=lambda f: os.path.basename(f))
def test_golden(fn):
    d = np.load(fn)
    p = json.loads(str(d["params"]))
    prob = sw_cases.libsw_problem(p)
    g = O.TwoDGrid(p["n"], aliased_fraction=p.get("af", 1 / 3))
    N0 = prob.calcN(d["ic"])
    assert _err(N0, d["N0"], g) < RTOL
    prob.sol = d["ic"]
    assert np.array_equal(prob.sol, g.dealias(d["ic"].copy()))
    done = 0
    for key in sorted((k for k in d.files if k.startswith("sol")), key=lambda k: int(k[3:])):
        s = int(key[3:])
        prob.stepforward(s - done)
        done = s
        e = _err(prob.sol, d[key], g)
        assert e < RTOL, (key, e)
    assert prob.clock.step == done
    prob.close()


@pytest.mark.parametrize("name", sw_cases.CASES)
@pytest.mark.parametrize("n", [128, 256])
def test_oracle_parity(name, n):
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    N_gpu = prob.calcN(pr.sol)
    N_cpu = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    assert _err(N_gpu, N_cpu, pr.grid) < RTOL
    for nsteps in (1, 2, 7):
        pr.stepforward(nsteps)
        prob.stepforward(nsteps)
        e = _err(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (nsteps, e)
    prob.close()


@pytest.mark.parametrize("name,n,steps", [("rsw_fab3", 1024, (5,)), ("qg2_ifmab3", 1024, (5,)),
                                          ("rsw_fab3", 2048, (4, 20, 40)), ("qg2_ifmab3", 2048, (4, 12)),
                                          ("qg2_ifmrk4", 1024, (2,))])
def test_oracle_parity_large(name, n, steps):
    """BASELINE sizes: 1024² (config 2) and 2048² (config 3; the metric config
    at the RSWDriver's own parameters, rsw/RSWDriver.jl:134-148, for 40 steps:
    3 Euler start-up steps and 37 AB3 steps), checked at each listed step."""
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    done = 0
    for k in steps:
        pr.stepforward(k - done)
        prob.stepforward(k - done)
        done = k
        e = _err(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (k, e)
    prob.close()


@pytest.mark.parametrize("name,n", [(c, 128 if c.startswith(("ty", "mlqg")) else 256) for c in sw_cases.ALL_CASES] +
                         [("rsw_fab3", 1024), ("qg2_ifmab3", 1024)])
def test_oracle_parity_100_steps(name, n):
    """SURVEY §8c parity metric: ≤ 1e-10 after 100 steps (checked every 25),
    every model × stepper, and at BASELINE config 2's 1024²."""
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    for done in (25, 50, 75, 100):
        pr.stepforward(25)
        prob.stepforward(25)
        e = _err(prob.sol, pr.sol, pr.grid)
        assert e < RTOL, (done, e)
    assert prob.clock.step == 100
    prob.close()


def test_nop_calcN_linear_exactness():
    """NOPcalcN! (rsw/RotatingShallowWater.jl:135-138): IFMAB3 with N ≡ 0 gives
    exp(L t)·sol0; this also checks the device Padé-13 expm against scipy."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW

    n, dt, steps = 64, 0.01, 9
    g = O.TwoDGrid(n)
    prob = RSW.Problem("gpu", nx=n, dt=dt, nu=1e-9, f=3.0, Cg=1.0, stepper="IFMAB3", nop_calcN=True)
    rng = np.random.default_rng(5)
    ic = g.dealias(rng.standard_normal((3, n, n // 2 + 1)) + 1j * rng.standard_normal((3, n, n // 2 + 1)))
    prob.ctx.set_state(ic)
    prob.ctx.step(steps)
    L = O.rsw_L(g, O.RSWParams(1e-9, 4, 3.0, 1.0))
    exact = O.mvmul(O.expm_batched(L * (steps * dt)), ic)
    assert _err(prob.ctx.get_state(), exact, g) < 1e-12
    prob.close()


@pytest.mark.parametrize("mode", ["default", "fuse_all", "fwd_step", "fwd_step_lds"])
@pytest.mark.parametrize("name", sw_cases.CASES + sw_cases.MLQG_CASES)
def test_fused_equals_unfused(name, mode, monkeypatch):
    """The fused column passes (RSW FilteredAB3: col_fwd + update + next col_inv
    in one kernel; the coupled-update pairs: col_fwd + update in one kernel)
    and the reference sequence of separate kernels give bitwise-identical
    states.  fuse_all: force the generic fully fused kernel on every pair;
    fwd_step: SW_FWD_STEP=1 (the forward + update kernel on every pair it is
    built for, not only where it is the default); fwd_step_lds: SW_FWD_STEP=2
    (its variant with N parked in LDS)."""
    if mode == "fuse_all":
        monkeypatch.setenv("SW_FUSE_ALL", "1")
    if mode == "fwd_step":
        monkeypatch.setenv("SW_FWD_STEP", "1")
    if mode == "fwd_step_lds":
        monkeypatch.setenv("SW_FWD_STEP", "2")
    p = sw_cases.case_params(name, 128)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    a = sw_cases.libsw_problem(p)
    monkeypatch.delenv("SW_FUSE_ALL", raising=False)
    monkeypatch.delenv("SW_FWD_STEP", raising=False)
    b = sw_cases.libsw_problem(p, unfused=True)
    a.sol = pr.sol
    b.sol = pr.sol
    for n in (2, 3, 4):  # Euler start-up, then AB3, crossing sw_step calls
        a.stepforward(n)
        b.stepforward(n)
        assert np.array_equal(a.sol, b.sol), n
    a.close()
    b.close()


@pytest.mark.parametrize("knob", ["SW_INV_SPLIT", "SW_ROW_SPLIT", "SW_FWD_SPLIT"])
@pytest.mark.parametrize("name,n", [("qg2_ifmab3", 128), ("mlqg_frk4", 512), ("qg2_fab3", 1024), ("rsw_ifmab3", 512),
                                    ("rsw_ifmrk4", 256), ("qg2_ifmrk4", 256), ("rsw_fab3", 256),
                                    ("ty_etdrk4", 128), ("ty_etdrk4", 512), ("ty_etdrk4", 1024)])
def test_split_passes_bitwise(name, n, knob, monkeypatch):
    """Short lines split over more blocks — the column inverse with one
    output per block (SW_INV_SPLIT, Geom::isplit: 2LQG / MultiLayerQG /
    Thomas–Yamada) and the 2LQG / MultiLayerQG row in two blocks
    (SW_ROW_SPLIT, Geom::rsplit) and the forward column pass with one term
    of N per block, completed by the update (SW_FWD_SPLIT) — give bitwise
    the states and calcN of the one-block passes."""
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    monkeypatch.setenv(knob, "1")
    a = sw_cases.libsw_problem(p)
    monkeypatch.setenv(knob, "0")
    b = sw_cases.libsw_problem(p)
    monkeypatch.delenv(knob, raising=False)
    a.sol = pr.sol
    b.sol = pr.sol
    for k in (2, 3):
        a.stepforward(k)
        b.stepforward(k)
        assert np.array_equal(a.sol, b.sol), k
    assert np.array_equal(a.calcN(pr.sol), b.calcN(pr.sol))
    a.close()
    b.close()


def test_determinism_2048():
    """Same inputs -> bitwise-identical state (no atomics on the data path)."""
    from juliaraytracingsw_amd import drivers

    a, _ = drivers.rsw_problem(2048, "FilteredAB3")
    b, _ = drivers.rsw_problem(2048, "FilteredAB3")
    a.stepforward(6)
    b.stepforward(6)
    assert np.array_equal(a.sol, b.sol)
    a.close()
    b.close()


def test_rsw_eta_floor_at_the_driver_state():
    """the RSW row transforms η + iζ as one complex line,
    so η carries an absolute error ~ eps·max|ζ̂| from the pair split — a floor
    relative to η of ~ eps·|ζ|/|η|, state-dependent.  At the metric
    configuration's own state (RSWDriver IC at 2048², 20 FilteredAB3 steps,
    max|ζ|/max|η| ≈ 25), each field's error against the oracle relative to
    that field's own magnitude (the SURVEY metric divides by the largest
    field, which would hide η's share): measured 3.8e-17 (u), 8.2e-17 (v),
    1.2e-16 (η), asserted within 1e-14."""
    p = sw_cases.case_params("rsw_fab3", 2048)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    pr.stepforward(20)
    prob.stepforward(20)
    got, ref, m = prob.sol, pr.sol, pr.grid.live
    rel = [float(np.max(np.abs(np.where(m, got[f] - ref[f], 0))) / np.max(np.abs(np.where(m, ref[f], 0))))
           for f in range(3)]
    v = O.rsw_updatevars(ref.copy(), pr.grid, pr.params)
    ratio = float(np.max(np.abs(v["zeta"])) / np.max(np.abs(v["eta"])))
    print(f"[eta floor] per-field relative errors u {rel[0]:.2e} v {rel[1]:.2e} eta {rel[2]:.2e}; "
          f"max|zeta| / max|eta| = {ratio:.1f}")
    assert max(rel) < 1e-14, rel
    prob.close()


def test_physical_and_energy():
    """updatevars! (rsw/RotatingShallowWater.jl:101-116) and KE/PE (:323-336)."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW

    p = sw_cases.case_params("rsw_fab3", 128)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    ref = O.rsw_updatevars(pr.sol.copy(), pr.grid, pr.params)
    got = RSW.updatevars(prob)
    for k in ("u", "v", "eta", "zeta"):
        assert np.max(np.abs(got[k] - ref[k])) < 1e-12 * np.max(np.abs(ref[k])), k
    KE, PE = O.rsw_energies(pr.sol, pr.grid, pr.params)
    assert abs(RSW.kinetic_energy(prob) / KE - 1) < 1e-12
    assert abs(RSW.potential_energy(prob) / PE - 1) < 1e-12
    prob.close()


def test_qg2_physical_and_energy():
    from juliaraytracingsw_amd import two_layer_qg as QG2

    p = sw_cases.case_params("qg2_ifmab3", 128)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    got = QG2.updatevars(prob)
    q = pr.grid.irfft(pr.sol)
    psih = O.qg2_streamfunction(pr.sol, pr.grid, pr.params)
    assert np.max(np.abs(got["q"] - q)) < 1e-12 * np.max(np.abs(q))
    psi = pr.grid.irfft(psih)
    assert np.max(np.abs(got["psi"] - psi)) < 1e-12 * np.max(np.abs(psi))
    (KE1, KE2), PE = O.qg2_energies(pr.sol, pr.grid, pr.params)
    assert abs(sum(QG2.kinetic_energy(prob)) / (KE1 + KE2) - 1) < 1e-12
    assert abs(QG2.potential_energy(prob) / PE - 1) < 1e-12
    prob.close()


@pytest.mark.parametrize("case", sw_cases.ALL_CASES)
def test_nan_detection(case):
    """sw_step's blow-up check is folded into every update kernel that stores
    the new state (StepPtrs::nan; no separate pass over the state): one
    non-finite mode in the state is reported as SW_E_NAN by the model/stepper
    pair's own update path (fused column step, forward + update, elementwise)."""
    from juliaraytracingsw_amd import LibSWError

    p = sw_cases.case_params(case, 64)
    prob = sw_cases.libsw_problem(p)
    ic = np.zeros_like(prob.sol)
    ic[0, 1, 1] = np.nan
    prob.sol = ic
    with pytest.raises(LibSWError) as ei:
        prob.stepforward(1)
    assert ei.value.code == -5
    # a finite state steps cleanly afterwards (the flag is re-armed per call)
    prob.sol = np.zeros_like(ic)
    prob.stepforward(3)
    prob.close()


def test_nan_detection_inf_and_record():
    """±Inf is reported as NaN is (the pass's isfinite), and sw_step_record
    reports it after filling the record."""
    from juliaraytracingsw_amd import LibSWError

    p = sw_cases.case_params("qg2_ifmab3", 64)
    prob = sw_cases.libsw_problem(p)
    ic = np.zeros_like(prob.sol)
    ic[1, 2, 3] = np.inf
    prob.sol = ic
    with pytest.raises(LibSWError) as ei:
        prob.stepforward(2)
    assert ei.value.code == -5
    prob.sol = ic
    with pytest.raises(LibSWError) as ei:
        prob.ctx.step_record(2)
    assert ei.value.code == -5 and ei.value.record[0] == prob.ctx.get_clock()[1]
    prob.close()


def test_config1_driver_params_blow_up_like_the_reference():
    """BASELINE config 1 (RSWDriver 128², FilteredAB3, driver νtune) is
    linearly unstable (tests/test_oracle.py); libsw reports it the way the
    driver does (rsw/RSWDriver.jl:213-218): SW_E_NAN, "Solution is NaN"."""
    from juliaraytracingsw_amd import LibSWError, drivers

    prob, _ = drivers.rsw_problem(128, "FilteredAB3")
    with pytest.raises(LibSWError) as ei:
        prob.stepforward(200)
    assert ei.value.code == -5
    prob.close()


@pytest.mark.parametrize("n", [512, 1024])
def test_fab3_driver_params_unstable_grids_report_nan(n):
    """RSW FilteredAB3 at the RSWDriver parameters is linearly unstable below
    2048² (tests/test_oracle.py::test_fab3_driver_params_stability_boundary):
    the run blows up from round-off and libsw reports SW_E_NAN, the driver's
    throw (rsw/RSWDriver.jl:213-218)."""
    from juliaraytracingsw_amd import LibSWError, drivers

    prob, _ = drivers.rsw_problem(n, "FilteredAB3")
    with pytest.raises(LibSWError) as ei:
        for _ in range(8):
            prob.stepforward(500)
    assert ei.value.code == -5
    prob.close()


def test_fab3_driver_params_2048_stays_finite():
    """The metric configuration is on the stable side of that boundary: 4000
    steps (0.41 time units) stay finite with the energy bounded."""
    from juliaraytracingsw_amd import drivers, rotating_shallow_water as RSW

    prob, _ = drivers.rsw_problem(2048, "FilteredAB3")
    e0 = RSW.energy(prob)
    prob.stepforward(4000)
    e1 = RSW.energy(prob)
    assert np.isfinite(e1) and e1 < 1.1 * e0
    prob.close()


@pytest.mark.parametrize("stepper", ["IFMAB3", "IFMRK4"])
def test_qg2_energy_records_match_the_undealiased_state_at_driver_params(stepper):
    """The reference's 2LQG energies read prob.sol after the step
    (swqg/TwoLayerQG.jl:230-252), aliased modes included.  libsw keeps live
    modes only; at the TwoLayerDriver set-up (512², q0 =
    1e-2·randn, swqg/TwoLayerDriver.jl:10-15,29-68) the aliased modes' share
    of the energy is ~1e-13, so the device-recorded energies match the
    oracle's UN-dealiased post-step energies to 1e-10 (the strongly nonlinear
    64² case above shows where that share grows)."""
    from juliaraytracingsw_amd import two_layer_qg as QG2

    p = sw_cases.case_params(f"qg2_{stepper.lower()}", 512)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    freq, nsteps = 10, 30
    KE = QG2.Diagnostic(QG2.kinetic_energy, prob, freq=freq, nsteps=nsteps)
    PE = QG2.Diagnostic(QG2.potential_energy, prob, freq=freq, nsteps=nsteps)
    expected = []
    for s in range(1, nsteps + 1):
        pr.stepforward(1)
        if s % freq == 0:
            expected.append(O.qg2_energies(pr.sol, pr.grid, pr.params))  # full array, not dealiased
    QG2.stepforward(prob, [KE, PE], nsteps)
    for i, ((k1, k2), pe) in enumerate(expected, start=1):
        assert np.allclose(np.atleast_1d(KE.data[i]), (k1, k2), rtol=RTOL, atol=0), (i, KE.data[i], (k1, k2))
        assert abs(PE.data[i] / pe - 1) < RTOL, (i, PE.data[i], pe)
    prob.close()


def test_invalid_config_fails_loudly():
    from juliaraytracingsw_amd import LibSWError, rotating_shallow_water as RSW

    with pytest.raises(LibSWError):
        RSW.Problem("gpu", nx=96)  # not a power of two
    for bad in (dict(nx=16384), dict(nx=16), dict(nx=64, ny=24), dict(nx=64, aliased_fraction=1.0)):
        with pytest.raises(LibSWError):  # outside [32, 8192], not a power of two, no live modes
            RSW.Problem("gpu", **bad)
    prob = RSW.Problem("gpu", nx=64)
    with pytest.raises(LibSWError) as e:
        prob.ctx.step(-1)
    assert e.value.code == _lib.SW_E_INVALID and "nsteps" in str(e.value)
    with pytest.raises(LibSWError):
        prob.ctx.diag(99)
    with pytest.raises(LibSWError):  # TY-only diagnostic on an RSW problem
        prob.ctx.diag(_lib.SW_DIAG_WAVE_KE)
    with pytest.raises(ValueError):  # wrong state shape never reaches the device
        prob.ctx.set_state(np.zeros((3, 64, 32), complex))
    rc = prob.ctx.lib.sw_set_state(prob.ctx._h, None, 0)  # raw ABI: null buffer
    assert rc == _lib.SW_E_INVALID
    prob.stepforward(2)  # the context stays usable after rejected calls
    assert prob.clock.step == 2
    prob.close()


def _rect_problem(name, nx, ny):
    """Oracle + libsw problems of one case on an nx x ny grid with a random
    smooth dealiased IC (the reference's IC builders assume square grids)."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW, two_layer_qg as QG2

    p = sw_cases.case_params(name, 256)
    dt = 2e-4
    if p["model"] == "rsw":
        params = O.RSWParams(1e-30, 4, p["f"], p["Cg"])
    else:
        params = O.QG2Params(p["U"], p["mu"], 1e-30, 4, F=p["F"])
    fk = dict(order=p["order"]) if p["stepper"] == "FilteredAB3" else {}
    pr = O.Problem(p["model"], p["stepper"], nx, dt, params=params, ny=ny, **fk)
    g = pr.grid
    rng = np.random.default_rng(7)
    nf = 3 if p["model"] == "rsw" else 2
    spec = g.rfft(rng.standard_normal((nf, ny, nx)))
    spec *= np.exp(-g.Krsq / (0.05 * (g.kc ** 2 + (g.ny / 3) ** 2)))  # smooth: energy at low K
    spec *= 0.2 / np.abs(g.irfft(spec)).max()
    pr.set_solution(spec)
    if p["model"] == "rsw":
        prob = RSW.Problem("gpu", nx=nx, ny=ny, dt=dt, nu=1e-30, nnu=4, f=p["f"], Cg=p["Cg"],
                           stepper=p["stepper"], **fk)
    else:
        prob = QG2.Problem("gpu", nx=nx, ny=ny, dt=dt, nu=1e-30, nnu=4, U=p["U"], mu=p["mu"], f0=p["f0"],
                           Cg=p["Cg"], drhorho0=p["drhorho0"], stepper=p["stepper"], T=np.float64, **fk)
    prob.sol = pr.sol
    return pr, prob


@pytest.mark.parametrize("nx,ny", [(8192, 32), (32, 8192), (4096, 64), (64, 4096)])
@pytest.mark.parametrize("name", ["rsw_fab3", "qg2_ifmab3", "rsw_ifmrk4", "qg2_ifmrk4"])
def test_rectangular_long_lines(name, nx, ny):
    """Every transform length up to 8192 (the 4096²/8192² configurations) on
    cheap rectangular grids: x lines of 4096/8192 exercise the row pass, y
    lines the column passes, at 1e-10 against the oracle."""
    pr, prob = _rect_problem(name, nx, ny)
    N_gpu = prob.calcN(pr.sol)
    N_cpu = pr.calcN(pr.sol.copy(), pr.grid, pr.params)
    assert _err(N_gpu, N_cpu, pr.grid) < RTOL
    pr.stepforward(4)
    prob.stepforward(4)
    assert _err(prob.sol, pr.sol, pr.grid) < RTOL
    prob.close()


@pytest.mark.parametrize("name", sw_cases.CASES)
def test_energy_diagnostics_recorded(name):
    """FF Diagnostic(kinetic_energy / potential_energy; freq) as the drivers
    keep them (rsw/RSWDriver.jl:193-196, swqg/TwoLayerDriver.jl:86-89),
    recorded on the device while stepping.  Entry 0 is the value at
    construction; then after every freq-th step RSW reads vars.uh/vh/ηh — the
    input of the step's last calcN (rsw/RotatingShallowWater.jl:147-149) — and
    2LQG the post-step sol (swqg/TwoLayerQG.jl:230-252).  libsw stores live
    modes only, so its 2LQG energies are of the dealiased post-step sol; the
    reference's also count the aliased modes the update has just written and
    the next calcN discards (relative 1e-12 (IFMAB3) to 1e-8 (IFMRK4) of the
    energy on this strongly nonlinear 64² case) — compared here against the
    oracle's dealiased post-step state; with sw_config.aliased_state libsw
    carries those modes too and matches the un-dealiased energies
    (tests/test_gpu_aliased.py)."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW, two_layer_qg as QG2

    rsw = name.startswith("rsw")
    M = RSW if rsw else QG2
    p = sw_cases.case_params(name, 64)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    freq, nsteps = 3, 10
    KE = M.Diagnostic(M.kinetic_energy, prob, freq=freq, nsteps=nsteps)
    PE = M.Diagnostic(M.potential_energy, prob, freq=freq, nsteps=nsteps)

    def energies(st):
        if rsw:
            return O.rsw_energies(st, pr.grid, pr.params)
        (k1, k2), pe = O.qg2_energies(st, pr.grid, pr.params)
        return (k1, k2), pe

    last = {}
    calcN = pr.calcN

    def spy(sol, grid, params):  # vars.uh etc. = the dealiased calcN input
        last["x"] = grid.dealias(sol.copy())
        return calcN(sol, grid, params)

    pr.calcN = spy
    expected = [(0, energies(pr.sol))]
    for s in range(1, nsteps + 1):
        pr.stepforward(1)
        if s % freq == 0:
            expected.append((s, energies(last["x"] if rsw else pr.grid.dealias(pr.sol.copy()))))
    M.stepforward(prob, [KE, PE], nsteps)
    assert KE.i == PE.i == len(expected) == 4
    for i, (s, (ke, pe)) in enumerate(expected):
        assert KE.steps[i] == s and PE.steps[i] == s
        assert abs(KE.t[i] - s * p["dt"]) < 1e-12
        assert np.allclose(np.atleast_1d(KE.data[i]), np.atleast_1d(ke), rtol=RTOL, atol=0), (i, KE.data[i], ke)
        assert abs(PE.data[i] / pe - 1) < RTOL, (i, PE.data[i], pe)
    prob.close()


@pytest.mark.parametrize("name", ["rsw_fab3", "qg2_ifmab3"])
def test_cfl_reduction(name):
    """dt · max(max|u|/dx, max|v|/dy) (rsw/RSWDriver.jl:207-208), both layers
    for 2LQG (swqg/TwoLayerDriver.jl:100-101), against the oracle's fields."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW, two_layer_qg as QG2

    p = sw_cases.case_params(name, 128)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    g = pr.grid
    if name.startswith("rsw"):
        ref = O.rsw_updatevars(pr.sol.copy(), g, pr.params)
        u, v = ref["u"], ref["v"]
        got = RSW.cfl(prob)
    else:
        psih = O.qg2_streamfunction(pr.sol, g, pr.params)
        u = g.irfft(-1j * g.l[:, None] * psih)
        v = g.irfft(1j * g.kr[None, :] * psih)
        got = QG2.cfl(prob)
    exp = p["dt"] * max(np.abs(u).max() / g.dx, np.abs(v).max() / g.dy)
    assert abs(got / exp - 1) < 1e-12
    prob.close()
