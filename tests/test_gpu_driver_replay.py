"""GPU replays of the three north-star drivers' ``start!`` through the C ABI,
as the Julia binding (integration/julia/SWLib.jl) issues it — its Python twin
tests/driver_replay.py — checked against the CPU oracle and by the C call
trace:

* RSWDriver.start! (rsw/RSWDriver.jl:134-226): dev = GPU(), T = Float32,
  the default IFMAB3 stepper, KE/PE Diagnostics, frames of output_freq steps;
* TYdriver.start! (thomasyamada/TYdriver.jl:111-231) with ARGS = ["GPU"]:
  start-up problem at startup_dt, then the main problem (LIBSW_CPU=1) at dt
  from the start-up state and clock, wave/geostrophic and barotropic energy
  Diagnostics every 25 steps;
* TwoLayerSimulation.start! (simulation/TwoLayerSimulation.jl:13-143):
  MultiLayerQG FilteredRK4 with aliased_fraction = 0, q̂₀ = filter·rfft(q₀),
  set_q!, energies every step.
"""
import numpy as np
import pytest

import driver_replay as R
import sw_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _sub(seq, sub):
    """index of the first occurrence of the contiguous sub-sequence sub in seq"""
    for i in range(len(seq) - len(sub) + 1):
        if seq[i:i + len(sub)] == sub:
            return i
    return -1


def test_rsw_driver_float32_replay():
    tw = R.Twin()
    nsteps, ofreq, dfreq = 240, 20, 10
    prob, diags, outputs, ic, cfls = R.rsw_driver_start(tw, nx=128, nsteps=nsteps, output_freq=ofreq,
                                                        diags_freq=dfreq, spinup_step=120)
    nframes = round(nsteps / ofreq) + 1
    total = nframes * ofreq
    # -- the C call sequence of SWLib.jl: FF's own stepforward!(prob, diags, n)
    # loop; the per-step seam makes no C call; the energy Diagnostics (steps
    # 10, 20 of each frame) run the counted steps (sw_step_record), the
    # driver's updatevars! downloads prob.sol once per frame
    c = tw.calls
    assert c[:2] == ["sw_config_default", "sw_create"]
    i = _sub(c, ["sw_set_state", "sw_get_state", "sw_set_clock"] + ["sw_get_physical"] * 4)
    assert i >= 0, "set_solution! (load_solution! + updatevars!)"
    assert c[i + 7:i + 10] == ["sw_diag"] * 3, "the Diagnostics' first value: sw_diag of the set state"
    frame = ["sw_step_record"] * (ofreq // dfreq) + ["sw_get_state"] + ["sw_get_physical"] * 4
    first = _sub(c, frame)
    assert first > i, "first stepforward!(prob, diags, n) + updatevars!"
    # the Diagnostics hold ceil((nsteps + 1) / dfreq) values (FF Diagnostic):
    # full after step nsteps, so the frames past it record nothing and
    # updatevars! runs their counted steps at once (one sw_step)
    full = nsteps // ofreq
    late = ["sw_step", "sw_get_state"] + ["sw_get_physical"] * 4
    assert c[first:] == frame * full + late * (nframes - full)
    assert c.count("sw_get_state") == 1 + nframes  # load_solution! + one per frame: none per step
    assert c.count("sw_step") == nframes - full
    assert "sw_set_energy_diagnostics" not in c and "sw_calcN" not in c
    # -- Float32 caller buffers (rsw/RSWDriver.jl:164)
    assert prob.sol.dtype == np.complex64 and prob.vars.u.dtype == np.float32
    assert all(o[1].dtype == np.complex64 for o in outputs[1:])
    assert prob.clock.step == total
    t32 = np.float32(0)
    for _ in range(total):
        t32 = np.float32(t32 + prob.clock.dt)
    assert prob.clock.t == t32 and isinstance(prob.clock.t, np.float32)
    # -- the oracle: IFMAB3 from the same (Float32) initial state, with the
    # Problem's Float32 parameters (Params{T}, Clock{T})
    g = O.TwoDGrid(128)
    p = O.RSWParams(float(prob.params.ν), 4, float(prob.params.f), 1.0)
    pr = O.Problem("rsw", "IFMAB3", 128, float(prob.clock.dt), params=p)
    pr.set_solution(ic.astype(np.complex128))
    ke, pe = [], []
    for s in range(total):
        if (s + 1) % dfreq == 0:  # RSW energies read vars.uh: the input of step s+1's calcN
            k, e = O.rsw_energies(pr.sol, g, p)
            ke.append(k)
            pe.append(e)
        pr.stepforward(1)
    # fp32 rounding of the fp64 device state
    assert O.parity_error(prob.sol.astype(np.complex128), pr.sol, g) < 2e-7
    n = min(diags[0].i - 1, len(ke))
    assert n == len(diags[0].t) - 1  # the Diagnostic is full: nsteps / freq records
    for d, ref in ((diags[0], ke), (diags[1], pe)):
        got = np.array(d.data[1:1 + n], float)
        assert all(isinstance(x, np.float32) for x in d.data[1:1 + n])  # the reference's T
        assert np.allclose(got, ref[:n], rtol=2e-7, atol=0), (got[:3], ref[:3])  # fp32 rounding
        assert list(d.steps[1:1 + n]) == [dfreq * (j + 1) for j in range(n)]
    # the physical fields the driver reads after each frame (updatevars!)
    v = O.rsw_updatevars(pr.sol.copy(), g, p)
    assert np.max(np.abs(prob.vars.η - v["eta"])) < 1e-6 * np.max(np.abs(v["eta"]))
    assert len(cfls) == 1 and 0 < cfls[0] < 1
    prob.timestepper.finalizer()


def test_rsw_driver_blowup_throws_on_its_frame():
    """RSWDriver's real cadence: diags_freq ≫ output_freq (RSWParameters.jl:
    diag_dt = 0.5 against output_dt = 0.025/f, ≈ 60×), so most frames run no
    energy Diagnostic, and the counted steps of a frame are still pending
    when the driver scans vars.η (rsw/RSWDriver.jl:212-213).  With the
    reference's CFL raised to 0.5 (a user's edit of RSWParameters.jl) the
    advection goes unstable on its own; the scan's read of vars.η (an SWField)
    runs the frame's steps, so the throw comes on the frame where the state
    went non-finite, no NaN snapshot is written, and prob.sol is still
    downloaded only once per frame."""
    tw = R.Twin()
    ofreq, dfreq = 20, 1000
    with pytest.raises(R.BlewUp) as ei:
        R.rsw_driver_start(tw, nx=128, nsteps=2000, output_freq=ofreq, diags_freq=dfreq, spinup_step=0,
                           parameters=dict(cfltune=0.5))
    bu = ei.value
    prob = bu.prob
    # the first non-finite step, from the same Float32 state on a second
    # context stepped one step per sw_step
    tw2 = R.Twin()
    p2 = R.rsw_problem(tw2, Lx=2 * np.pi, nx=128, dt=float(prob.clock.dt), f=3.0, Cg=1.0, T=np.float32, nnu=4,
                       nu=float(prob.params.ν), aliased_fraction=1 / 3, order=8, use_filter=False)
    p2.sol[...] = bu.ic
    tw2.load_solution(p2)
    first = None
    for k in range(1, 2001):
        rc = tw2.c("sw_step", p2.timestepper.ctx, 1)
        if rc == R.SW_E_NAN:
            first = k
            break
        assert rc == 0
    assert first is not None and first > 3 * ofreq, first  # mid-run, past the first frames
    # thrown on the frame that holds the first non-finite step
    assert bu.step == -(-first // ofreq) * ofreq, (bu.step, first)
    assert prob.clock.step == bu.step
    # every snapshot written is finite and precedes the blow-up
    snaps = [o for o in bu.outputs[1:]]
    assert len(snaps) == bu.step // ofreq  # frame 0's enforce_reality_condition! output + one per frame before
    assert all(np.all(np.isfinite(o[1])) for o in snaps)
    assert max(o[0] for o in snaps) < first
    # no per-step state traffic: load_solution! + one download per completed frame
    c = tw.calls
    assert c.count("sw_get_state") == 1 + (bu.step // ofreq - 1)
    assert c.count("sw_step") == bu.step // ofreq  # one per frame (updatevars!'s, then the scan's)
    assert c.count("sw_step_record") == 0  # no Diagnostic step before the blow-up (dfreq ≫ first)
    # the throw's frame ran its steps in one sw_step (the scan's vars.η read) and
    # downloaded nothing
    assert c[-1] == "sw_step"
    assert np.all(np.isnan(prob.vars.η))
    prob.timestepper.finalizer()
    p2.timestepper.finalizer()


def test_two_layer_driver_float32_replay():
    """TwoLayerDriver.start! (swqg/TwoLayerDriver.jl:10-117): dev = GPU(),
    T = Float32, IFMAB3, KE/PE Diagnostics, frames of output_freq steps, the
    NaN scan of vars.q (a 3-D SWField of the two layers) after each frame."""
    tw = R.Twin()
    nsteps, ofreq, dfreq = 240, 20, 10
    prob, diags, outputs, ic, cfls = R.two_layer_driver_start(tw, nx=128, nsteps=nsteps, output_freq=ofreq,
                                                              diags_freq=dfreq, spinup_step=120)
    nframes = round(nsteps / ofreq) + 1
    total = nframes * ofreq
    c = tw.calls
    i = _sub(c, ["sw_set_state", "sw_get_state", "sw_set_clock"] + ["sw_get_physical"] * 10)
    assert i >= 0, "set_solution! (load_solution! + updatevars!: 5 fields x 2 layers)"
    frame = ["sw_step_record"] * (ofreq // dfreq) + ["sw_get_state"] + ["sw_get_physical"] * 10
    first = _sub(c, frame)
    assert first > i
    full = nsteps // ofreq
    late = ["sw_step", "sw_get_state"] + ["sw_get_physical"] * 10
    assert c[first:] == frame * full + late * (nframes - full)
    assert c.count("sw_get_state") == 1 + nframes  # none per step
    assert prob.sol.dtype == np.complex64 and prob.vars.q.dtype == np.float32
    assert prob.clock.step == total
    # the oracle from the same Float32 state, the Problem's Float32 parameters
    p = prob.params
    op = O.QG2Params(float(p.U), float(p.μ), float(p.ν), p.nν, F=float(p.F))
    pr = O.Problem("qg2", "IFMAB3", 128, float(prob.clock.dt), params=op)
    pr.set_solution(ic.astype(np.complex128))
    ke, pe = [], []
    for s in range(total):
        pr.stepforward(1)
        if (s + 1) % dfreq == 0:  # 2LQG energies read prob.sol after the step
            (k1, k2), e = O.qg2_energies(pr.grid.dealias(pr.sol.copy()), pr.grid, op)
            ke.append((k1, k2))
            pe.append(e)
    assert O.parity_error(prob.sol.astype(np.complex128), pr.sol, pr.grid) < 2e-7
    n = diags[0].i - 1
    assert n == len(diags[0].t) - 1
    got_ke = np.array([np.array(x, float) for x in diags[0].data[1:1 + n]])
    assert np.allclose(got_ke, np.array(ke[:n]), rtol=2e-7, atol=0)
    assert np.allclose(np.array(diags[1].data[1:1 + n], float), pe[:n], rtol=2e-7, atol=0)
    # the physical PV the driver scans (updatevars! after the last frame)
    q1 = pr.grid.irfft(pr.grid.dealias(pr.sol.copy())[0])
    assert np.max(np.abs(prob.vars.q[0] - q1)) < 1e-6 * np.max(np.abs(q1))
    assert len(cfls) == 1 and 0 < cfls[0] < 1
    prob.timestepper.finalizer()


def test_two_layer_driver_blowup_throws_on_its_frame():
    """TwoLayerDriver's cadence (swqg/TwoLayerParameters.jl: diag_dt = 0.5/f
    against output_dt = 0.025/f, 20×) with the CFL raised to 1: the IFMAB3
    advection goes unstable mid-run; the NaN scan of vars.q
    (swqg/TwoLayerDriver.jl:106) runs the frame's steps and throws on the frame
    where the state went non-finite, with every snapshot finite."""
    tw = R.Twin()
    ofreq, dfreq = 20, 400
    with pytest.raises(R.BlewUp) as ei:
        R.two_layer_driver_start(tw, nx=128, nsteps=3000, output_freq=ofreq, diags_freq=dfreq, spinup_step=0,
                                 parameters=dict(cfltune=1.0))
    bu = ei.value
    prob = bu.prob
    # the first non-finite step, from the same Float32 state and parameters on
    # a second context stepped one sw_step at a time
    tw2 = R.Twin()
    d = O.qg2_driver_params(128, cfltune=1.0)
    p2 = R.qg2_problem(tw2, nx=128, dt=d["dt"], f0=3.0, Cg=1.0, U=d["U"], drhorho0=d["drhorho0"], mu=d["mu"],
                       nu=d["nu"], nnu=4, T=np.float32, stepper="IFMAB3")
    for a, b in ((p2.params.U, prob.params.U), (p2.params.μ, prob.params.μ), (p2.params.ν, prob.params.ν),
                 (p2.params.F, prob.params.F), (p2.clock.dt, prob.clock.dt)):
        assert a == b
    p2.sol[...] = bu.ic
    tw2.load_solution(p2)
    first = None
    for k in range(1, 3001):
        rc = tw2.c("sw_step", p2.timestepper.ctx, 1)
        if rc == R.SW_E_NAN:
            first = k
            break
        assert rc == 0
    assert first is not None and first > 3 * ofreq, first
    assert bu.step == -(-first // ofreq) * ofreq, (bu.step, first)
    snaps = bu.outputs[1:]
    assert len(snaps) == bu.step // ofreq
    assert all(np.all(np.isfinite(o[1])) for o in snaps)
    c = tw.calls
    assert c.count("sw_get_state") == 1 + (bu.step // ofreq - 1)
    assert c[-1] == "sw_step"
    assert np.all(np.isnan(prob.vars.q))
    prob.timestepper.finalizer()
    p2.timestepper.finalizer()


def test_ty_driver_replay():
    tw = R.Twin()
    sp, sdiags, diags, _, outputs, ic, startup_steps = R.ty_driver_start(
        tw, nx=64, startup_dt=3e-2, dt=5e-3, startup_nsteps=200, startup_nsubs=50, nsteps=60, nsubs=20)
    prob = sp  # the main problem
    c = tw.calls
    assert c.count("sw_create") == 2
    assert c.count("sw_destroy") == 1  # startup_prob = nothing
    # set_solution! of the main problem pushes the start-up clock
    i = [k for k, x in enumerate(c) if x == "sw_create"][1]
    assert c[i + 1:i + 4] == ["sw_set_state", "sw_get_state", "sw_set_clock"]
    main_steps = (round(60 / 20) + 1) * 20
    assert prob.clock.step == main_steps
    # -- oracle: start-up at startup_dt, then a fresh problem at dt
    Lx = 6 * np.pi
    nu = 5.0e-34 * (Lx / (2 * np.pi)) ** 16
    tp = O.TYParams(nu, 8, 1.0)
    a = O.Problem("ty", "ETDRK4", 64, 3e-2, Lx=Lx, params=tp)
    a.set_solution(ic)
    rec_s = []
    for s in range(startup_steps):
        a.stepforward(1)
        if (s + 1) % 25 == 0:
            rec_s.append(O.ty_energies(a.grid.dealias(a.sol.copy()), a.grid))
    b = O.Problem("ty", "ETDRK4", 64, 5e-3, Lx=Lx, params=tp)
    b.set_solution(a.sol.copy())
    rec_m = []
    for s in range(main_steps):
        b.stepforward(1)
        if (s + 1) % 25 == 0:
            rec_m.append(O.ty_energies(b.grid.dealias(b.sol.copy()), b.grid))
    assert O.parity_error(prob.sol, b.sol, b.grid) < 1e-10
    # Diagnostics: wave_geostrophic_energy and barotropic_energy records, on
    # the dealiased post-step state (the reference's prob.sol also holds the
    # aliased modes the update has just written: DESIGN §5b)
    for ds, ref in ((sdiags, rec_s), (diags, rec_m)):
        wg, bt = ds
        n = min(wg.i - 1, len(ref))
        assert n >= 2
        for j in range(n):
            bt_ref, _, wg_ref = ref[j]
            assert np.allclose(np.array(wg.data[1 + j]).ravel(), np.array(wg_ref).ravel(), rtol=1e-9, atol=1e-14)
            assert np.isclose(bt.data[1 + j], bt_ref, rtol=1e-9, atol=1e-14)
    # the main problem's clock continues the start-up time (:190)
    t = 0.0
    for _ in range(startup_steps):
        t += 3e-2
    for _ in range(main_steps):
        t += 5e-3
    assert prob.clock.t == pytest.approx(t, rel=1e-14)
    prob.timestepper.finalizer()


def test_two_layer_simulation_replay():
    tw = R.Twin()
    nsteps, nsubs = 100, 25
    prob, diags, outputs, ic = R.mlqg_simulation_start(tw, nx=64, nsteps=nsteps, nsubs=nsubs)
    total = (round(nsteps / nsubs) + 1) * nsubs
    c = tw.calls
    i = _sub(c, ["sw_set_state", "sw_get_state", "sw_set_clock"] + ["sw_get_physical"] * 8)
    assert i >= 0, "set_q! (load_solution! + MultiLayerQG.updatevars!)"
    # energies every step (freq 1): one sw_step_record per step while the
    # Diagnostic has room, then the counted steps run at updatevars! (sw_step)
    assert c.count("sw_step_record") == nsteps and c.count("sw_step") == 1
    # timestepper.filter is FF's makefilter (the driver multiplies q̂₀ by it, :44)
    g = prob.grid
    assert prob.timestepper.filter.shape == (2, g.nl, g.nkr)
    assert np.array_equal(prob.timestepper.filter[0], O.makefilter(g))
    # oracle: GF MultiLayerQG restated, FilteredRK4, aliased_fraction = 0
    pr = O.Problem("mlqg", "FilteredRK4", 64, float(prob.clock.dt), aliased_fraction=0.0, params=prob.params)
    pr.set_solution(ic)
    rec = []
    for _ in range(total):
        pr.stepforward(1)
        rec.append(O.mlqg_energies(pr.grid.dealias(pr.sol.copy()), pr.grid, prob.params))
    assert O.parity_error(prob.sol, pr.sol, pr.grid) < 1e-10
    E = diags[0]
    n = E.i - 1
    assert n == nsteps  # capacity: nsteps + 1 entries, entry 0 at construction
    for j in range(n):
        (k1, k2), (pe,) = E.data[1 + j]
        KE, PE = rec[j]
        assert np.allclose([k1, k2, pe], [KE[0], KE[1], PE], rtol=1e-9, atol=1e-16)
    # the nonlinear term acted: energies moved off their initial values
    assert abs(E.data[n][0][0] - E.data[0][0][0]) > 1e-6 * abs(E.data[0][0][0])
    # updatevars! after the last frame: ψh on the host, q per layer from the device
    psih = O.mlqg_streamfunction(pr.sol.copy(), pr.grid, prob.params)
    assert np.max(np.abs(prob.vars.ψh - psih)) <= 1e-10 * np.max(np.abs(psih))
    q1 = pr.grid.irfft(pr.sol[0].copy())
    assert np.max(np.abs(prob.vars.q[0] - q1)) <= 1e-10 * np.max(np.abs(q1))
    prob.timestepper.finalizer()
