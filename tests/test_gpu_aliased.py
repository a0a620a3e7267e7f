"""Aliased-state tracking (sw_config.aliased_state): the
modes the 2/3 rule removes, carried as the reference carries them.

The reference's 2LQG calcN! dealiases its input in place but returns N on
every mode (swqg/TwoLayerQG.jl:152-182: rfft of the products, no dealias of
N), and the IF/AB3 update writes E·dt·(…N…) into prob.sol there
(utils/IFMAB3.jl:142-160), so between steps prob.sol holds aliased modes,
which its energies (:230-252) count and the next calcN!/updatevars!
discards.  Thomas–Yamada's calcN! and ETDRK4 update do the same
(thomasyamada/ThomasYamada.jl:130; its energies read prob.sol).  With
aliased_state = 1 libsw carries them too (RSW, 2LQG, TY and MultiLayerQG, any
nx up to 8192, one slab or several in one process); the oracle keeps the
full arrays, so every comparison here is
over ALL modes of the full (nkr, nl) array, at the strongly nonlinear 64²
cases of tests/sw_cases.py.  RSW (whose update writes those modes into
prob.sol too) carries them with its calcN in the reference's advective form
(the vorticity form is exact on the live modes only); its energies read the
dealiased vars.uh, so its records are unchanged.
"""
import numpy as np
import pytest

import sw_cases
import sw_oracle as O
from juliaraytracingsw_amd import two_layer_qg as QG2
from juliaraytracingsw_amd._lib import LibSWError

pytestmark = pytest.mark.gpu
QG_CASES = ["qg2_ifmab3", "qg2_ifmrk4", "qg2_fab3"]
RTOL = 1e-10


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _setup(name, n=64):
    p = sw_cases.case_params(name, n)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p, aliased_state=True)
    prob.sol = pr.sol
    return p, pr, prob


def _aliased_mask(grid):
    live = np.zeros((grid.nl, grid.nkr), bool)
    d = grid.dealias(np.ones((1, grid.nl, grid.nkr), np.complex128))[0]
    live[d != 0] = True
    return ~live


def _full_err(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


@pytest.mark.parametrize("name", QG_CASES + ["rsw_fab3", "rsw_ifmab3", "rsw_ifmrk4", "ty_etdrk4"])
def test_full_state_matches_the_reference_array(name):
    """prob.sol after each of 12 steps equals the oracle's un-dealiased
    post-step state on every mode, the aliased ones included (nonzero)."""
    p, pr, prob = _setup(name)
    mask = _aliased_mask(pr.grid)
    for s in range(12):
        pr.stepforward(1)
        prob.stepforward(1)
        got = prob.sol
        assert _full_err(got, pr.sol) < RTOL, (s, _full_err(got, pr.sol))
    amax = np.max(np.abs(pr.sol[:, mask]))
    assert amax > 1e-9 * np.max(np.abs(pr.sol))  # the aliased modes are there
    # and right on their own scale, not just below the state's
    aerr = np.max(np.abs(got[:, mask] - pr.sol[:, mask])) / amax
    print(f"[aliased] {name}: aliased modes up to {amax / np.max(np.abs(pr.sol)):.1e} of the state, "
          f"their error {aerr:.1e} of themselves")
    assert aerr < 1e-8
    prob.close()


@pytest.mark.parametrize("name,n,steps", [("qg2_ifmab3", 512, 6), ("qg2_ifmrk4", 1024, 3)])
def test_full_state_larger_grids(name, n, steps):
    """The same on one-line-per-block grids (512², 1024²: the aliased column
    kernel's other block shape, aliased regions of 86k / 350k modes)."""
    p, pr, prob = _setup(name, n)
    pr.stepforward(steps)
    prob.stepforward(steps)
    got = prob.sol
    assert _full_err(got, pr.sol) < RTOL
    mask = _aliased_mask(pr.grid)
    assert np.max(np.abs(pr.sol[:, mask])) > 0
    prob.close()


@pytest.mark.parametrize("name", QG_CASES)
def test_energy_records_of_the_undealiased_state(name):
    """The device energy records (swqg/TwoLayerDriver.jl:86-89) against the
    oracle's energies of the UN-dealiased post-step state within 1e-10 — the
    done-criterion of VERDICT r02 #8 (the default mode is compared with the
    dealiased state in test_gpu_parity.py)."""
    p, pr, prob = _setup(name)
    freq, nsteps = 3, 12
    KE = QG2.Diagnostic(QG2.kinetic_energy, prob, freq=freq, nsteps=nsteps)
    PE = QG2.Diagnostic(QG2.potential_energy, prob, freq=freq, nsteps=nsteps)
    expected, gap = [O.qg2_energies(pr.sol, pr.grid, pr.params)], 0.0
    for s in range(1, nsteps + 1):
        pr.stepforward(1)
        if s % freq == 0:
            full = O.qg2_energies(pr.sol, pr.grid, pr.params)
            deal = O.qg2_energies(pr.grid.dealias(pr.sol.copy()), pr.grid, pr.params)
            gap = max(gap, abs(full[1] / deal[1] - 1), max(abs(a / b - 1) for a, b in zip(full[0], deal[0])))
            expected.append(full)
    QG2.stepforward(prob, [KE, PE], nsteps)
    assert KE.i == len(expected)
    for i, ((k1, k2), pe) in enumerate(expected):
        assert np.allclose(np.atleast_1d(KE.data[i]), [k1, k2], rtol=RTOL, atol=0), (i, KE.data[i], (k1, k2))
        assert abs(PE.data[i] / pe - 1) < RTOL, (i, PE.data[i], pe)
    print(f"[aliased] {name}: full-array vs dealiased energies differ by up to {gap:.2e} (relative)")
    # the instantaneous diagnostics read the same full array
    (k1, k2), pe = O.qg2_energies(pr.sol, pr.grid, pr.params)
    assert abs(QG2.potential_energy(prob) / pe - 1) < RTOL
    prob.close()


@pytest.mark.parametrize("name", ["qg2_ifmab3", "qg2_ifmrk4", "rsw_ifmab3", "ty_etdrk4"])
def test_calcN_on_every_mode(name):
    """sw_calcN returns N on the full array, as the reference's calcN!."""
    p, pr, prob = _setup(name)
    pr.stepforward(2)
    prob.stepforward(2)
    x = pr.sol.copy()
    ref = pr.calcN(x.copy(), pr.grid, pr.params)
    got = prob.calcN(x)
    mask = _aliased_mask(pr.grid)
    amax = np.max(np.abs(ref[:, mask]))
    assert amax > 1e-7 * np.max(np.abs(ref))
    assert _full_err(got, ref) < RTOL
    assert np.max(np.abs(got[:, mask] - ref[:, mask])) < 1e-8 * amax  # on the aliased modes' own scale
    prob.close()


def test_ty_energies_of_the_undealiased_state():
    """Thomas–Yamada's energies read prob.sol (thomasyamada/ThomasYamada.jl
    :333-367), whose aliased modes the ETDRK4 update sets (α N₁ + 2β (N₂ +
    N₃) + Γ N₄ there, calcN! returning N on every mode): barotropic,
    baroclinic and the wave/geostrophic split of the full array within 1e-10."""
    from juliaraytracingsw_amd import thomas_yamada as TY

    p, pr, prob = _setup("ty_etdrk4")
    for _ in range(3):
        pr.stepforward(2)
        prob.stepforward(2)
        bt, bc, wg = O.ty_energies(pr.sol.copy(), pr.grid)
        deal = O.ty_energies(pr.grid.dealias(pr.sol.copy()), pr.grid)
        assert abs(TY.barotropic_energy(prob) / bt - 1) < RTOL
        assert np.allclose(TY.baroclinic_energy(prob), bc, rtol=RTOL, atol=0)
        got = TY.wave_geostrophic_energy(prob)
        assert np.allclose(np.ravel(got), np.ravel(wg), rtol=RTOL, atol=0), (got, wg)
    gap = abs(bc[0] / deal[1][0] - 1)
    print(f"[aliased] ty_etdrk4: full-array vs dealiased baroclinic KE differ by {gap:.2e} (relative)")
    assert gap > 1e-14  # the aliased modes count
    prob.close()


def test_checkpoint_carries_the_aliased_history():
    """IFMAB3's AB3 combination at the aliased modes needs N of the two
    previous steps there: a checkpoint/restart continues bitwise on every mode
    (records included)."""
    p, pr, prob = _setup("qg2_ifmab3")
    prob.stepforward(7)
    blob = prob.ctx.get_checkpoint()
    prob.stepforward(5)
    want = prob.sol
    b = sw_cases.libsw_problem(p, aliased_state=True)
    b.ctx.set_checkpoint(blob)
    b.stepforward(5)
    assert np.array_equal(b.sol, want)
    assert np.max(np.abs(want[:, _aliased_mask(pr.grid)])) > 0
    b.close()
    prob.close()


def test_abi8_checkpoint_aliased_state_inferred():
    """before ABI 9 the checkpoint header's aliased_state field
    was reserved (0) whatever the writer tracked.  An ABI-8 blob is matched
    by its own aliased modes: one written with aliased_state (nonzero there)
    restores into an aliased context — bitwise, as an ABI-9 one — and is
    refused by a default one (which would drop those modes); a default
    context's ABI-8 blob (zeros there) restores into either."""

    def abi8(blob):
        b = blob.copy()
        b[8:12] = np.frombuffer(np.int32(8).tobytes(), np.uint8)     # CkptHeader.abi
        b[56:64] = np.frombuffer(np.int64(0).tobytes(), np.uint8)    # aliased_state: reserved then
        return b

    p, pr, prob = _setup("qg2_ifmab3")
    prob.stepforward(7)
    blob = abi8(prob.ctx.get_checkpoint())
    prob.stepforward(5)
    want = prob.sol
    b = sw_cases.libsw_problem(p, aliased_state=True)
    b.ctx.set_checkpoint(blob)
    b.stepforward(5)
    assert np.array_equal(b.sol, want)
    d = sw_cases.libsw_problem(p)
    with pytest.raises(LibSWError, match="holding aliased modes"):
        d.ctx.set_checkpoint(blob)
    d.sol = pr.sol
    d.stepforward(4)
    dblob = abi8(d.ctx.get_checkpoint())
    d2 = sw_cases.libsw_problem(p)
    d2.ctx.set_checkpoint(dblob)
    d.stepforward(3)
    d2.stepforward(3)
    assert np.array_equal(d.sol, d2.sol)
    #  a blob with all-zero aliased modes is valid for an
    # aliased_state context too: the same state as the default run's, its
    # aliased modes then evolve from zero
    b.ctx.set_checkpoint(dblob)
    b.stepforward(3)
    got = pr.grid.dealias(b.sol.copy())
    assert np.max(np.abs(got - d2.sol)) <= 1e-13 * np.max(np.abs(d2.sol))
    for x in (b, d, d2, prob):
        x.close()


def test_abi8_step0_aliased_blob_loads_both_ways():
    """an aliased_state context's ABI-8 checkpoint taken right
    after set_state with a dealiased IC (all aliased modes zero) restores into
    a default context and into an aliased_state one, and both continue as the
    context it was taken from does on the live modes."""
    p, pr, prob = _setup("qg2_ifmab3")
    prob.sol = pr.grid.dealias(pr.sol.copy())
    blob = prob.ctx.get_checkpoint().copy()
    blob[8:12] = np.frombuffer(np.int32(8).tobytes(), np.uint8)
    blob[56:64] = 0
    prob.stepforward(4)
    want = prob.sol
    for alias in (False, True):
        q = sw_cases.libsw_problem(p, aliased_state=alias)
        q.ctx.set_checkpoint(blob)
        q.stepforward(4)
        got = q.sol if alias else pr.grid.dealias(q.sol.copy())
        ref = want if alias else pr.grid.dealias(want.copy())
        assert np.max(np.abs(got - ref)) <= 1e-13 * np.max(np.abs(ref))
        q.close()
    prob.close()


def test_abi8_blob_of_another_problem_same_size_refused():
    """an ABI-8 blob of the same byte count but another
    problem — 2LQG IFMAB3 64x64 (state + 2 history slots of 2 fields) against
    RSW IFMRK4 64x128 (the state alone, 3 fields: 3*2*33*64 = 3*33*128
    modes) — is refused as another problem before its aliased modes are
    scanned (the scan would read 3 arrays of the RSW shape past the blob)."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW

    p, pr, prob = _setup("qg2_ifmab3")
    blob = prob.ctx.get_checkpoint().copy()
    blob[8:12] = np.frombuffer(np.int32(8).tobytes(), np.uint8)
    blob[56:64] = 0
    r = RSW.Problem("gpu", nx=64, ny=128, dt=1e-3, stepper="IFMRK4")
    assert r.ctx.get_checkpoint().nbytes == blob.nbytes
    with pytest.raises(LibSWError, match="different problem"):
        r.ctx.set_checkpoint(blob)
    r.close()
    prob.close()


def test_updatevars_dealiases_the_state():
    """updatevars! begins with dealias!(sol, grid) (swqg/TwoLayerQG.jl:115):
    after it prob.sol has zeros at the aliased modes, as the reference's."""
    p, pr, prob = _setup("qg2_ifmab3")
    prob.stepforward(4)
    mask = _aliased_mask(pr.grid)
    assert np.max(np.abs(prob.sol[:, mask])) > 0
    QG2.updatevars(prob)
    assert np.max(np.abs(prob.sol[:, mask])) == 0
    prob.close()


def test_default_mode_unchanged():
    """aliased_state off: live modes only, zeros elsewhere (the round-2
    behaviour the other parity tests pin)."""
    p = sw_cases.case_params("qg2_ifmab3", 64)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    prob = sw_cases.libsw_problem(p)
    prob.sol = pr.sol
    prob.stepforward(5)
    got = prob.sol
    assert np.max(np.abs(got[:, _aliased_mask(pr.grid)])) == 0
    prob.close()


@pytest.mark.parametrize("stepper,slabs", [("FilteredRK4", (1, 2)), ("FilteredAB3", (1, 2))])
def test_mlqg_full_state(stepper, slabs):
    """GeophysicalFlows MultiLayerQG with aliased_fraction = 0, stepped by
    FilteredRK4 (simulation/TwoLayerSimulation.jl:37-38, Parameters.jl:25) or
    FilteredAB3 (FreelyEvolvingSimulation.jl:38-39, FreelyEvolvingParameters
    .jl:7).  GF's calcN! dealiases its input (the Nyquist column and row) and
    returns N there; the update writes filter·dt·(RK4 or AB3 sum of N) into
    prob.sol there (the stage inputs' L·x reads the dealiased zeros), with
    the filter ≤ tol = 1e-15 at K ≥ 1: values ~1e-18 of the state, compared
    here on their own scale.  Also: calcN on every mode, the full-array
    energies, updatevars! clearing them, and in-process slabs bitwise."""
    from juliaraytracingsw_amd import multilayer_qg as MLQG

    p = dict(sw_cases.case_params("mlqg_frk4", 64), stepper=stepper)
    pr = sw_cases.oracle_problem(p)
    pr.set_solution(sw_cases.initial_condition(p, pr.grid))
    ic = pr.sol.copy()
    mask = _aliased_mask(pr.grid)
    steps = 12
    pr.stepforward(steps)
    got = {}
    for P in slabs:
        prob = sw_cases.libsw_problem(p, aliased_state=True,
                                      decomposition=None if P == 1 else dict(nranks=P, local_slabs=P))
        prob.sol = ic
        prob.stepforward(steps)
        got[P] = prob.sol
        if P != slabs[0]:
            prob.close()
            continue
        keep = prob
    for P in slabs[1:]:
        assert np.array_equal(got[P], got[slabs[0]]), P
    prob, sol = keep, got[slabs[0]]
    assert _full_err(sol, pr.sol) < RTOL
    amax = np.max(np.abs(pr.sol[:, mask]))
    assert amax > 0  # the aliased modes are there, however small
    aerr = np.max(np.abs(sol[:, mask] - pr.sol[:, mask])) / amax
    print(f"[aliased] mlqg {stepper}: aliased modes {amax / np.max(np.abs(pr.sol)):.1e} of the state, "
          f"their error {aerr:.1e} of themselves")
    assert aerr < 1e-8
    (k1, k2), (pe,) = MLQG.energies(prob)
    (o1, o2), po = O.mlqg_energies(pr.sol, pr.grid, pr.params)
    assert np.allclose([k1, k2, pe], [o1, o2, po], rtol=RTOL, atol=0)
    x = pr.sol.copy()
    ref = pr.calcN(x.copy(), pr.grid, pr.params)
    gotN = prob.calcN(x)
    nmax = np.max(np.abs(ref[:, mask]))
    assert nmax > 1e-3 * np.max(np.abs(ref))
    assert _full_err(gotN, ref) < RTOL
    # (the oracle's mean-flow and background-gradient terms go through the
    # transforms as GF's do: round-off at the Nyquist modes, ~1e-15 of N there)
    assert np.max(np.abs(gotN[:, mask] - ref[:, mask])) < 1e-8 * nmax
    MLQG.updatevars(prob)  # GF's updatevars! dealiases sol first
    assert np.max(np.abs(prob.sol[:, mask])) == 0
    prob.close()


def test_rejected_where_not_built():
    """Only where it is built: RSW / 2LQG with IFMAB3/IFMRK4/FilteredAB3,
    Thomas–Yamada with ETDRK4, MultiLayerQG (not 2LQG with FilteredRK4).
    (One slab per process is built: tests/test_gpu_multiprocess.py.)"""
    from juliaraytracingsw_amd import _lib

    cfg = _lib.default_config()
    cfg.model, cfg.stepper, cfg.nx, cfg.ny = _lib.SW_MODEL_QG2, _lib.STEPPERS["IFMAB3"], 64, 64
    cfg.aliased_state = 1
    cfg.stepper = _lib.STEPPERS["FilteredRK4"]
    with pytest.raises(LibSWError, match="aliased_state"):
        _lib.Context(cfg)


def _alias_case(name, nx, ny, amp, seed=11):
    """Oracle problem on an nx × ny grid with a random IC spread over the live
    band (products then reach the aliased modes), and a libsw builder."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW
    from juliaraytracingsw_amd import thomas_yamada as TY

    p = sw_cases.case_params(name, 256)
    dt = 1e-3
    if p["model"] == "ty":  # (ν K^16 negligible: every mode, the aliased ones, stays active)
        pr = O.Problem("ty", "ETDRK4", nx, dt, Lx=p["Lx"], ny=ny, params=O.TYParams(1e-50, 8, p["Ro"]))
        pr.set_solution(pr.grid.rfft(amp * np.random.default_rng(seed).standard_normal((4, ny, nx))))

        def make_ty(P):
            dec = None if P == 1 else dict(nranks=P, local_slabs=P)
            return TY.Problem("gpu", nx=nx, ny=ny, Lx=p["Lx"], dt=dt, nu=1e-50, nnu=8, Ro=p["Ro"],
                              aliased_state=True, decomposition=dec)
        return pr, make_ty
    if p["model"] == "rsw":
        params = O.RSWParams(1e-30, 4, p["f"], p["Cg"])
    else:
        params = O.QG2Params(p["U"], p["mu"], 1e-30, 4, F=p["F"])
    fk = dict(order=p["order"]) if p["stepper"] == "FilteredAB3" else {}
    pr = O.Problem(p["model"], p["stepper"], nx, dt, params=params, ny=ny, **fk)
    g = pr.grid
    nf = 3 if p["model"] == "rsw" else 2
    spec = g.rfft(amp * np.random.default_rng(seed).standard_normal((nf, ny, nx)))
    pr.set_solution(spec)

    def make(P):
        dec = None if P == 1 else dict(nranks=P, local_slabs=P)
        if p["model"] == "rsw":
            return RSW.Problem("gpu", nx=nx, ny=ny, dt=dt, nu=1e-30, nnu=4, f=p["f"], Cg=p["Cg"],
                               stepper=p["stepper"], aliased_state=True, decomposition=dec, **fk)
        return QG2.Problem("gpu", nx=nx, ny=ny, dt=dt, nu=1e-30, nnu=4, U=p["U"], mu=p["mu"], f0=p["f0"],
                           Cg=p["Cg"], drhorho0=p["drhorho0"], stepper=p["stepper"], T=np.float64,
                           aliased_state=True, decomposition=dec, **fk)
    return pr, make


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,nx,ny,slabs,steps,amp", [
    ("qg2_ifmab3", 4096, 4096, (1, 4), 4, 2.0),   # P = 4 at 4096²
    ("qg2_ifmrk4", 8192, 32, (1,), 3, 2.0),      # an 8192-point row (the full-length row with ALIAS)
    ("rsw_ifmab3", 256, 256, (1, 2, 4), 6, 0.3),  # RSW's advective form on 2 and 4 slabs
    ("qg2_fab3", 512, 512, (1, 2, 8), 6, 2.0),
    ("ty_etdrk4", 256, 256, (1, 2, 4), 3, 0.5),    # Thomas–Yamada's ETDRK4 on slabs
    ("ty_etdrk4", 8192, 32, (1,), 2, 0.5),         # and an 8192-point row
])
def test_full_state_on_slabs_and_long_rows(name, nx, ny, slabs, steps, amp):
    """prob.sol on every mode of the full array, the aliased ones included,
    against the oracle's un-dealiased state after `steps` steps, within 1e-10
    — on P in-process slabs (the aliased columns on slab 0, every slab's
    aliased rows of its own columns) bitwise equal to one slab — and its
    aliased modes on their own scale."""
    pr, make = _alias_case(name, nx, ny, amp)
    ic = pr.sol.copy()
    pr.stepforward(steps)
    ref = pr.sol
    mask = _aliased_mask(pr.grid)
    amax = np.max(np.abs(ref[:, mask]))
    assert amax > 1e-12 * np.max(np.abs(ref))  # the aliased modes are there
    got = {}
    for P in slabs:
        prob = make(P)
        prob.sol = ic
        prob.stepforward(steps)
        got[P] = prob.sol
        prob.close()
    for P in slabs[1:]:
        assert np.array_equal(got[P], got[slabs[0]]), P
    g1 = got[slabs[0]]
    assert _full_err(g1, ref) < RTOL, _full_err(g1, ref)
    aerr = np.max(np.abs(g1[:, mask] - ref[:, mask])) / amax
    print(f"[aliased] {name} {nx}x{ny} P={slabs}: aliased modes {amax / np.max(np.abs(ref)):.1e} of the state, "
          f"their error {aerr:.1e} of themselves")
    assert aerr < 1e-6


@pytest.mark.parametrize("stepper", ["IFMAB3", "IFMRK4"])
def test_nop_calcN_zeroes_the_aliased_N(stepper):
    """With NOPcalcN! (rsw/RotatingShallowWater.jl:135) N is zero on every
    mode, the aliased ones included (their N buffers were left as
    they were): the IF steppers then propagate the full state linearly,
    exp(n dt L)·sol0 per mode, at the aliased modes too."""
    from juliaraytracingsw_amd import rotating_shallow_water as RSW

    n, dt, steps = 64, 0.01, 7
    g = O.TwoDGrid(n)
    prob = RSW.Problem("gpu", nx=n, dt=dt, nu=1e-9, f=3.0, Cg=1.0, stepper=stepper, nop_calcN=True,
                       aliased_state=True)
    rng = np.random.default_rng(7)
    ic = rng.standard_normal((3, n, n // 2 + 1)) + 1j * rng.standard_normal((3, n, n // 2 + 1))
    c0 = ic[:, :, 0]
    ic[:, :, 0] = 0.5 * (c0 + np.conj(c0[:, (-np.arange(n)) % n]))  # a real field's kr = 0 column
    ic[:, :, -1] = 0.0  # the Nyquist column is not carried
    prob.ctx.set_state(ic)
    x = prob.ctx.get_state()
    mask = _aliased_mask(g)
    assert np.max(np.abs(x[:, mask])) > 0.1  # the aliased modes are held
    assert np.max(np.abs(prob.calcN(x))) == 0.0
    prob.ctx.step(steps)
    L = O.rsw_L(g, O.RSWParams(1e-9, 4, 3.0, 1.0))
    exact = O.mvmul(O.expm_batched(L * (steps * dt)), x)
    assert _full_err(prob.ctx.get_state(), exact) < 1e-12
    prob.close()
