"""Slab decomposition on one GPU: every slab of the
decomposition held by this process (local_slabs == nranks), the transposes
done as device copies with exactly the block pattern the RCCL all-to-all
moves.  Each column and each row is transformed by the same kernel code as in
the single-slab run, so the states must be bitwise identical."""
import numpy as np
import pytest

import sw_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded(libsw):
    return libsw


def _slabbed(p, P, **kw):
    return sw_cases.libsw_problem(p, decomposition=dict(nranks=P, local_slabs=P), **kw)


@pytest.mark.parametrize("overlap", [True, False, "chunks"])
@pytest.mark.parametrize("unfused", [False, True])
@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("name", sw_cases.ALL_CASES)
def test_slabs_bitwise(name, P, unfused, overlap, monkeypatch):
    """overlap: the pipelined schedule (column groups launched one by one,
    their transposes on the side stream, events between the streams); else
    the sequential schedule (SW_OVERLAP=0); "chunks": pipelined with the row
    pass in chunks of rows, each behind its part of the last inverse group's
    transposes (SW_ROW_CHUNKS).  All bitwise equal P = 1."""
    p = sw_cases.case_params(name, 128)
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    a = sw_cases.libsw_problem(p, unfused=unfused)
    monkeypatch.setenv("SW_OVERLAP", "0" if overlap is False else "1")
    if overlap == "chunks":
        monkeypatch.setenv("SW_ROW_CHUNKS", "4" if P == 2 else "2")
    b = _slabbed(p, P, unfused=unfused)
    monkeypatch.delenv("SW_OVERLAP", raising=False)
    monkeypatch.delenv("SW_ROW_CHUNKS", raising=False)
    a.sol = ic
    b.sol = ic
    assert np.array_equal(a.sol, b.sol)
    assert np.array_equal(a.calcN(ic), b.calcN(ic))
    for n in (2, 3, 4):
        a.stepforward(n)
        b.stepforward(n)
        assert np.array_equal(a.sol, b.sol), n
    a.close()
    b.close()


@pytest.mark.parametrize("overlap", [True, False, "chunks"])
@pytest.mark.parametrize("P", [2, 8])
def test_slabs_bitwise_2048(P, overlap, monkeypatch):
    """The metric configuration (RSW 2048² FilteredAB3) split 2 and 8 ways,
    pipelined (the RCCL default: at P = 2 its row pass runs in 4 chunks),
    pipelined in 4 row chunks, and sequential."""
    from juliaraytracingsw_amd import drivers

    a, _ = drivers.rsw_problem(2048, "FilteredAB3")
    monkeypatch.setenv("SW_OVERLAP", "0" if overlap is False else "1")
    if overlap == "chunks":
        monkeypatch.setenv("SW_ROW_CHUNKS", "4")
    b, _ = drivers.rsw_problem(2048, "FilteredAB3", decomposition=dict(nranks=P, local_slabs=P))
    monkeypatch.delenv("SW_OVERLAP", raising=False)
    monkeypatch.delenv("SW_ROW_CHUNKS", raising=False)
    a.stepforward(5)
    b.stepforward(5)
    assert np.array_equal(a.sol, b.sol)
    a.close()
    b.close()


@pytest.mark.parametrize("name", ["rsw_fab3", "qg2_ifmab3"])
def test_slabs_physical_and_energy(name):
    from juliaraytracingsw_amd import rotating_shallow_water as RSW, two_layer_qg as QG2

    M = RSW if name.startswith("rsw") else QG2
    p = sw_cases.case_params(name, 128)
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    a = sw_cases.libsw_problem(p)
    b = _slabbed(p, 4)
    a.sol = ic
    b.sol = ic
    a.stepforward(3)
    b.stepforward(3)
    va, vb = M.updatevars(a), M.updatevars(b)
    for k in va:
        assert np.array_equal(va[k], vb[k]), k
    # energies: per-column sums added in global column order -> bitwise equal
    assert np.sum(M.kinetic_energy(b)) == np.sum(M.kinetic_energy(a))
    assert M.potential_energy(b) == M.potential_energy(a)
    a.close()
    b.close()


def test_slabs_ty_energies():
    """TY's seven Parseval sums (barotropic, baroclinic, wave/geostrophic)
    repeat bitwise for any slab decomposition."""
    from juliaraytracingsw_amd import thomas_yamada as TY

    p = sw_cases.case_params("ty_etdrk4", 128)
    pr = sw_cases.oracle_problem(p)
    ic = sw_cases.initial_condition(p, pr.grid)
    a = sw_cases.libsw_problem(p)
    b = _slabbed(p, 4)
    a.sol = ic
    b.sol = ic
    a.stepforward(2)
    b.stepforward(2)
    for f in (TY.barotropic_energy, TY.baroclinic_energy, TY.wave_geostrophic_energy):
        assert f(a) == f(b), f.__name__
    a.close()
    b.close()


def test_slab_config_errors():
    from juliaraytracingsw_amd import LibSWError, rotating_shallow_water as RSW

    with pytest.raises(LibSWError):  # not a power of two
        RSW.Problem("gpu", nx=128, decomposition=dict(nranks=3, local_slabs=3))
    with pytest.raises(LibSWError):  # ny / nranks < 32
        RSW.Problem("gpu", nx=64, decomposition=dict(nranks=4, local_slabs=4))
    with pytest.raises(LibSWError):  # RCCL slab without a unique id
        RSW.Problem("gpu", nx=128, decomposition=dict(nranks=2, rank=0, local_slabs=1))


@pytest.mark.parametrize("overlap", [False, "chunks"])
def test_slabs_bitwise_8192_rows_forward_tiles(overlap, monkeypatch):
    """8192-point rows of the 2LQG family write their forward fields as 4×2
    tiles (Geom::fa = 2, config 5's layout); on several slabs those tiles' lines
    are in row order, so a chunk of rows stays one contiguous piece per peer
    block and the forward transposes can follow the row pass chunk by chunk.
    2LQG IFMRK4 on an 8192 × 512 grid over 2 slabs, sequential and pipelined in
    4 row chunks: bitwise equal to one slab."""
    from juliaraytracingsw_amd import two_layer_qg as QG2

    p = sw_cases.case_params("qg2_ifmrk4", 64)

    def make(dec=None):
        return QG2.Problem("gpu", nx=8192, ny=512, dt=1e-3, nu=1e-30, nnu=4, U=p["U"], mu=p["mu"], f0=p["f0"],
                           Cg=p["Cg"], drhorho0=p["drhorho0"], stepper="IFMRK4", T=np.float64,
                           decomposition=dec)

    a = make()
    rng = np.random.default_rng(5)
    shape = a.sol.shape
    ic = 1e-3 * (rng.standard_normal(shape) + 1j * rng.standard_normal(shape))
    a.sol = ic
    monkeypatch.setenv("SW_OVERLAP", "0" if overlap is False else "1")
    if overlap == "chunks":
        monkeypatch.setenv("SW_ROW_CHUNKS", "4")
    b = make(dict(nranks=2, local_slabs=2))
    monkeypatch.delenv("SW_OVERLAP", raising=False)
    monkeypatch.delenv("SW_ROW_CHUNKS", raising=False)
    b.sol = ic
    a.stepforward(2)
    b.stepforward(2)
    assert np.array_equal(a.sol, b.sol)
    assert np.max(np.abs(a.sol)) > 0
    a.close()
    b.close()
