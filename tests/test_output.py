"""CPU tests of the snapshot output / restart layer (juliaraytracingsw_amd.output,
SURVEY §8f rank 4): the JLD2 key layout, SequencedOutputs' roll-over
accounting (utils/SequencedOutputs.jl:37-57) and load_from_snapshot!'s
spectral resampling (rsw/RSWDriver.jl:17-36), on a host stand-in problem."""
import numpy as np

from juliaraytracingsw_amd import output
from juliaraytracingsw_amd.grid import TwoDGrid


class _Clock:
    def __init__(self):
        self.dt, self.t, self.step = 0.1, 0.0, 0

    def set(self, t, step):
        self.t, self.step = t, step


class _Ctx:
    """Host stand-in for the libsw context: records sw_reset_history."""

    def __init__(self):
        self.resets = 0

    def reset_history(self):
        self.resets += 1

    def history_slots(self):
        return 2


class _Prob:
    """Host stand-in with the Problem attributes output.py reads."""

    def __init__(self, n, nf=3):
        from juliaraytracingsw_amd import _lib

        self.grid = TwoDGrid(n, 2 * np.pi, n, 2 * np.pi, 1 / 3)
        self.model, self.stepper = _lib.SW_MODEL_RSW, "FilteredAB3"
        self.params = {"f": 3.0, "Cg": 1.0}
        self.clock = _Clock()
        self.ctx = _Ctx()
        self._sol = np.zeros((nf, n, n // 2 + 1), complex)

    @property
    def sol(self):
        return self._sol.copy()

    @sol.setter
    def sol(self, v):
        self._sol = np.asarray(v, complex).copy()


def test_output_layout_and_restart(tmp_path):
    pr = _Prob(32)
    rng = np.random.default_rng(0)
    fn = str(tmp_path / "rsw.jld2")
    out = output.Output(pr, fn)
    output.saveproblem(out)
    states = {}
    for step in (0, 5, 10):
        pr.clock.set(step * 0.1, step)
        pr.sol = rng.standard_normal(pr._sol.shape) + 1j * rng.standard_normal(pr._sol.shape)
        states[step] = pr.sol
        output.saveoutput(out)
    with np.load(fn) as d:
        assert int(d["grid/nx"]) == 32 and float(d["grid/Lx"]) == 2 * np.pi
        assert float(d["clock/dt"]) == 0.1 and str(d["eqn/model"]) == "RotatingShallowWater"
        assert np.array_equal(d["snapshots/sol/5"], states[5])
        assert float(d["snapshots/t/10"]) == 1.0
    assert output.snapshot_keys(fn) == ["snapshots/sol/0", "snapshots/sol/5", "snapshots/sol/10"]
    q = _Prob(32)
    assert output.restart(q, fn) == 10
    assert np.array_equal(q.sol, states[10]) and q.clock.t == 1.0 and q.clock.step == 10
    # no history in a snapshot file: the AB3 steppers restart with Euler steps
    assert q.ctx.resets == 1


def test_sequenced_output_rolls_over(tmp_path):
    pr = _Prob(32)
    name = lambda i: str(tmp_path / f"out.{i:08d}")  # noqa: E731  (RSWDriver.jl:186 naming)
    so = output.SequencedOutput(pr, name, max_writes=3)
    so.saveproblem()  # 1 write
    for step in range(1, 6):
        pr.clock.set(step, step)
        so.saveoutput()  # 1 write each (one field)
    # writes: problem + 2 outputs fill file 0; 3 outputs file 1; file 2 opened empty
    assert so.file_index == 2 and so.current_writes == 0
    assert output.snapshot_keys(name(0)) == ["snapshots/sol/1", "snapshots/sol/2"]
    assert output.snapshot_keys(name(1)) == ["snapshots/sol/3", "snapshots/sol/4", "snapshots/sol/5"]
    assert output.snapshot_keys(name(2)) == []


def test_load_from_snapshot_resampling():
    """A 32² spectrum embedded in a 64² grid by load_from_snapshot! is the
    same physical field: irfft2 on the fine grid of the embedded spectrum
    equals the coarse field sampled at every other point."""
    coarse = TwoDGrid(32, 2 * np.pi, 32, 2 * np.pi, 1 / 3)
    rng = np.random.default_rng(1)
    f = rng.standard_normal((1, 32, 32))
    fh = np.fft.rfft2(f)
    fh[..., 16] = 0  # drop the coarse Nyquist (not resolvable without a sign convention)
    fh[:, 16, :] = 0
    fine = _Prob(64, nf=1)
    output.load_from_snapshot(fine, fh)
    g = np.fft.irfft2(fine.sol, s=(64, 64))
    assert np.max(np.abs(g[:, ::2, ::2] - np.fft.irfft2(fh, s=(32, 32)))) < 1e-13
    assert coarse.nkr == 17
