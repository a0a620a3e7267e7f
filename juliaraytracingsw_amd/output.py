"""Snapshot output and restart.

Mirrors what the reference drivers write and read through FourierFlows
``Output`` / ``saveproblem`` / ``saveoutput`` and ``utils/SequencedOutputs.jl``
(rolling files of at most ``max_writes`` writes), and the restart path
``load_initial_condition_from_file!`` / ``load_from_snapshot!``
(rsw/RSWDriver.jl:10-36) with its spectral resampling onto a finer grid.

JLD2 (HDF5) is not available in this image, so a file is a zip archive of
``.npy`` members under the JLD2 key layout the reference's analysis scripts
read (rsw/fourier-analysis/FourierRSW.jl):

    grid/nx, grid/ny, grid/Lx, grid/Ly, grid/aliased_fraction
    params/<name>, clock/dt, eqn/model, timestepper/name
    snapshots/<field>/<step>, snapshots/t/<step>

readable with ``numpy.load(path)[key]`` (no pickles).  The state arrays are
the Julia column-major ``(nkr, nl, nf)`` spectra as numpy ``[nf][nl][nkr]``.
Host-side I/O only: the data come from ``sw_get_state`` once per write.
"""
from __future__ import annotations

import io
import zipfile

import numpy as np


def _put(zf: zipfile.ZipFile, key: str, value):
    buf = io.BytesIO()
    np.lib.format.write_array(buf, np.asarray(value), allow_pickle=False)
    zf.writestr(key + ".npy", buf.getvalue())


def _model_name(prob):
    from . import _lib

    return {_lib.SW_MODEL_RSW: "RotatingShallowWater", _lib.SW_MODEL_QG2: "TwoLayerQG",
            _lib.SW_MODEL_TY: "ThomasYamada", _lib.SW_MODEL_MLQG: "MultiLayerQG"}[prob.model]


class Output:
    """FF ``Output(prob, filename, (:name, getter), …)``.  ``fields`` maps a
    name to a function of ``prob`` (default: ``{"sol": lambda p: p.sol}``,
    the drivers' ``get_sol``, rsw/RSWDriver.jl:186-188)."""

    def __init__(self, prob, filename, fields=None):
        self.prob = prob
        self.path = filename
        self.fields = dict(fields or {"sol": lambda p: p.sol})
        with zipfile.ZipFile(self.path, "w"):
            pass

    def saveproblem(self):
        """FF ``saveproblem(out)``: grid, params, clock, equation, stepper."""
        p = self.prob
        g = p.grid
        with zipfile.ZipFile(self.path, "a") as zf:
            for k in ("nx", "ny", "Lx", "Ly", "aliased_fraction"):
                _put(zf, f"grid/{k}", getattr(g, k))
            for k, v in p.params.items():
                _put(zf, f"params/{k}", v)
            _put(zf, "clock/dt", p.clock.dt)
            _put(zf, "eqn/model", np.array(_model_name(p)))
            _put(zf, "timestepper/name", np.array(p.stepper))

    def saveoutput(self):
        """FF ``saveoutput(out)``: every field and t under the current step."""
        p = self.prob
        step = p.clock.step
        with zipfile.ZipFile(self.path, "a") as zf:
            _put(zf, f"snapshots/t/{step}", p.clock.t)
            for name, get in self.fields.items():
                _put(zf, f"snapshots/{name}/{step}", get(p))


def saveproblem(out):
    out.saveproblem()


def saveoutput(out):
    out.saveoutput()


class SequencedOutput:
    """utils/SequencedOutputs.jl:7-70: an ``Output`` that rolls over to
    ``filename_function(file_index + 1)`` once ``max_writes`` writes were made
    (saveproblem counts 1, saveoutput one per field)."""

    def __init__(self, prob, filename_function, fields=None, max_writes=100):
        self.max_writes = int(max_writes)
        self.current_writes = 0
        self.file_index = 0
        self.get_filename = filename_function
        self.output_file = Output(prob, filename_function(0), fields)

    def _check_writes(self):
        if self.current_writes >= self.max_writes:
            self.current_writes = 0
            self.file_index += 1
            o = self.output_file
            self.output_file = Output(o.prob, self.get_filename(self.file_index), o.fields)

    def saveproblem(self):
        self.output_file.saveproblem()
        self.current_writes += 1
        self._check_writes()

    def saveoutput(self):
        self.output_file.saveoutput()
        self.current_writes += len(self.output_file.fields)
        self._check_writes()

    def close(self):
        return None


def snapshot_keys(filename, field="sol"):
    """The ``snapshots/<field>/<step>`` keys of a file, in step order."""
    with np.load(filename) as d:
        ks = [k for k in d.files if k.startswith(f"snapshots/{field}/")]
    return sorted(ks, key=lambda k: int(k.rsplit("/", 1)[1]))


def load_from_snapshot(prob, snapshot):
    """rsw/RSWDriver.jl:17-36 ``load_from_snapshot!``: a (nf, snl, snkr)
    spectrum from a coarser (or equal) grid placed into this grid's
    (nf, nl, nkr) array — kr columns [0, snkr), l rows [0, half) and the last
    ``half`` rows, half = snkr - 1 — scaled by (nl / snl)² (the unnormalised
    r2c of the finer grid), then ``set_solution!`` (dealiases)."""
    snap = np.asarray(snapshot)
    g = prob.grid
    nf, snl, snkr = snap.shape
    if snkr > g.nkr or snl > g.nl:
        raise ValueError("snapshot grid is finer than the problem grid")
    half = snkr - 1
    scale = g.nl ** 2 / snl ** 2
    new = np.zeros((nf, g.nl, g.nkr), np.complex128)
    new[:, :half, :snkr] = scale * snap[:, :half, :]
    new[:, g.nl - half:, :snkr] = scale * snap[:, half:, :]
    prob.sol = new


def load_initial_condition_from_file(prob, filename, key):
    """rsw/RSWDriver.jl:10-15 ``load_initial_condition_from_file!``."""
    with np.load(filename) as d:
        snap = d[key[:-4] if key.endswith(".npy") else key]
    load_from_snapshot(prob, snap)


def checkpoint(prob, filename):
    """Write a restart file: the problem description (``saveproblem``), the
    state in the caller's precision (``checkpoint/sol``, for reading), and
    libsw's fp64 restart blob (``checkpoint/blob``, ``sw_get_checkpoint``):
    state, stepper history (RHS₋₁/RHS₋₂ or N₋₁/N₋₂ of the AB3 steppers),
    clock and any pending Euler start-up steps, all in fp64 whatever the
    problem's ``T`` — so that ``restart`` continues bit for bit as if the run
    had not stopped (a ``T = Float32`` problem's device state is fp64; a
    ComplexF32 copy would round it)."""
    out = Output(prob, filename)
    out.saveproblem()
    ctx = prob.ctx
    with zipfile.ZipFile(filename, "a") as zf:
        _put(zf, "checkpoint/sol", ctx.get_state())
        t, step = ctx.get_clock()
        _put(zf, "checkpoint/t", t)
        _put(zf, "checkpoint/step", step)
        _put(zf, "checkpoint/blob", ctx.get_checkpoint())
    return out


def restart(prob, filename, field="sol"):
    """Resume a run on the same grid.

    From a ``checkpoint`` file: the fp64 blob restores state, clock and
    stepper history, so the continuation equals uninterrupted stepping
    bitwise (also for ``T = Float32``).  From an ``Output`` file (its last
    ``snapshots/<field>/<step>``): state and clock (t, step); the history is
    not in the file, so the AB3 steppers restart with three forward-Euler
    steps (``sw_reset_history``), as they start at step 0 — which is what the
    reference's snapshot restart does (``load_from_snapshot!``,
    rsw/RSWDriver.jl:10-36, clock from zero)."""
    with np.load(filename) as d:
        if "checkpoint/blob" in d.files:
            prob.ctx.set_checkpoint(d["checkpoint/blob"])
            return int(d["checkpoint/step"])
        if "checkpoint/sol" in d.files:  # a checkpoint written before the blob (round 2 format)
            prob.sol = d["checkpoint/sol"]
            step = int(d["checkpoint/step"])
            prob.clock.set(float(d["checkpoint/t"]), step)
            k = 1
            while f"checkpoint/history/{k}" in d.files:
                prob.ctx.set_history(k, d[f"checkpoint/history/{k}"])
                k += 1
            if k == 1 and prob.ctx.history_slots() > 0:
                prob.ctx.reset_history()
            return step
    key = snapshot_keys(filename, field)[-1]
    step = int(key.rsplit("/", 1)[1])
    with np.load(filename) as d:
        prob.sol = d[key]
        t = float(d[f"snapshots/t/{step}"])
    prob.clock.set(t, step)
    prob.ctx.reset_history()
    return step
