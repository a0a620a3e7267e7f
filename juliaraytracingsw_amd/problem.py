"""Host-side mirror of the FourierFlows ``Problem`` that the reference drivers
hold (rsw/RotatingShallowWater.jl:70-99, swqg/TwoLayerQG.jl:55-90).  All
stepping happens in libsw on the GPU; this object only carries the handle,
the grid description and the clock view, so driver code reads like the
reference's (``prob.sol``, ``prob.clock``, ``stepforward!(prob, n)`` …).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from .grid import TwoDGrid


class Clock:
    """FF ``Clock``: a live view of the libsw clock (t, step) plus dt."""

    def __init__(self, ctx, dt):
        self._ctx, self.dt = ctx, float(dt)

    @property
    def t(self):
        return self._ctx.get_clock()[0]

    @property
    def step(self):
        return self._ctx.get_clock()[1]

    def set(self, t, step):
        self._ctx.set_clock(t, step)


class Problem:
    """A model + stepper instance resident on one GPU."""

    def __init__(self, model, *, nx, ny, Lx, Ly, dt, aliased_fraction, stepper, params,
                 use_filter=False, filter_kw=None, device=0, check_nan=True, T=np.float64,
                 nop_calcN=False, unfused=False, nranks=1, rank=0, local_slabs=1,
                 comm_unique_id=None, exchange=None, aliased_state=False):
        # T: the element type of the caller's buffers (prob.sol, vars), as the
        # reference's Problem(...; T) (rsw/RSWDriver.jl:164 and
        # swqg/TwoLayerDriver.jl:63 pass Float32); libsw computes in fp64
        if np.dtype(T) not in (np.dtype(np.float64), np.dtype(np.float32)):
            raise _lib.LibSWError(f"T must be Float64 or Float32, got {np.dtype(T)}")
        if stepper not in _lib.STEPPERS:
            raise ValueError(f"unknown stepper {stepper!r}; expected one of {list(_lib.STEPPERS)}")
        fk = dict(order=4, innerK=0.65, outerK=1.0, tol=1e-15)
        unknown = set(filter_kw or {}) - set(fk)
        if unknown:
            raise TypeError(f"unknown stepper kwargs {sorted(unknown)}")
        fk.update(filter_kw or {})
        cfg = _lib.default_config()
        cfg.model = model
        cfg.stepper = _lib.STEPPERS[stepper]
        cfg.nx, cfg.ny = int(nx), int(ny)
        cfg.Lx, cfg.Ly = float(Lx), float(Ly)
        cfg.aliased_fraction = float(aliased_fraction)
        cfg.dt = float(dt)
        for k, v in params.items():
            if k in ("H", "b", "Ulayer"):
                getattr(cfg, k)[:] = [float(x) for x in v]
            else:
                setattr(cfg, k, v)
        cfg.use_filter = 1 if use_filter else 0
        cfg.filter_order = int(fk["order"])
        cfg.filter_innerK = float(fk["innerK"])
        cfg.filter_outerK = float(fk["outerK"])
        cfg.filter_tol = float(fk["tol"])
        cfg.precision = _lib.SW_PREC_F32 if np.dtype(T) == np.float32 else _lib.SW_PREC_F64
        cfg.device = int(device)
        cfg.check_nan = 1 if check_nan else 0
        cfg.nop_calcN = 1 if nop_calcN else 0
        cfg.unfused = 1 if unfused else 0
        # carry the modes the 2/3 rule removes (RSW / 2LQG, slabs in one process: include/sw.h)
        cfg.aliased_state = 1 if aliased_state else 0
        # slab decomposition: nranks slabs; local_slabs == nranks
        # holds them all on this GPU, else this process holds slab `rank` and
        # transposes over RCCL with the broadcast comm_unique_id bytes
        cfg.nranks, cfg.rank, cfg.local_slabs = int(nranks), int(rank), int(local_slabs)
        self._uid = None
        if comm_unique_id is not None:
            self._uid = C.create_string_buffer(bytes(comm_unique_id), 128)
            cfg.comm_unique_id = C.cast(self._uid, C.c_void_p)
        self._xchg = exchange  # keep the callback alive as long as the context
        if exchange is not None:
            cfg.exchange = exchange
        self.ctx = _lib.Context(cfg)
        self.model = model
        self.stepper = stepper
        self.grid = TwoDGrid(nx, Lx, ny, Ly, aliased_fraction)
        self.clock = Clock(self.ctx, dt)
        self.params = dict(params)
        self.T = np.dtype(T).type
        self._efreq = None  # energy-diagnostics frequency recorded on the device

    # FF prob.sol (a host copy; assignment uploads and dealiases)
    @property
    def sol(self):
        return self.ctx.get_state()

    @sol.setter
    def sol(self, value):
        self.ctx.set_state(value)

    def stepforward(self, nsteps=1):
        """FF ``stepforward!(prob, nsteps)`` (rsw/RSWDriver.jl:212)."""
        self.ctx.step(nsteps)

    def calcN(self, sol):
        """``equation.calcN!(N, sol, …)`` on a caller state (no stepping)."""
        return self.ctx.calcN(sol)

    def close(self):
        self.ctx.close()

    def _attach_energy_diagnostics(self, freq, ndata):
        if self._efreq is None:
            self.ctx.set_energy_diagnostics(freq, ndata)
            self._efreq = freq
        elif freq != self._efreq:
            raise NotImplementedError("libsw records one energy-diagnostics frequency per problem")


class Diagnostic:
    """FF ``Diagnostic(calc, prob; freq, nsteps, ndata)`` for the energy
    diagnostics the drivers keep (rsw/RSWDriver.jl:193-196,
    swqg/TwoLayerDriver.jl:86-89): ``calc`` is a module's ``kinetic_energy``
    or ``potential_energy``.  Entry 0 is ``calc(prob)`` at construction; after
    every step with ``clock.step % freq == 0`` libsw reduces the energies on
    the device while stepping (sw_set_energy_diagnostics — no host round
    trip per diagnostic), and ``stepforward(prob, diags, n)`` appends them.
    Fields as FF's: ``data``, ``t``, ``steps``, ``value``, ``i`` (entries held),
    ``freq``."""

    def __init__(self, calc, prob, *, freq=1, nsteps=100, ndata=None):
        field = getattr(calc, "_sw_energy", None)
        if field is None:
            raise ValueError("libsw records the models' energy diagnostics (kinetic_energy, "
                             "potential_energy, baroclinic_energy, barotropic_energy, "
                             "wave_geostrophic_energy, energies)")
        ndata = int(ndata or math.ceil((nsteps + 1) / freq))
        prob._attach_energy_diagnostics(int(freq), ndata)
        self.calc, self.prob, self.freq, self._field = calc, prob, int(freq), field
        self.value = calc(prob)
        self.data = [None] * ndata
        self.t = np.zeros(ndata)
        self.steps = np.zeros(ndata, np.int64)
        self.data[0], self.t[0], self.steps[0] = self.value, prob.clock.t, prob.clock.step
        self.i = 1
        self._seen = 0  # device records consumed

    def _take(self, records):
        for step, t, ke, ke2, pe, wg in records[self._seen:]:
            if self.i >= len(self.data):
                break
            v = {"ke": ke, "pe": pe, "ke12": (ke, ke2), "bc": (ke, pe), "bt": ke2,
                 "mlqg": ((ke, ke2), (pe,)), "wg": ((wg[0], wg[1]), (wg[2], wg[3]))}[self._field]
            self.data[self.i], self.t[self.i], self.steps[self.i] = v, t, step
            self.value = v
            self.i += 1
        self._seen = len(records)


def increment(diags):
    """FF ``increment!(diags)``: pull the device-recorded energies."""
    diags = [diags] if isinstance(diags, Diagnostic) else list(diags)
    if diags:
        recs = diags[0].prob.ctx.energy_diagnostics()
        for d in diags:
            d._take(recs)


def stepforward(prob: Problem, diags_or_nsteps=1, nsteps=None):
    """``stepforward!(prob, nsteps)`` or ``stepforward!(prob, diags, nsteps)``
    (rsw/RSWDriver.jl:212, swqg/TwoLayerDriver.jl:105)."""
    if nsteps is None:
        prob.stepforward(int(diags_or_nsteps))
        return
    prob.stepforward(int(nsteps))
    increment(diags_or_nsteps)
