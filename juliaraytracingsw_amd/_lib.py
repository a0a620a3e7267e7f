"""ctypes binding of libsw.so (include/sw.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every entry point raises ``LibSWError`` loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

SW_ABI_VERSION = 9
SW_MODEL_RSW, SW_MODEL_QG2, SW_MODEL_TY, SW_MODEL_MLQG = 0, 1, 2, 3
SW_STEP_FILTERED_AB3, SW_STEP_IFMAB3, SW_STEP_IFMRK4, SW_STEP_ETDRK4, SW_STEP_FILTERED_RK4 = 0, 1, 2, 3, 4
SW_OK, SW_E_INVALID, SW_E_NOMEM, SW_E_HIP, SW_E_COMM, SW_E_NAN, SW_E_STATE = 0, -1, -2, -3, -4, -5, -6
SW_PHYS_U, SW_PHYS_V, SW_PHYS_ETA, SW_PHYS_ZETA, SW_PHYS_Q, SW_PHYS_PSI = 0, 1, 2, 3, 4, 5
SW_DIAG_NAN, SW_DIAG_KE, SW_DIAG_PE, SW_DIAG_CFL, SW_DIAG_KE2, SW_DIAG_KE1, SW_DIAG_BT = 0, 1, 2, 3, 4, 5, 6
SW_DIAG_WAVE_KE, SW_DIAG_WAVE_PE, SW_DIAG_GEO_KE, SW_DIAG_GEO_PE = 7, 8, 9, 10
SW_PREC_F64, SW_PREC_F32 = 0, 1

STEPPERS = {"FilteredAB3": SW_STEP_FILTERED_AB3, "IFMAB3": SW_STEP_IFMAB3, "IFMRK4": SW_STEP_IFMRK4,
            "ETDRK4": SW_STEP_ETDRK4, "FilteredRK4": SW_STEP_FILTERED_RK4}

# every symbol include/sw.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "sw_config_default", "sw_create", "sw_destroy", "sw_last_error", "sw_get_dims",
    "sw_set_state", "sw_get_state", "sw_set_clock", "sw_get_clock", "sw_step", "sw_calcN",
    "sw_get_physical", "sw_diag", "sw_set_energy_diagnostics", "sw_get_energy_diagnostics",
    "sw_profile_steps", "sw_step_alg_bytes", "sw_comm_unique_id",
    "sw_history_slots", "sw_get_history", "sw_set_history", "sw_reset_history", "sw_slab_geometry",
    "sw_checkpoint_bytes", "sw_get_checkpoint", "sw_set_checkpoint", "sw_step_record",
    "sw_comm_profile", "sw_get_link_model",
]


class LibSWError(RuntimeError):
    """Raised for any libsw failure (load failure or a negative return code)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


# int exchange(void* user, const void* send, void* recv, size_t block_bytes, int32_t nranks)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int32)


class SwConfig(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32), ("model", C.c_int32), ("stepper", C.c_int32),
        ("nx", C.c_int32), ("ny", C.c_int32),
        ("Lx", C.c_double), ("Ly", C.c_double), ("aliased_fraction", C.c_double), ("dt", C.c_double),
        ("f", C.c_double), ("Cg", C.c_double), ("nu", C.c_double), ("nnu", C.c_int32),
        ("U", C.c_double), ("mu", C.c_double), ("F", C.c_double),
        ("use_filter", C.c_int32), ("filter_order", C.c_int32),
        ("filter_innerK", C.c_double), ("filter_outerK", C.c_double), ("filter_tol", C.c_double),
        ("device", C.c_int32), ("check_nan", C.c_int32), ("nop_calcN", C.c_int32), ("unfused", C.c_int32),
        ("nranks", C.c_int32), ("rank", C.c_int32), ("local_slabs", C.c_int32),
        ("comm_unique_id", C.c_void_p),
        ("exchange", EXCHANGE_FN), ("exchange_user", C.c_void_p),
        ("Ro", C.c_double),
        ("f0", C.c_double), ("beta", C.c_double),
        ("H", C.c_double * 2), ("b", C.c_double * 2), ("Ulayer", C.c_double * 2),
        ("precision", C.c_int32),
        ("aliased_state", C.c_int32),
    ]


class SwEnergyRecord(C.Structure):
    _fields_ = [("step", C.c_int64), ("t", C.c_double), ("ke", C.c_double), ("ke2", C.c_double),
                ("pe", C.c_double), ("wg", C.c_double * 4)]


class SwCommStats(C.Structure):
    _fields_ = [("nranks", C.c_int32), ("transport", C.c_int32), ("rccl_ranks", C.c_int32),
                ("pipelined", C.c_int32), ("row_chunks", C.c_int32), ("reserved", C.c_int32),
                ("step_us", C.c_double), ("exposed_us", C.c_double), ("bytes_sent", C.c_double)]


XPORT_NAMES = {0: "none", 1: "rccl", 2: "host-staged", 3: "in-process"}


class SwLinkModel(C.Structure):
    _fields_ = [("probed", C.c_int32), ("transport", C.c_int32), ("pipelined", C.c_int32),
                ("row_chunks", C.c_int32), ("latency_us", C.c_double), ("GBps", C.c_double),
                ("nhalf_bytes", C.c_double), ("msg_bytes", C.c_double), ("peer_GBps", C.c_double * 8)]


class SwKernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_int64), ("avg_ms", C.c_double),
                ("alg_bytes", C.c_double)]


_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsw.so")


def load(path: str | None = None):
    """Load libsw.so (once).  Raises LibSWError if it is missing."""
    global _LIB
    if _LIB is not None:
        return _LIB
    p = path or os.environ.get("LIBSW_PATH") or LIB_PATH
    if not os.path.exists(p):
        raise LibSWError(f"libsw.so not found at {p}: run __graft_entry__.build() (hipcc, gfx950)")
    try:
        lib = C.CDLL(p)
    except OSError as e:  # pragma: no cover
        raise LibSWError(f"failed to load {p}: {e}") from e
    vp, i32, i64, dbl, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_double, C.c_size_t
    sig = {
        "sw_config_default": (None, [C.POINTER(SwConfig)]),
        "sw_create": (C.c_int, [C.POINTER(vp), C.POINTER(SwConfig)]),
        "sw_destroy": (None, [vp]),
        "sw_last_error": (C.c_char_p, [vp]),
        "sw_get_dims": (C.c_int, [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
        "sw_set_state": (C.c_int, [vp, vp, sz]),
        "sw_get_state": (C.c_int, [vp, vp, sz]),
        "sw_set_clock": (C.c_int, [vp, dbl, i64]),
        "sw_get_clock": (C.c_int, [vp, C.POINTER(dbl), C.POINTER(i64)]),
        "sw_step": (C.c_int, [vp, i64]),
        "sw_calcN": (C.c_int, [vp, vp, vp, sz]),
        "sw_get_physical": (C.c_int, [vp, i32, vp, sz]),
        "sw_diag": (C.c_int, [vp, i32, C.POINTER(dbl)]),
        "sw_set_energy_diagnostics": (C.c_int, [vp, i64, i64]),
        "sw_get_energy_diagnostics": (C.c_int, [vp, C.POINTER(SwEnergyRecord), i64, C.POINTER(i64)]),
        "sw_profile_steps": (C.c_int, [vp, i64, C.POINTER(SwKernelStat), i32, C.POINTER(i32)]),
        "sw_step_alg_bytes": (dbl, [vp]),
        "sw_comm_unique_id": (C.c_int, [vp]),
        "sw_history_slots": (C.c_int, [vp, C.POINTER(i32)]),
        "sw_get_history": (C.c_int, [vp, i32, vp, sz]),
        "sw_set_history": (C.c_int, [vp, i32, vp, sz]),
        "sw_reset_history": (C.c_int, [vp]),
        "sw_slab_geometry": (C.c_int, [C.POINTER(SwConfig), i32, C.POINTER(i32)]),
        "sw_checkpoint_bytes": (C.c_int, [vp, C.POINTER(sz)]),
        "sw_get_checkpoint": (C.c_int, [vp, vp, sz]),
        "sw_set_checkpoint": (C.c_int, [vp, vp, sz]),
        "sw_step_record": (C.c_int, [vp, i64, C.POINTER(SwEnergyRecord)]),
        "sw_comm_profile": (C.c_int, [vp, i64, C.POINTER(SwCommStats)]),
        "sw_get_link_model": (C.c_int, [vp, C.POINTER(SwLinkModel)]),
    }
    for name, (res, args) in sig.items():
        if name == "sw_get_link_model" and not hasattr(lib, name):
            continue  # (a library from before round 6: diagnostics only; tests/test_abi.py requires it)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def default_config() -> SwConfig:
    lib = load()
    cfg = SwConfig()
    lib.sw_config_default(C.byref(cfg))
    return cfg


def slab_geometry(cfg: SwConfig, slab: int) -> dict:
    """sw_slab_geometry: the library's own slab layout (no GPU needed)."""
    out = (C.c_int32 * 8)()
    rc = load().sw_slab_geometry(C.byref(cfg), int(slab), out)
    if rc != SW_OK:
        raise LibSWError(f"sw_slab_geometry failed (code {rc})", rc)
    return dict(zip(("kc", "kcl", "kr0", "kcn", "nyl", "y0", "Lr", "LrP"), list(out)))


def comm_unique_id() -> bytes:
    """RCCL unique id (128 bytes) for rank 0 to broadcast (sw_comm_unique_id)."""
    buf = C.create_string_buffer(128)
    rc = load().sw_comm_unique_id(buf)
    if rc != SW_OK:
        raise LibSWError(f"sw_comm_unique_id failed (code {rc})", rc)
    return buf.raw


class Context:
    """Owning handle around one ``sw_ctx`` (one GPU, one problem)."""

    def __init__(self, cfg: SwConfig):
        self.lib = load()
        self._h = C.c_void_p()
        self.cfg = cfg
        rc = self.lib.sw_create(C.byref(self._h), C.byref(cfg))
        if rc != SW_OK:
            msg = self.lib.sw_last_error(self._h).decode() if self._h else "sw_create failed"
            self.lib.sw_destroy(self._h)
            self._h = C.c_void_p()
            raise LibSWError(f"sw_create: {msg} (code {rc})", rc)
        nkr, nl, nf = C.c_int32(), C.c_int32(), C.c_int32()
        self._check(self.lib.sw_get_dims(self._h, C.byref(nkr), C.byref(nl), C.byref(nf)), "sw_get_dims")
        self.nkr, self.nl, self.nf = nkr.value, nl.value, nf.value
        # caller-buffer element types (sw_config.precision, the reference's T)
        f32 = cfg.precision == SW_PREC_F32
        self.cdtype = np.dtype(np.complex64 if f32 else np.complex128)
        self.rdtype = np.dtype(np.float32 if f32 else np.float64)

    def _check(self, rc, what):
        if rc != SW_OK:
            raise LibSWError(f"{what}: {self.lib.sw_last_error(self._h).decode()} (code {rc})", rc)

    def close(self):
        if self._h:
            self.lib.sw_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- state: numpy [nf][nl][nkr] complex == Julia (nkr, nl, nf) ----------
    @property
    def state_shape(self):
        return (self.nf, self.nl, self.nkr)

    def _state_in(self, sol, what):
        a = np.ascontiguousarray(sol, dtype=self.cdtype)
        if a.shape != self.state_shape:
            raise ValueError(f"{what}: shape {a.shape} != {self.state_shape}")
        return a

    def _state_out(self, out, what):
        if out is None:
            return np.empty(self.state_shape, self.cdtype)
        if out.shape != self.state_shape or out.dtype != self.cdtype or not out.flags.c_contiguous:
            raise ValueError(f"{what}: out must be C-contiguous {self.cdtype} of the state shape")
        return out

    def set_state(self, sol):
        a = self._state_in(sol, "set_state")
        self._check(self.lib.sw_set_state(self._h, a.ctypes.data, a.nbytes), "sw_set_state")

    def get_state(self, out=None):
        """The state as Julia's (nkr, nl, nf) array; ``out`` (C-contiguous, of
        the caller precision and that shape) is filled in place, as FF's
        ``prob.sol``."""
        a = self._state_out(out, "get_state")
        self._check(self.lib.sw_get_state(self._h, a.ctypes.data, a.nbytes), "sw_get_state")
        return a

    def history_slots(self):
        n = C.c_int32()
        self._check(self.lib.sw_history_slots(self._h, C.byref(n)), "sw_history_slots")
        return n.value

    def get_history(self, slot, out=None):
        """RHS/N of ``slot`` (1 or 2) steps ago, state layout (sw_get_history)."""
        a = self._state_out(out, "get_history")
        self._check(self.lib.sw_get_history(self._h, int(slot), a.ctypes.data, a.nbytes), "sw_get_history")
        return a

    def set_history(self, slot, value):
        a = self._state_in(value, "set_history")
        self._check(self.lib.sw_set_history(self._h, int(slot), a.ctypes.data, a.nbytes), "sw_set_history")

    def reset_history(self):
        self._check(self.lib.sw_reset_history(self._h), "sw_reset_history")

    def get_checkpoint(self):
        """The fp64 restart blob (sw_get_checkpoint) as a uint8 array: state,
        history, clock, pending Euler start-up steps — exact whatever the
        caller precision."""
        n = C.c_size_t()
        self._check(self.lib.sw_checkpoint_bytes(self._h, C.byref(n)), "sw_checkpoint_bytes")
        buf = np.empty(n.value, np.uint8)
        self._check(self.lib.sw_get_checkpoint(self._h, buf.ctypes.data, buf.nbytes), "sw_get_checkpoint")
        return buf

    def set_checkpoint(self, blob):
        a = np.ascontiguousarray(blob, dtype=np.uint8)
        self._check(self.lib.sw_set_checkpoint(self._h, a.ctypes.data, a.nbytes), "sw_set_checkpoint")

    def calcN(self, sol):
        a = self._state_in(sol, "calcN")
        out = np.empty(self.state_shape, self.cdtype)
        self._check(self.lib.sw_calcN(self._h, a.ctypes.data, out.ctypes.data, a.nbytes), "sw_calcN")
        return out

    def set_clock(self, t, step):
        self._check(self.lib.sw_set_clock(self._h, float(t), int(step)), "sw_set_clock")

    def get_clock(self):
        t, s = C.c_double(), C.c_int64()
        self._check(self.lib.sw_get_clock(self._h, C.byref(t), C.byref(s)), "sw_get_clock")
        return t.value, s.value

    def step(self, n=1):
        self._check(self.lib.sw_step(self._h, int(n)), "sw_step")

    def physical(self, field_id, ny, nx):
        out = np.empty((ny, nx), self.rdtype)
        self._check(self.lib.sw_get_physical(self._h, int(field_id), out.ctypes.data, out.nbytes),
                    "sw_get_physical")
        return out

    def diag(self, diag_id):
        v = C.c_double()
        self._check(self.lib.sw_diag(self._h, int(diag_id), C.byref(v)), "sw_diag")
        return v.value

    def set_energy_diagnostics(self, freq, capacity):
        self._check(self.lib.sw_set_energy_diagnostics(self._h, int(freq), int(capacity)),
                    "sw_set_energy_diagnostics")

    def energy_diagnostics(self, max_records=None):
        """[(step, t, ke, ke2, pe, wg), …] recorded on the device while stepping
        (wg: TY's (wave KE, wave PE, geostrophic KE, geostrophic PE))."""
        cap = 1 << 20 if max_records is None else int(max_records)
        n = C.c_int64()
        self._check(self.lib.sw_get_energy_diagnostics(self._h, None, 0, C.byref(n)),
                    "sw_get_energy_diagnostics")
        buf = (SwEnergyRecord * max(1, min(cap, n.value)))()
        self._check(self.lib.sw_get_energy_diagnostics(self._h, buf, min(cap, n.value), C.byref(n)),
                    "sw_get_energy_diagnostics")
        return [(buf[i].step, buf[i].t, buf[i].ke, buf[i].ke2, buf[i].pe, tuple(buf[i].wg)) for i in range(n.value)]

    def step_record(self, n=1):
        """sw_step_record: n steps, the energies FF's Diagnostic functions read
        after the last one -> (step, t, ke, ke2, pe, wg).  SW_E_NAN raises
        LibSWError with ``.record`` set."""
        r = SwEnergyRecord()
        rc = self.lib.sw_step_record(self._h, int(n), C.byref(r))
        rec = (r.step, r.t, r.ke, r.ke2, r.pe, tuple(r.wg))
        if rc != SW_OK:
            e = LibSWError(f"sw_step_record: {self.lib.sw_last_error(self._h).decode()} (code {rc})", rc)
            e.record = rec
            raise e
        return rec

    def comm_profile(self, nsteps):
        """sw_comm_profile: nsteps steps of the production schedule (the state
        advances; collective on one slab per process) -> the exchange's
        transport, schedule and per-step exposed transpose time of this rank."""
        st = SwCommStats()
        self._check(self.lib.sw_comm_profile(self._h, int(nsteps), C.byref(st)), "sw_comm_profile")
        return dict(nranks=st.nranks, transport=XPORT_NAMES.get(st.transport, str(st.transport)),
                    rccl_ranks=st.rccl_ranks, schedule="pipelined" if st.pipelined else "sequential",
                    row_chunks=st.row_chunks, step_us=st.step_us, exposed_transpose_us=st.exposed_us,
                    sent_bytes_per_step=st.bytes_sent)

    def link_model(self):
        """sw_get_link_model: the link probe of sw_create (one slab per
        process) and the slab schedule chosen from it."""
        m = SwLinkModel()
        self._check(self.lib.sw_get_link_model(self._h, C.byref(m)), "sw_get_link_model")
        return dict(probed=bool(m.probed), transport=XPORT_NAMES.get(m.transport, str(m.transport)),
                    pipelined=bool(m.pipelined), row_chunks=m.row_chunks, latency_us=m.latency_us,
                    GBps_per_peer_direction=m.GBps, nhalf_bytes=m.nhalf_bytes, msg_bytes=m.msg_bytes,
                    peer_GBps=[x for x in m.peer_GBps])

    def profile(self, nsteps):
        st = (SwKernelStat * 16)()
        n = C.c_int32()
        self._check(self.lib.sw_profile_steps(self._h, int(nsteps), st, 16, C.byref(n)), "sw_profile_steps")
        return [dict(name=st[i].name.decode(), launches=st[i].launches, avg_ms=st[i].avg_ms,
                     alg_bytes=st[i].alg_bytes) for i in range(n.value)]

    def step_alg_bytes(self):
        return self.lib.sw_step_alg_bytes(self._h)
