"""The GPU box's state around a timed region, for bench.py's JSON line.

A 5-10 % box-to-box swing (config 4's col_step read 345
µs on one box and 381 on another, same build) cannot be told apart from a
regression unless the line says what the box was doing.  This module reads
the amdsmi library in-process (the same firmware metrics table `amd-smi
metric` prints; no subprocess, no GPU work):

* ``static``: product, board serial, OAM id, PCI BDF, compute / memory
  partition (SPX/CPX, NPS1/NPS2), socket power cap, clock ranges, HBM peak;
* ``region``: sampled every ~5 ms by a thread while the timed region runs
  (the stepping thread sits in hipStreamSynchronize inside a ctypes call,
  which releases the GIL): mean / min / max of the current gfx clock (mean
  over the XCDs), memory clock, socket power, hotspot / HBM temperature; and
  deltas of the firmware accumulators over the region: energy (-> average
  power) and the throttle residencies (PPT, thermal, PROCHOT), so a region
  that ran power- or temperature-limited says so.

Every call is guarded: on a box without amdsmi (or a CPU container) the
fields are null with the reason, and bench.py's measurement is unaffected.
Not imported by the product (juliaraytracingsw_amd/) or the tests' GPU path.
"""
from __future__ import annotations

import socket
import statistics
import threading
import time


def _num(x):
    """amdsmi values: int/float, or 'N/A' / dicts with 'value'."""
    if isinstance(x, dict):
        x = x.get("value")
    if isinstance(x, (int, float)) and not isinstance(x, bool):
        # the firmware's "not supported" sentinels (0xFFFF, 0xFFFFFFFF, …)
        if x in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
            return None
        return x
    return None


def _clk_mean(v):
    """current_gfxclks is a list over the XCDs; N/A entries dropped."""
    if isinstance(v, (list, tuple)):
        xs = [_num(a) for a in v]
        xs = [a for a in xs if a]
        return statistics.fmean(xs) if xs else None
    return _num(v)


class BoxMonitor:
    def __init__(self, hip_device=0):
        self.err = None
        self.h = None
        self._samples = []
        self._stop = threading.Event()
        self._thread = None
        self._m0 = self._t0 = self._e0 = None
        try:
            import amdsmi

            self.smi = amdsmi
            amdsmi.amdsmi_init()
            handles = amdsmi.amdsmi_get_processor_handles()
            bdf = None
            try:  # the HIP device's PCI address -> the amdsmi handle of that GPU
                import torch

                p = torch.cuda.get_device_properties(hip_device)
                bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
            except Exception:  # noqa: BLE001
                bdf = None
            self.h = handles[min(hip_device, len(handles) - 1)] if handles else None
            if bdf:
                for h in handles:
                    try:
                        if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().startswith(bdf):
                            self.h = h
                            break
                    except Exception:  # noqa: BLE001
                        pass
            if self.h is None:
                self.err = "amdsmi: no GPU handle"
        except Exception as exc:  # noqa: BLE001 - recorded in the line
            self.err = f"amdsmi unavailable: {type(exc).__name__}: {exc}"

    # ------------------------------------------------------------------ static
    def static(self):
        out = {"host": socket.gethostname(), "error": self.err}
        if self.h is None:
            return out
        s, h = self.smi, self.h

        def get(name, fn):
            try:
                out[name] = fn()
            except Exception as exc:  # noqa: BLE001
                out[name] = f"n/a ({type(exc).__name__})"

        get("bdf", lambda: s.amdsmi_get_gpu_device_bdf(h))
        get("product", lambda: s.amdsmi_get_gpu_asic_info(h).get("market_name"))
        get("board_serial", lambda: s.amdsmi_get_gpu_board_info(h).get("product_serial"))
        get("oam_id", lambda: s.amdsmi_get_gpu_asic_info(h).get("oam_id"))
        get("compute_partition", lambda: s.amdsmi_get_gpu_compute_partition(h))
        get("memory_partition", lambda: s.amdsmi_get_gpu_memory_partition(h))

        def cap():
            c = s.amdsmi_get_power_cap_info(h)
            # microwatts in this amdsmi; reported in W
            return {k: (v / 1e6 if isinstance(v, (int, float)) and v > 1e4 else v) for k, v in c.items()}

        get("power_cap_W", cap)

        def clocks():
            r = {}
            for name, typ in (("gfx", s.AmdSmiClkType.GFX), ("mem", s.AmdSmiClkType.MEM)):
                c = s.amdsmi_get_clock_info(h, typ)
                r[name] = {k: c.get(k) for k in ("min_clk", "max_clk", "clk_locked", "clk_deep_sleep") if k in c}
            return r

        get("clock_range_MHz", clocks)

        def idle():
            m = s.amdsmi_get_gpu_metrics_info(h)
            return {"gfx_MHz": _clk_mean(m.get("current_gfxclks") or m.get("current_gfxclk")),
                    "mem_MHz": _num(m.get("current_uclk")), "hotspot_C": _num(m.get("temperature_hotspot")),
                    "hbm_C": _num(m.get("temperature_mem")), "socket_W": _num(m.get("current_socket_power"))}

        get("before_run", idle)
        return out

    # ------------------------------------------------------------------ region
    def _metrics(self):
        return self.smi.amdsmi_get_gpu_metrics_info(self.h)

    def _energy(self):
        try:
            e = self.smi.amdsmi_get_energy_count(self.h)
            return e["energy_accumulator"], e["counter_resolution"]
        except Exception:  # noqa: BLE001
            return None

    def _sample_loop(self, period):
        while not self._stop.is_set():
            try:
                m = self._metrics()
                self._samples.append((_clk_mean(m.get("current_gfxclks") or m.get("current_gfxclk")),
                                      _num(m.get("current_uclk")), _num(m.get("current_socket_power")),
                                      _num(m.get("temperature_hotspot")), _num(m.get("temperature_mem"))))
            except Exception:  # noqa: BLE001
                pass
            self._stop.wait(period)

    def start(self, period=0.005):
        if self.h is None:
            return
        self._samples = []
        self._stop.clear()
        try:
            self._m0 = self._metrics()
        except Exception:  # noqa: BLE001
            self._m0 = None
        self._e0 = self._energy()
        self._t0 = time.perf_counter()
        self._n0 = 0
        self._start_mark = (self._t0, self._m0, self._e0, 0)
        self._thread = threading.Thread(target=self._sample_loop, args=(period,), daemon=True)
        self._thread.start()

    def _mark(self):
        """(time, metrics, energy, sample count) now, for region boundaries"""
        try:
            m = self._metrics()
        except Exception:  # noqa: BLE001
            m = None
        return time.perf_counter(), m, self._energy(), len(self._samples)

    def lap(self):
        """the region since start() or the previous lap(), sampling continues
        (bench.py: the untimed warm-up as its own region inside the headline's)"""
        if self.h is None:
            return {"error": self.err}
        t1, m1, e1, n1 = self._mark()
        out = self._summary(self._t0, self._m0, self._e0, self._n0, t1, m1, e1, n1)
        self._t0, self._m0, self._e0, self._n0 = t1, m1, e1, n1
        return out

    def stop(self, whole=False):
        """the region since the last lap() (whole: since start())"""
        if self.h is None:
            return {"error": self.err}
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
        t1, m1, e1, n1 = self._mark()
        if whole:
            return self._summary(*self._start_mark, t1, m1, e1, n1)
        return self._summary(self._t0, self._m0, self._e0, self._n0, t1, m1, e1, n1)

    def _summary(self, t0, m0, e0, n0, t1, m1, e1, n1):
        dt = t1 - t0
        if e0 and e1 and e1[0] >= e0[0] and dt > 0:
            # energy counter x its resolution (µJ) over the region's wall time
            out_energy = (e1[0] - e0[0]) * e1[1] * 1e-6 / dt
            joules = (e1[0] - e0[0]) * e1[1] * 1e-6
        else:
            out_energy = joules = None
        smp = self._samples[n0:n1]
        out = {"seconds": dt, "samples": len(smp), "avg_power_W_from_energy": out_energy, "energy_J": joules}
        for i, name in enumerate(("gfx_MHz", "mem_MHz", "socket_W", "hotspot_C", "hbm_C")):
            xs = [q[i] for q in smp if q[i] is not None]
            out[name] = ({"mean": statistics.fmean(xs), "min": min(xs), "max": max(xs)} if xs else None)
        out["throttle_fraction"] = None
        out["throttle_status_after"] = None
        if m0 and m1:
            acc0, acc1 = _num(m0.get("accumulation_counter")), _num(m1.get("accumulation_counter"))
            res = {}
            for k in ("ppt_residency_acc", "socket_thm_residency_acc", "vr_thm_residency_acc",
                      "hbm_thm_residency_acc", "prochot_residency_acc"):
                a, b = _num(m0.get(k)), _num(m1.get(k))
                if a is not None and b is not None and acc0 is not None and acc1 is not None and acc1 > acc0:
                    # residency counters advance with accumulation_counter while
                    # the limit is active: the fraction of the region limited
                    res[k.replace("_residency_acc", "")] = (b - a) / (acc1 - acc0)
            out["throttle_fraction"] = res or None
            out["throttle_status_after"] = _num(m1.get("throttle_status"))
        return out
