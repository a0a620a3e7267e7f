#!/usr/bin/env python3
"""Driver-cadence rates: the frame loops of the drivers the
north star names, at the reference's own parameter files, through the ctypes
twin of integration/julia/SWLib.jl (tests/driver_replay.py: the same C calls
in the same order as the Julia binding), timed per frame and per C entry
point, beside the device-only rate of the same problem (one sw_step block).

    python tools/driver_cadence.py [--frames F] [--out FILE] [--only NAME ...]

Per driver (one JSON object each, and a table on stderr):
  steps_per_s_driver   steps of the frame loop / its wall time
  steps_per_s_device   the same context stepped in one sw_step block
  gpu_idle_fraction    1 - steps / (device rate x loop time)
  calls                per C entry point: count, total ms, ms per call
  host_ms              loop time outside every C call (the twin's Python:
                       FF's per-step seam and increment!, the NaN scan,
                       host copies for saveoutput, FFTW stand-ins)

The host share is the Python twin's, not Julia's: the C calls and their
synchronisation are the binding's own, the rest is an upper bound of what a
Julia driver spends there (Julia's loop overhead is smaller; JLD2 writes are
not replayed).  Reference: rsw/RSWDriver.jl:184-226 (RSWParameters.jl),
swqg/TwoLayerDriver.jl:71-117 (TwoLayerParameters.jl),
simulation/TwoLayerSimulation.jl:52,108-128 (Parameters.jl),
thomasyamada/TYdriver.jl:111-231 (gpu-setup/Parameters.jl).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import driver_replay as R  # noqa: E402
import sw_oracle as O  # noqa: E402


def rsw_cadence(nx=512):
    """rsw/RSWDriver.jl:134-154 with RSWParameters.jl (nx = 512, cfltune
    0.01, ag + aw = 0.3, output_dt = 0.025/f, diag_dt = 0.5, f = 3)"""
    dx = 2 * np.pi / nx
    dt = 0.01 / 0.3 * dx
    return dict(output_freq=max(math.floor(0.025 / 3 / dt), 1), diags_freq=max(math.floor(0.5 / dt), 1), dt=dt)


def qg2_cadence(nx=2048):
    """swqg/TwoLayerDriver.jl:29-58 with TwoLayerParameters.jl (nx = 2048,
    output_dt = 0.025/f, diag_dt = 0.5/f, f = 3)"""
    dt = O.qg2_driver_params(nx)["dt"]
    return dict(output_freq=max(math.floor(0.025 / 3 / dt), 1), diags_freq=max(math.floor(0.5 / 3 / dt), 1), dt=dt)


def _loop_window(tw, start="frames", end="end"):
    t = {lab: (tt, nc) for lab, tt, nc in tw.marks}
    return t[start][0], t[end][0], t[start][1], t[end][1]


def _calls_between(tw, times_before, times_after):
    out = {}
    for k, (n1, s1) in times_after.items():
        n0, s0 = times_before.get(k, (0, 0.0))
        if n1 > n0:
            out[k] = {"count": n1 - n0, "ms": (s1 - s0) * 1e3, "ms_per_call": (s1 - s0) * 1e3 / (n1 - n0)}
    return out


class Recorder:
    """snapshots of the twin's per-call totals at the loop marks"""

    def __init__(self, tw):
        self.tw, self.snap = tw, {}
        orig = tw.mark

        def mark(label):
            self.snap[label] = {k: tuple(v) for k, v in tw.times.items()}
            orig(label)

        tw.mark = mark


def device_rate(tw, ctx, target_s=0.4):
    """sw_step in one block on the driver's own context (its state advances)"""
    n = 8
    while True:
        tw.lib.sw_step(ctx, 2)  # warm
        t0 = time.perf_counter()
        rc = tw.lib.sw_step(ctx, n)
        dt = time.perf_counter() - t0
        if rc != 0:
            raise RuntimeError(f"sw_step: {tw.lib.sw_last_error(ctx).decode()}")
        if dt >= target_s or n >= 1 << 16:
            return n / dt, n
        n = int(min(1 << 16, max(2 * n, n * target_s / max(dt, 1e-4))))


def summarize(name, tw, rec, steps, ctx, params, start="frames", end="end"):
    t0, t1, _, _ = _loop_window(tw, start, end)
    wall = t1 - t0
    calls = _calls_between(tw, rec.snap[start], rec.snap[end])
    in_c = sum(c["ms"] for c in calls.values())
    dev, ndev = device_rate(tw, ctx)
    drv = steps / wall
    return {"driver": name, "params": params, "steps": steps, "loop_s": wall, "steps_per_s_driver": drv,
            "steps_per_s_device": dev, "device_block_steps": ndev, "driver_over_device": drv / dev,
            "gpu_idle_fraction": max(0.0, 1.0 - steps / (dev * wall)), "calls": calls, "c_calls_ms": in_c,
            "host_ms": wall * 1e3 - in_c, "host_ms_per_frame": None}


def run_rsw(frames):
    c = rsw_cadence()
    tw = R.Twin()
    tw.times, tw.marks = {}, []
    rec = Recorder(tw)
    nsteps = frames * c["output_freq"]
    prob, _, outputs, _, _ = R.rsw_driver_start(tw, nx=512, nsteps=nsteps, output_freq=c["output_freq"],
                                                 diags_freq=c["diags_freq"], spinup_step=0, T=np.float32)
    nfr = round(nsteps / c["output_freq"]) + 1
    out = summarize("RSWDriver 512^2 IFMAB3 (T=Float32)", tw, rec, nfr * c["output_freq"], prob.timestepper.ctx,
                    dict(c, frames=nfr, spinup_step=0, note="spinup_step = 0: every frame saves its snapshot"))
    out["host_ms_per_frame"] = out["host_ms"] / nfr
    return out


def run_qg2(frames, nx=2048):
    c = qg2_cadence(nx)
    tw = R.Twin()
    tw.times, tw.marks = {}, []
    rec = Recorder(tw)
    nsteps = frames * c["output_freq"]
    prob, _, _, _, _ = R.two_layer_driver_start(tw, nx=nx, nsteps=nsteps, output_freq=c["output_freq"],
                                                diags_freq=c["diags_freq"], spinup_step=0, T=np.float32)
    nfr = round(nsteps / c["output_freq"]) + 1
    out = summarize(f"TwoLayerDriver {nx}^2 IFMAB3 (T=Float32)", tw, rec, nfr * c["output_freq"],
                    prob.timestepper.ctx, dict(c, frames=nfr, spinup_step=0))
    out["host_ms_per_frame"] = out["host_ms"] / nfr
    return out


def run_mlqg(frames, nx=512, nsubs=50):
    tw = R.Twin()
    tw.times, tw.marks = {}, []
    rec = Recorder(tw)
    nsteps = frames * nsubs
    prob, _, _, _ = R.mlqg_simulation_start(tw, nx=nx, nsteps=nsteps, nsubs=nsubs, amplitude_scale=1.0)
    nfr = round(nsteps / nsubs) + 1
    out = summarize(f"TwoLayerSimulation {nx}^2 FilteredRK4 (Diagnostic freq = 1)", tw, rec, nfr * nsubs,
                    prob.timestepper.ctx, dict(nsubs=nsubs, frames=nfr, diag_freq=1, dt=float(prob.clock.dt)))
    out["host_ms_per_frame"] = out["host_ms"] / nfr
    return out


def run_ty(frames, nx=512, startup_nsubs=2000):
    """TYdriver's two phases: the start-up problem (one block of
    startup_nsubs steps; the driver's is 500000) and the main problem at
    nsubs = 1 (a step, enforce_reality_condition!, updatevars!, saveoutput per
    frame) — libsw's with LIBSW_CPU=1 (the reference's is Problem(CPU()))"""
    tw = R.Twin()
    tw.times, tw.marks = {}, []
    rec = Recorder(tw)
    prob, _, _, _, _, _, _ = R.ty_driver_start(tw, nx=nx, startup_nsteps=100, startup_nsubs=startup_nsubs,
                                               nsteps=frames, nsubs=1)
    main = summarize(f"TYdriver {nx}^2 ETDRK4 main phase (nsubs = 1)", tw, rec, frames + 1,
                     prob.timestepper.ctx, dict(nsubs=1, frames=frames + 1, dt=5e-3))
    main["host_ms_per_frame"] = main["host_ms"] / (frames + 1)
    t0, t1, _, _ = _loop_window(tw, "startup", "startup_end")
    calls = _calls_between(tw, rec.snap["startup"], rec.snap["startup_end"])
    su = {"driver": f"TYdriver {nx}^2 ETDRK4 start-up phase", "steps": startup_nsubs, "loop_s": t1 - t0,
          "steps_per_s_driver": startup_nsubs / (t1 - t0), "calls": calls,
          "params": dict(startup_nsubs=startup_nsubs, note="the driver's startup_nsubs is 500000: one block")}
    su["steps_per_s_device"] = None  # (the main phase's device rate: the same kernels)
    return [su, main]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", nargs="*", default=None, choices=["rsw", "qg2", "mlqg", "mlqg384", "ty"])
    args = ap.parse_args()
    todo = args.only or ["rsw", "qg2", "mlqg", "ty"]
    res = []
    for name in todo:
        t0 = time.perf_counter()
        if name == "rsw":
            r = [run_rsw(args.frames)]
        elif name == "qg2":
            r = [run_qg2(max(4, args.frames // 4))]
        elif name == "mlqg":
            r = [run_mlqg(max(4, args.frames // 2))]
        elif name == "mlqg384":  # simulation/MattParameters.jl's grid (the generic engine)
            r = [run_mlqg(max(4, args.frames // 2), nx=384)]
        else:
            r = run_ty(4 * args.frames)
        for x in r:
            print(f"[cadence] {x['driver']}: driver {x['steps_per_s_driver']:.0f} steps/s"
                  + (f", device {x['steps_per_s_device']:.0f} ({x['driver_over_device']:.2f}),"
                     f" GPU idle {x['gpu_idle_fraction']:.2f}, host {x['host_ms_per_frame']:.3f} ms/frame"
                     if x.get("steps_per_s_device") else "") + f"  [{time.perf_counter() - t0:.1f} s]",
                  file=sys.stderr, flush=True)
        res.extend(r)
    js = json.dumps({"drivers": res}, indent=1)
    if args.out:
        open(args.out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
