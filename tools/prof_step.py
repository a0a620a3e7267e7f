"""Stepping driver for rocprofv3 runs (no torch), warm like bench.py:
    python tools/prof_step.py [--model rsw] [--stepper FilteredAB3] [--grid 2048] [--steps 200] [--warmup 20]

After `--warmup` steps, untimed steps continue until `--min-warmup-s` of
stepping has run (bench.py's steady state), then libsw's own per-kernel
profile of 2 steps gives the kernel launches per step, then `--steps` timed
steps.  Prints one JSON line (steps/s of the timed region and launches per
step) that tools/trace_summary.py reads to pick the timed region's
dispatches out of the kernel trace."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from juliaraytracingsw_amd import drivers  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="rsw")
ap.add_argument("--stepper", default="FilteredAB3")
ap.add_argument("--grid", dest="n", type=int, default=2048)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=20)
ap.add_argument("--min-warmup-s", type=float, default=0.2)
ap.add_argument("--nutune", type=float, default=None)
ap.add_argument("--cfltune", type=float, default=None)
a = ap.parse_args()
if a.model == "ty":
    prob, _ = drivers.ty_problem(a.n)
elif a.model == "mlqg":
    prob, _ = drivers.mlqg_problem(a.n)
elif a.model == "rsw":
    over = {k: v for k, v in (("nutune", a.nutune), ("cfltune", a.cfltune)) if v is not None}
    prob, _ = drivers.rsw_problem(a.n, a.stepper, **over)
else:
    prob, _ = drivers.qg2_problem(a.n, a.stepper)
t0 = time.perf_counter()
prob.stepforward(a.warmup)
dt = time.perf_counter() - t0
extra = 0
if dt < a.min_warmup_s:
    extra = int((a.min_warmup_s - dt) / max(dt / max(a.warmup, 1), 1e-6)) + 1
    prob.stepforward(extra)
stats = prob.ctx.profile(2)
lps = sum(s["launches"] for s in stats if s["name"] != "transpose") / 2
t0 = time.perf_counter()
prob.stepforward(a.steps)  # returns when the stream is drained (one NaN check at the end)
el = time.perf_counter() - t0
print(json.dumps({"config": f"{a.model}{a.n}_{a.stepper}", "steps": a.steps, "warmup_steps": a.warmup + extra,
                  "launches_per_step": lps, "ms_per_step": el / a.steps * 1e3, "steps_per_s": a.steps / el}))
