"""Minimal stepping driver for rocprofv3 runs (no torch):
    python tools/prof_step.py [--model rsw] [--stepper FilteredAB3] [--n 2048] [--steps 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from juliaraytracingsw_amd import drivers  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="rsw")
ap.add_argument("--stepper", default="FilteredAB3")
ap.add_argument("--grid", dest="n", type=int, default=2048)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
a = ap.parse_args()
if a.model == "ty":
    prob, _ = drivers.ty_problem(a.n)
elif a.model == "mlqg":
    prob, _ = drivers.mlqg_problem(a.n)
else:
    mk = drivers.rsw_problem if a.model == "rsw" else drivers.qg2_problem
    prob, _ = mk(a.n, a.stepper)
prob.stepforward(a.warmup)
prob.stepforward(a.steps)
print("done", prob.clock.step)
