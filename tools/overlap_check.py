"""Time the slab-decomposed step on ONE GPU with every slab held in-process
(local_slabs == nranks: the transposes are device copies with the RCCL block
pattern), pipelined (side-stream transposes overlapped with the column groups)
against the sequential schedule (SW_OVERLAP=0).

    python tools/overlap_check.py [--n 2048] [--P 2 4] [--steps 50]

Prints one JSON line per (model, P, schedule).  The copies share the GPU's
HBM with the kernels, so this measures that the schedule overlaps, not the
xGMI cost of a multi-GPU run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(model, n, P, overlap, steps, warmup):
    from juliaraytracingsw_amd import drivers

    os.environ["SW_OVERLAP"] = "1" if overlap else "0"
    dec = dict(nranks=P, local_slabs=P) if P > 1 else None
    if model == "rsw":
        prob, _ = drivers.rsw_problem(n, "FilteredAB3", decomposition=dec)
    elif model == "qg2":
        prob, _ = drivers.qg2_problem(n, "IFMAB3", decomposition=dec)
    else:
        prob, _ = drivers.ty_problem(n, decomposition=dec)
    prob.stepforward(warmup)
    t0 = time.perf_counter()
    prob.stepforward(steps)
    dt = time.perf_counter() - t0
    prob.close()
    os.environ.pop("SW_OVERLAP", None)
    return steps / dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--P", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--models", nargs="+", default=["rsw", "qg2"])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    for m in a.models:
        base = run(m, a.n, 1, True, a.steps, a.warmup)
        print(json.dumps(dict(model=m, n=a.n, P=1, steps_per_s=base)), flush=True)
        for P in a.P:
            for ov in (False, True):
                v = run(m, a.n, P, ov, a.steps, a.warmup)
                print(json.dumps(dict(model=m, n=a.n, P=P, schedule="pipelined" if ov else "sequential",
                                      steps_per_s=v)), flush=True)


if __name__ == "__main__":
    main()
