"""Do two independent RSW 2048² FilteredAB3 problems, stepped at once from
two host threads (each context on its own HIP stream), overlap on one GPU?

A row pass is issue-bound (SQ counters) and the fused column
step HBM-bound; if kernels of the two streams share the CUs, the pair's
aggregate rate exceeds one problem's.  That decides whether a one-problem
schedule running a row part beside a column-step part (two streams) can pay.

usage: python tools/micro/concurrency_probe.py [--n 2048] [--steps 400] [--k 2]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--block", type=int, default=20)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--stepper", default="FilteredAB3")
    a = ap.parse_args()
    from juliaraytracingsw_amd import drivers

    probs = [drivers.rsw_problem(a.n, a.stepper, seed=100 + i)[0] for i in range(a.k)]
    for p in probs:
        p.stepforward(50)

    def run(p, steps):
        for _ in range(steps // a.block):
            p.stepforward(a.block)

    out = {"n": a.n, "stepper": a.stepper, "steps": a.steps, "block": a.block}
    for rep in range(3):
        t0 = time.perf_counter()
        run(probs[0], a.steps)
        t1 = time.perf_counter()
        out.setdefault("one_steps_per_s", []).append(a.steps / (t1 - t0))
        th = [threading.Thread(target=run, args=(p, a.steps)) for p in probs]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        t1 = time.perf_counter()
        out.setdefault(f"k{a.k}_aggregate_steps_per_s", []).append(a.k * a.steps / (t1 - t0))
    for p in probs:
        p.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
