"""DESIGN.md's numbers table from a round's profile directory
(tools/profile_round.sh outputs copied to profiles/rNN/): per configuration
the bench line's steps/s and, per kernel, the HIP-event average (bench.py),
the rocprofv3 warm average (trace_summary.py), the algorithmic bytes per
launch, their rate against 8 TB/s, and the PMC bytes per launch
(2·FETCH_SIZE + WRITE_SIZE, traffic_from_pmc.py) over the algorithmic bytes.

usage: python tools/numbers_table.py profiles/r06
"""
import glob
import json
import os
import sys

PEAK = 8000.0  # GB/s (MI355X_MICROARCH.md)


def main(d):
    print("| config | steps/s | kernel | per step | µs (events) | µs (rocprof) | alg MB / launch | GB/s | of 8 TB/s "
          "| PMC MB / launch | PMC / alg |")
    print("|---|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for bf in sorted(glob.glob(os.path.join(d, "bench_*_*.json"))):
        tag = os.path.basename(bf)[len("bench_"):-len(".json")]
        wf, tf = os.path.join(d, f"warm_{tag}.json"), os.path.join(d, f"traffic_{tag}.json")
        if not (os.path.exists(wf) and os.path.exists(tf)):
            continue
        b, w, t = json.load(open(bf)), json.load(open(wf)), json.load(open(tf))
        first = True
        for k in sorted(b["kernels"], key=lambda k: -k["avg_us"] * k["per_step"]):
            name, us, ab = k["name"], k["avg_us"], k["alg_bytes"]
            wk = w["kernels"].get(name, {}).get("avg_us")
            tr = t["kernels"].get(name)
            gbs = ab / us / 1e3
            head = f"| {tag} | {b['value']:.1f} " if first else "| | "
            print(head + f"| {name} | {k['per_step']:g} | {us:.1f} | {'' if wk is None else f'{wk:.1f}'} | {ab / 1e6:.1f} "
                  f"| {gbs:.0f} | {gbs / PEAK:.2f} | {'' if tr is None else f'{tr / 1e6:.1f}'} "
                  f"| {'' if tr is None else f'{tr / ab:.2f}'} |")
            first = False


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/r06")
