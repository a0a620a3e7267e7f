"""Per-kernel averages over the timed region of a tools/prof_step.py run
under `rocprofv3 --kernel-trace`: the last steps × launches_per_step libsw
step kernels before the final NaN check.  Compares the kernel sum per step
with the run's own ms/step.

    python tools/trace_summary.py KERNEL_TRACE.csv PROF_STEP.json OUT.json
"""
import csv
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from traffic_from_pmc import short  # noqa: E402

STEP_KERNELS = {"row", "col_step", "col_inv", "col_fwd", "update", "col_fwd_step"}
# the generic engine's fused stage (csrc/sw_generic.hip): three kernels per
# FilteredRK4 stage, four stages per step (libsw's profile counts one
# "generic_step" launch per step)
GEN_KERNELS = {"gen::k_gcol_inv", "gen::k_grow", "gen::k_gcol_fwd"}


def main(trace_csv, run_json, out):
    run = json.loads([ln for ln in open(run_json) if ln.startswith("{")][-1])
    allrows = list(csv.DictReader(open(trace_csv)))
    rows = [r for r in allrows if short(r["Kernel_Name"]) in STEP_KERNELS]
    per_step = run["launches_per_step"]
    if not rows:
        rows = [r for r in allrows if short(r["Kernel_Name"]) in GEN_KERNELS]
        per_step = 3 * 4
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = int(round(run["steps"] * per_step))
    sel = rows[-n:]
    dur = defaultdict(list)
    for r in sel:
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    kern = {k: {"avg_us": sum(v) / len(v), "per_step": len(v) / run["steps"]} for k, v in dur.items()}
    ksum = sum(k["avg_us"] * k["per_step"] for k in kern.values())
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) * 1e-3 / run["steps"]
    res = {"config": run["config"], "steps": run["steps"], "warmup_steps": run["warmup_steps"],
           "kernels": kern, "kernel_sum_us_per_step": ksum, "trace_span_us_per_step": span,
           "run_ms_per_step_traced": run["ms_per_step"], "kernel_sum_vs_run": ksum / (run["ms_per_step"] * 1e3)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
