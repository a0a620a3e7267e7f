"""Per-kernel HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE collected in separate runs), with the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of wide coalesced
reads (x2); WRITE_SIZE is exact for 16-B stores.  Both counters are in KB.

    python tools/traffic_from_pmc.py FETCH.csv WRITE.csv CONFIG OUT.json
"""
import csv
import json
import sys
from collections import defaultdict

SHORT = {"k_row": "row", "k_row_qg_h": "row", "k_row_rsw_h": "row", "k_col_step_fab3_rsw": "col_step", "k_col_step": "col_step",
         "k_col_inv": "col_inv", "k_col_fwd": "col_fwd", "k_step_elem": "update"}


def short(name):
    full = name.replace("void ", "").split("(")[0].replace("sw::", "")
    base = full.split("<")[0]
    targs = [a.strip() for a in full[len(base) + 1:].rstrip(">").split(",")] if "<" in full else []
    if base == "k_col_step" and len(targs) > 3 and targs[3] == "false":  # k_col_step<M, L, OP, INV = false, …>
        return "col_fwd_step"
    return SHORT.get(base, base)


def means(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fetch_csv, write_csv, config, out):
    f = means(fetch_csv, "FETCH_SIZE")
    w = means(write_csv, "WRITE_SIZE")
    kern = {k: 2 * f.get(k, 0.0) + w.get(k, 0.0) for k in set(f) | set(w)}
    json.dump({"config": config, "unit": "bytes/launch", "correction": "2*FETCH_SIZE + WRITE_SIZE",
               "kernels": kern, "fetch_bytes": {k: 2 * v for k, v in f.items()}, "write_bytes": w},
              open(out, "w"), indent=1)
    print(json.dumps(kern, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
