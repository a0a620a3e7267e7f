"""Markdown table of SQ counters per kernel from tools/pmc_summary.py output
(tools/ab/r6_sq.sh: two --pmc passes, 8 SQ counters each).

Per kernel (means over launches): waves per launch, instructions per wave
(VALU, LDS, SALU, VMEM read/write) and the split of SQ_WAVE_CYCLES into
issuing (ACTIVE_INST_ANY), parked on s_waitcnt/barrier (WAIT_ANY) and
issue-stalled (WAIT_INST_ANY, of which LDS-issue WAIT_INST_LDS); the three
are disjoint and sum to WAVE_CYCLES (MI355X_MICROARCH.md, PMC table).
LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

usage: python tools/sq_table.py [--min-share 0.05] pmc_sq_<config>.txt ...
"""
import argparse
import os
import re


def parse(path):
    out, k = {}, None
    for line in open(path):
        if not line.startswith(" ") and line.strip():
            k = line.strip()
            out[k] = {}
        else:
            m = re.match(r"\s+(\S+)\s+(\S+)\s+\(n=(\d+)\)", line)
            if m and k:
                out[k][m.group(1)] = float(m.group(2))
                out[k].setdefault("n", int(m.group(3)))
    return out


SETUP = ("k_gather", "k_make_spec", "k_scatter", "__amd_rocclr")  # set_state / IC kernels, not the step


def rows(path, min_share):
    d = {k: v for k, v in parse(path).items() if "SQ_WAVE_CYCLES" in v and "SQ_WAVES" in v and v["SQ_WAVES"] > 0
         and not any(s in k for s in SETUP)}
    cyc = lambda v: v["SQ_WAVE_CYCLES"] * v["n"]  # over all launches of the profiled run
    tot = sum(cyc(v) for v in d.values())
    cfg = os.path.basename(path).replace("pmc_sq_", "").replace(".txt", "")
    for k, v in sorted(d.items(), key=lambda kv: -cyc(kv[1])):
        if cyc(v) < min_share * tot:
            continue
        w, wc = v["SQ_WAVES"], v["SQ_WAVE_CYCLES"]
        pw = lambda c: v.get(c, 0.0) / w
        pc = lambda c: 100.0 * v.get(c, 0.0) / wc
        conf = 100.0 * v.get("SQ_LDS_BANK_CONFLICT", 0) / max(v.get("SQ_LDS_IDX_ACTIVE", 0), 1)
        yield (f"| {cfg} | `{k.replace('sw::', '')}` | {100 * cyc(v) / tot:.0f} | {w:.0f} | {pw('SQ_INSTS_VALU'):.0f} | {pw('SQ_INSTS_LDS'):.0f} | "
               f"{pw('SQ_INSTS_SALU'):.0f} | {pw('SQ_INSTS_VMEM_RD'):.0f} / {pw('SQ_INSTS_VMEM_WR'):.0f} | "
               f"{pc('SQ_ACTIVE_INST_ANY'):.0f} | {pc('SQ_WAIT_ANY'):.0f} | {pc('SQ_WAIT_INST_ANY'):.0f} "
               f"({pc('SQ_WAIT_INST_LDS'):.0f}) | {conf:.1f} |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-share", type=float, default=0.05, help="skip kernels below this share of wave cycles")
    ap.add_argument("files", nargs="+")
    a = ap.parse_args()
    print("| config | kernel | share of wave cycles % | waves | VALU/wave | LDS/wave | SALU/wave | VMEM rd / wr per wave | issuing % | "
          "parked % | issue-stall % (LDS) | LDS conflict % |")
    print("|---|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for f in a.files:
        for r in rows(f, a.min_share):
            print(r)


if __name__ == "__main__":
    main()
