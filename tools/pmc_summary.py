"""Summarise rocprofv3 counter_collection.csv files: mean counter value per kernel."""
import csv
import glob
import sys
from collections import defaultdict

def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "")
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        print(k)
        for c, v in sorted(acc[k].items()):
            print(f"   {c:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")

if __name__ == "__main__":
    main(sys.argv[1:] or glob.glob("gpurun_out/pmc*/**/*counter_collection.csv", recursive=True))
