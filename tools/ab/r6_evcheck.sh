#!/bin/bash
# bench.py's per-kernel event averages against the kernel trace of the same
# command (deferred event reads, round 6): the headline configuration
# untraced and under rocprofv3 --kernel-trace --stats.  usage: bash tools/ab/r6_evcheck.sh TAG
set -o pipefail
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-config5 --no-config4"
timeout -k 10 300 $B > $O/bench_plain.json 2> $O/bench_plain.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/bench_traced.json 2> $O/bench_traced.err || exit 2
cp $(find $O/trace -name '*kernel_stats.csv') $O/kernel_stats_bench.csv || exit 3
rm -rf $O/trace
python - <<PY
import csv, json
for f in ("$O/bench_plain.json", "$O/bench_traced.json"):
    b = json.load(open(f)); print(f, round(b["value"], 1), [(k["name"], round(k["avg_us"], 2)) for k in b["kernels"]])
for r in csv.DictReader(open("$O/kernel_stats_bench.csv")):
    if float(r["Percentage"]) > 2: print(r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
