#!/bin/bash
# Round 4: rocprofv3 kernel trace + stats of the default bench command itself
# (the bench line's roofline kernel average must agree with its rocprof average)
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --no-cpu-baseline \
  > $O/bench_traced.json 2> $O/bench_traced.err || exit 1
cp $(find $O/trace -name '*kernel_stats.csv') $O/kernel_stats_bench.csv || exit 2
rm -rf $O/trace
python -c "import json; d=json.load(open('$O/bench_traced.json')); print(round(d['value'],1), d['roofline']['avg_us_per_launch'], d['roofline']['frac'])"
head -4 $O/kernel_stats_bench.csv
