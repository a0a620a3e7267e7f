#!/bin/bash
# Round 4 GPU check after the RSW row's forward-pair change: the whole GPU
# suite, smoke, the default bench line, its rocprofv3 kernel trace, then the
# warm profiles of the two configurations whose kernels changed (RSW 2048²,
# 1024²; tools/profile_round.sh r04g).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
cat $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 3
python -c "import json; d=json.load(open('$O/bench_default.json')); print(round(d['value'],1), d['roofline']['frac'], [(k['name'], round(k['avg_us'],1)) for k in d['kernels']], d['config5']['value'], d['config4']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --no-cpu-baseline \
  > $O/bench_traced.json 2> $O/bench_traced.err || exit 4
cp $(find $O/trace -name '*kernel_stats.csv') $O/kernel_stats_bench.csv || exit 5
rm -rf $O/trace
python -c "import json; d=json.load(open('$O/bench_traced.json')); print('traced', round(d['value'],1), d['roofline']['avg_us_per_launch'], d['roofline']['frac'])"
head -3 $O/kernel_stats_bench.csv
timeout -k 10 900 bash tools/profile_round.sh r04g "rsw:2048:FilteredAB3:400:2000 rsw:1024:FilteredAB3:800:4000:2.5:0.005" || exit 6
