#!/bin/bash
# Round 4 closing GPU check at HEAD: the whole GPU suite, smoke, the default bench line.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
cat $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 3
python -c "import json; d=json.load(open('$O/bench_default.json')); print(round(d['value'],1), d['roofline']['frac'], [(k['name'], round(k['avg_us'],1)) for k in d['kernels']], d['config5']['value'], d['config4']['value'])"
