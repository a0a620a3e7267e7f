#!/bin/bash
# Round 4 final GPU check at HEAD: the whole GPU suite, smoke, the default
# bench line, then the warm profile of every BASELINE configuration
# (tools/profile_round.sh r04f).
set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04f/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r04f/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04f/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f/smoke.txt 2>&1 || exit 2
cat gpurun_out/r04f/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r04f/bench_default.json 2> gpurun_out/r04f/bench_default.err || exit 3
python -c "import json; d=json.load(open('gpurun_out/r04f/bench_default.json')); print(round(d['value'],1), d['roofline']['frac'], [(k['name'], round(k['avg_us'],1)) for k in d['kernels']], d['config5']['value'], d['config4']['value'])"
timeout -k 10 1500 bash tools/profile_round.sh r04f || exit 4
