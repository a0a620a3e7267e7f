#!/bin/bash
# Round-6 GPU check (one box): the given GPU tests, smoke(), the driver-like
# headline line (20 steps, as the round-end bench), the default line, the
# driver-cadence table, then an interleaved A/B of sweep_var/*.so.
# usage: bash tools/ab/r6_check.sh TAG "pytest -k expr" [AB_ROUNDS] [AB_CHECK_EXPR]
set -o pipefail
TAG=$1; K=$2; R=${3:-0}; AK=$4
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.txt 2>&1
  rc=$?; tail -2 $O/gpu_tests.txt
  [ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; exit 1; }
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 2; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driverlike.json 2> $O/bench_driverlike.err || { tail $O/bench_driverlike.err; exit 3; }
python -c "import json; b=json.load(open('$O/bench_driverlike.json')); print('driverlike', round(b['value'],1), round(b['roofline']['frac'],3), b['kernels'], b['box']['per_rank'][0]['regions']['headline'].get('samples'), b['box']['per_rank'][0]['regions']['headline'].get('throttle_fraction'))"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 4; }
python -c "import json; b=json.load(open('$O/bench_default.json')); print('default', round(b['value'],1), round(b['roofline']['frac'],3), [(k['name'], round(k['avg_us'],1)) for k in b['kernels']], round(b['config5']['value'],2), round(b['config4']['value'],1))"
timeout -k 10 600 python tools/driver_cadence.py --out $O/driver_cadence.json > /dev/null 2> $O/driver_cadence.err || { tail $O/driver_cadence.err; exit 5; }
grep cadence $O/driver_cadence.err
if [ "$R" -gt 0 ]; then
  if [ -n "$AK" ]; then bash tools/ab/ab.sh --check "$AK" $R || exit 6; else bash tools/ab/ab.sh $R || exit 6; fi
  cp -r gpurun_out/ab $O/ab
fi
echo done
