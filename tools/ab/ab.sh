#!/bin/bash
# On the GPU box: A/B of sweep_var/*.so — optional GPU parity tests per
# variant, then R rounds of the default bench (variants interleaved per round,
# so box drift hits all alike).  usage: bash tools/ab/ab.sh [--check "pytest -k expr"] [R] [extra bench args]
mkdir -p gpurun_out/ab
CHECK=""
if [ "$1" = "--check" ]; then CHECK=$2; shift 2; fi
R=${1:-2}; shift
if [ -n "$CHECK" ]; then
  for so in sweep_var/*.so; do n=$(basename $so .so)
    LIBSW_PATH=$PWD/$so timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py -q -x \
      --timeout 300 --timeout-method thread -k "$CHECK" > gpurun_out/ab/$n.test.log 2>&1 \
      || { echo "$n TESTS FAILED"; tail -5 gpurun_out/ab/$n.test.log; exit 1; }
    echo "$n tests: $(tail -1 gpurun_out/ab/$n.test.log)"
  done
fi
for r in $(seq $R); do for so in sweep_var/*.so; do n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --steps 2000 --warmup 200 "$@" \
    > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.$r.err || { echo "$n failed"; exit 1; }
  echo "r$r $n $(python -c "import json; d=json.load(open('gpurun_out/ab/$n.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
