#!/bin/bash
# On the GPU box: short bench of every sweep_var/*.so (per-kernel HIP-event times).
# usage: bash tools/ab/sweep.sh [--check] [extra bench args]
#   --check: first run the RSW FilteredAB3 parity/slab GPU tests against each variant
mkdir -p gpurun_out/sweep
CHECK=0
if [ "$1" = "--check" ]; then CHECK=1; shift; fi
for so in sweep_var/*.so; do
  n=$(basename $so .so)
  if [ $CHECK = 1 ]; then
    LIBSW_PATH=$PWD/$so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py -q -x -k "rsw_fab3" \
      > gpurun_out/sweep/$n.test.log 2>&1 || { echo "$n TESTS FAILED"; tail -5 gpurun_out/sweep/$n.test.log; exit 1; }
  fi
  SW_CHECK_NAN=${SW_CHECK_NAN:-1} LIBSW_PATH=$PWD/$so timeout -k 10 120 python bench.py --no-cpu-baseline --no-config5 --no-config4 --steps 100 --warmup 10 "$@" \
    > gpurun_out/sweep/$n.json 2> gpurun_out/sweep/$n.err || { echo "$n failed rc=$?"; exit 1; }
  echo "$n $(python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$n.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done
