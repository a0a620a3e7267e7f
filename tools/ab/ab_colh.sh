#!/bin/bash
# On the GPU box: the half-length 2LQG col_inv (k_col_inv_qg_h) at 8192:
# 8192-length parity with the all-length build, then config 5 interleaved
mkdir -p gpurun_out/colh
LIBSW_PATH=$PWD/sweep_var/allc.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_pins.py tests/test_gpu_slabs.py -k "qg2 or mlqg or lengths or large" \
  > gpurun_out/colh/test.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/colh/test.log; exit 1; }
echo "allc tests: $(tail -1 gpurun_out/colh/test.log)"
for r in 1 2; do for v in c13 c13h; do
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 \
    --model qg2 --grid 8192 --stepper IFMRK4 --steps 12 --warmup 3 > gpurun_out/colh/$v.json 2> gpurun_out/colh/$v.err \
    || { echo "$v failed"; tail -3 gpurun_out/colh/$v.err; exit 1; }
  echo "r$r $v $(python -c "import json; d=json.load(open('gpurun_out/colh/$v.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
