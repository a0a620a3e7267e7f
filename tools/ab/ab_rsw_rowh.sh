#!/bin/bash
# On the GPU box: the half-length RSW row (k_row_rsw_h) against k_row.
# Parity first with the all-length build (sweep_var/rall.so), then interleaved
# benches of the --len builds r11*/r12*/r13* (RSW FilteredAB3 2048²/4096²/8192²).
# usage: bash tools/ab/ab_rsw_rowh.sh [R]
mkdir -p gpurun_out/ab
R=${1:-2}
LIBSW_PATH=$PWD/sweep_var/rall.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_slabs.py -k "rsw or lengths" \
  > gpurun_out/ab/rall.test.log 2>&1 || { echo "rall TESTS FAILED"; tail -30 gpurun_out/ab/rall.test.log; exit 1; }
echo "rall tests: $(tail -1 gpurun_out/ab/rall.test.log)"
run() {  # name grid steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 \
    --model rsw --grid $2 --stepper FilteredAB3 --steps $3 --warmup $4 > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err \
    || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in $(seq $R); do
  for v in r11h r11h3 r11f; do run $v 2048 2000 200 || exit 1; done
  for v in r12h r12f; do run $v 4096 400 40 || exit 1; done
  for v in r13h r13f; do run $v 8192 60 10 || exit 1; done
done
