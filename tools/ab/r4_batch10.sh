#!/bin/bash
# Round 4 GPU batch 10: config-5 column passes with the first resident round
# half delayed (SW_COL_DESYNC = 0 / 3 / 6 sleeps of 127 × 64 cycles).
mkdir -p gpurun_out/ab
run() {  # tag so
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model qg2 --grid 8192 --stepper IFMRK4 --steps 12 --warmup 3 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do for v in q13ds0 q13ds3 q13ds6; do run $v $v || exit 1; done; done
