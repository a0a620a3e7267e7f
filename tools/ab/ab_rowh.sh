#!/bin/bash
# On the GPU box: the half-length 2LQG row (k_row_qg_h) against the
# full-length pair row, interleaved: config 5 (8192² IFMRK4, --len 13
# builds h13/f13) and config 3 (2048² IFMAB3, --len 11 builds h11/f11).
# usage: bash tools/ab/ab_rowh.sh [R]
mkdir -p gpurun_out/ab
R=${1:-2}
run() {  # name grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 \
    --model qg2 --grid $2 --stepper $3 --steps $4 --warmup $5 > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err \
    || { echo "$1 failed"; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in $(seq $R); do
  for v in h13 f13; do run $v 8192 IFMRK4 12 3 || exit 1; done
  for v in h11 f11; do run $v 2048 IFMAB3 2000 200 || exit 1; done
done
