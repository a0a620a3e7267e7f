#!/bin/bash
# On the GPU box (round 4): decimated column transforms (SW_COL_DEC_MIN) —
# interleaved benches of sweep_var/c14.so (natural-order Stockham columns),
# c12.so (decimated from 4096: the default) and c11.so (from 2048) on
# config 5, config 4, the 2048² metric and 2LQG 2048² IFMAB3.
# usage: bash tools/ab/ab_r4_coldec.sh [R]
mkdir -p gpurun_out/ab
R=${1:-2}
run() {  # variant tag model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 \
    > gpurun_out/ab/$1_$2.$r.json 2> gpurun_out/ab/$1_$2.$r.err \
    || { echo "$1 $2 failed"; tail -5 gpurun_out/ab/$1_$2.$r.err; exit 1; }
  echo "r$r $1 $2 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1_$2.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in $(seq $R); do
  for v in c14 c12; do run $v c5 qg2 8192 IFMRK4 12 3 || exit 1; done
  for v in c14 c12; do run $v c4 rsw 4096 FilteredAB3 100 20 || exit 1; done
  for v in c14 c11; do run $v m rsw 2048 FilteredAB3 1000 200 || exit 1; done
  for v in c14 c11; do run $v q3 qg2 2048 IFMAB3 1000 200 || exit 1; done
done
