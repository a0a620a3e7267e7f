#!/bin/bash
# On the GPU box (round 6): the 2LQG 2048 row with the live band and one slab
# at compile time (SW_ROW_KC_QG=1) against the default (2048-only builds).
set -o pipefail
O=gpurun_out/qgkc; mkdir -p $O
for so in sweep_var/*.so; do
  LIBSW_PATH=$PWD/$so timeout -k 10 200 python tools/state_hash.py 6 2048 qg2 IFMAB3 >> $O/hash.txt 2>> $O/hash.err || exit 1
done
cat $O/hash.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
    --no-box-state --steps 2000 --warmup 100 --model qg2 --grid 2048 --stepper IFMAB3 > $O/$n.$r.json 2> $O/$n.$r.err || exit 3
  echo "r$r $n $(python -c "import json; d=json.load(open('$O/$n.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
