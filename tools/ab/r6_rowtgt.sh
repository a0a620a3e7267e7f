#!/bin/bash
# On the GPU box (round 6): threads per block of the RSW row on 512-point
# lines (SW_RSW_ROW_TGT_SHORT 256 / 128 / 64; 512-only builds): bitwise hashes,
# then interleaved RSWDriver 512² IFMAB3 benches.
set -o pipefail
O=gpurun_out/rowtgt; mkdir -p $O
for so in sweep_var/*.so; do
  LIBSW_PATH=$PWD/$so timeout -k 10 120 python tools/state_hash.py 20 512 rsw IFMAB3 >> $O/hash.txt 2>> $O/hash.err || exit 1
done
cat $O/hash.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
    --no-box-state --steps 8000 --warmup 400 --grid 512 --stepper IFMAB3 > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; exit 2; }
  echo "r$r $n $(python -c "import json; d=json.load(open('$O/$n.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
