#!/bin/bash
# On the GPU box (round 6, experiment): the column kernels with their live-row
# band at compile time (b_band1.so: the 2/3 rule, RSW / TY; c_band2.so:
# aliased_fraction = 0, MultiLayerQG) against a_base.so; 512-only builds.
set -o pipefail
O=gpurun_out/band; mkdir -p $O
for c in "a_base 20 512 rsw IFMAB3" "b_band1 20 512 rsw IFMAB3" "a_base 8 512 ty ETDRK4" "b_band1 8 512 ty ETDRK4" \
         "a_base 6 512 mlqg FilteredRK4" "c_band2 6 512 mlqg FilteredRK4"; do
  set -- $c
  LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 200 python tools/state_hash.py ${@:2} >> $O/hash.txt 2>> $O/hash.err || exit 1
done
cat $O/hash.txt
for r in 1 2 3; do
  for c in "a_base rsw 512 IFMAB3 8000" "b_band1 rsw 512 IFMAB3 8000" "a_base ty 512 ETDRK4 2000" "b_band1 ty 512 ETDRK4 2000" \
           "a_base mlqg 512 FilteredRK4 2000" "c_band2 mlqg 512 FilteredRK4 2000"; do
    set -- $c
    LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps $5 --warmup 200 --model $2 --grid $3 --stepper $4 > $O/$1.$2.$r.json 2> $O/$1.$2.$r.err \
      || { echo "$1 failed"; exit 3; }
    echo "r$r $1 $2 $(python -c "import json; d=json.load(open('$O/$1.$2.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done
