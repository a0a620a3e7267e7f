#!/bin/bash
# On the GPU box (round 6): the drivers' 512-point split rows (RSW, Thomas–
# Yamada) with the live band at compile time (b_kc9.so) against the runtime
# band (a_base9.so, SW_ROW_KC_SHORT=0); 512-only builds.
set -o pipefail
O=gpurun_out/rowkc9; mkdir -p $O
for so in sweep_var/*.so; do
  for c in "20 512 rsw IFMAB3" "8 512 ty ETDRK4"; do
    LIBSW_PATH=$PWD/$so timeout -k 10 200 python tools/state_hash.py $c >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  for cfg in "rsw 512 IFMAB3 8000" "ty 512 ETDRK4 2000"; do
    set -- $cfg
    LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps $4 --warmup 200 --model $1 --grid $2 --stepper $3 > $O/$n.$1.$r.json 2> $O/$n.$1.$r.err \
      || { echo "$n failed"; exit 3; }
    echo "r$r $n $1$2 $(python -c "import json; d=json.load(open('$O/$n.$1.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
