#!/bin/bash
# On the GPU box (round 6): MultiLayerQG's 512-point split rows with kc = nx/2
# at compile time (b_mlqgkc.so) against the runtime band (a_mlqg.so); 512-only.
set -o pipefail
O=gpurun_out/rowkc_mlqg; mkdir -p $O
for so in sweep_var/*.so; do
  LIBSW_PATH=$PWD/$so timeout -k 10 200 python tools/state_hash.py 6 512 mlqg FilteredRK4 >> $O/hash.txt 2>> $O/hash.err || exit 1
done
cat $O/hash.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
    --no-box-state --steps 2000 --warmup 200 --model mlqg --grid 512 > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; exit 3; }
  echo "r$r $n $(python -c "import json; d=json.load(open('$O/$n.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
