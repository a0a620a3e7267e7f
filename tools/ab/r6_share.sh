#!/bin/bash
# On the GPU box (round 6): stage-twiddle powers shared across the RSW row's
# transforms (SW_ROW_TW_SHARE=1, room left by the pipelined wave-local pairs)
# against the default: bitwise hash at 2048², interleaved RSW 2048² benches.
set -o pipefail
O=gpurun_out/share; mkdir -p $O
for so in sweep_var/*.so; do
  LIBSW_PATH=$PWD/$so timeout -k 10 120 python tools/state_hash.py 10 2048 >> $O/hash.txt 2>> $O/hash.err || exit 1
done
cat $O/hash.txt
for r in 1 2 3 4; do for so in sweep_var/*.so; do n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
    --no-box-state --steps 2000 --warmup 100 > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; exit 3; }
  echo "r$r $n $(python -c "import json; d=json.load(open('$O/$n.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
