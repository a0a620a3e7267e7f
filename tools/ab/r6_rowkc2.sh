#!/bin/bash
# On the GPU box (round 6): the full-length rows with the live band at compile
# time (sweep_var/b_rowkc.so) against HEAD (a_base.so): bitwise hashes (RSW
# 2048², 1024², config 3), the 2048/1024 parity + slab tests on the variant,
# interleaved benches of the headline, config 3 and RSW 1024².
set -o pipefail
O=gpurun_out/rowkc2; mkdir -p $O
for so in sweep_var/*.so; do
  for c in "10 2048 rsw FilteredAB3" "10 1024 rsw FilteredAB3" "6 2048 qg2 IFMAB3"; do
    LIBSW_PATH=$PWD/$so timeout -k 10 200 python tools/state_hash.py $c >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
LIBSW_PATH=$PWD/sweep_var/b_rowkc.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py \
  -x -q --timeout 300 --timeout-method thread -k "2048 or 1024" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 2; }
tail -1 $O/tests.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  for cfg in "rsw 2048 FilteredAB3" "qg2 2048 IFMAB3" "rsw 1024 FilteredAB3 --nutune 2.5 --cfltune 0.005"; do
    set -- $cfg
    LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps 2000 --warmup 100 --model $1 --grid $2 --stepper $3 ${@:4} > $O/$n.$1$2.$r.json 2> $O/$n.$1$2.$r.err \
      || { echo "$n failed"; exit 3; }
    echo "r$r $n $1$2 $(python -c "import json; d=json.load(open('$O/$n.$1$2.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
