#!/bin/bash
# On the GPU box (round 6): the paired 2LQG / MultiLayerQG row (SW_QG_ROW_PAIR)
# against the default — bitwise hashes (config 3, 2LQG 1024² IFMAB3, MLQG
# 2048² FilteredRK4), the 2LQG/MLQG GPU parity tests on the variant, then
# interleaved benches of config 3 and MLQG 2048².
set -o pipefail
O=gpurun_out/qgpair; mkdir -p $O
for so in sweep_var/*.so; do
  for c in "2048 qg2 IFMAB3" "1024 qg2 IFMAB3" "2048 mlqg FilteredRK4"; do
    LIBSW_PATH=$PWD/$so timeout -k 10 120 python tools/state_hash.py 6 $c >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
LIBSW_PATH=$PWD/sweep_var/b_qgpair.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mlqg.py \
  tests/test_gpu_invariants.py -x -q --timeout 300 --timeout-method thread -k "qg2 or mlqg or QG" > $O/tests.txt 2>&1 \
  || { tail -20 $O/tests.txt; exit 2; }
tail -1 $O/tests.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  for cfg in "qg2 2048 IFMAB3" "mlqg 2048 FilteredRK4"; do
    set -- $cfg
    LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps 1000 --warmup 100 --model $1 --grid $2 --stepper $3 > $O/$n.$1.$r.json 2> $O/$n.$1.$r.err \
      || { echo "$n failed"; exit 3; }
    echo "r$r $n $1 $(python -c "import json; d=json.load(open('$O/$n.$1.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
