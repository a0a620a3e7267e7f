#!/bin/bash
# On the GPU box (round 6): the half rows with the live band at compile time
# (sweep_var/b_kc.so) against the HEAD build (a_base.so): bitwise hashes at
# config 4, config 5 and 2LQG 4096², the large-grid parity tests on the
# variant, then interleaved config-4 / config-5 benches.
set -o pipefail
O=gpurun_out/rowkc; mkdir -p $O
for so in sweep_var/*.so; do
  for c in "2 8192 qg2 IFMRK4" "6 4096 rsw FilteredAB3" "4 4096 qg2 IFMAB3"; do
    LIBSW_PATH=$PWD/$so timeout -k 10 200 python tools/state_hash.py $c >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
LIBSW_PATH=$PWD/sweep_var/b_kc.so timeout -k 10 700 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py \
  -x -q --timeout 300 --timeout-method thread -k "large or 4096 or 8192 or rect" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 2; }
tail -1 $O/tests.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  for cfg in "rsw 4096 FilteredAB3 300" "qg2 8192 IFMRK4 30"; do
    set -- $cfg
    LIBSW_PATH=$PWD/$so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps $4 --warmup 10 --model $1 --grid $2 --stepper $3 > $O/$n.$1.$r.json 2> $O/$n.$1.$r.err \
      || { echo "$n failed"; exit 3; }
    echo "r$r $n $1$2 $(python -c "import json; d=json.load(open('$O/$n.$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
