#!/bin/bash
# On the GPU box (round 6): the KC row kernels specialised to one slab
# (sweep_var/b_s1.so: no slab-division paths) against HEAD (a_base.so):
# bitwise hashes, the whole GPU suite on the variant, interleaved benches.
# usage: r6_slab1.sh [check|bench]
set -o pipefail
O=gpurun_out/s1; mkdir -p $O
if [ "$1" != "bench" ]; then
for so in sweep_var/*.so; do
  for c in "20 512 rsw IFMAB3" "8 512 ty ETDRK4" "6 512 mlqg FilteredRK4" "10 2048 rsw FilteredAB3" "6 2048 qg2 IFMAB3" \
           "2 8192 qg2 IFMRK4" "6 4096 rsw FilteredAB3" "8 1024 rsw IFMRK4"; do
    LIBSW_PATH=$PWD/$so timeout -k 10 200 python tools/state_hash.py $c >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
LIBSW_PATH=$PWD/sweep_var/b_s1.so timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 2; }
tail -1 $O/gpu_tests.txt
fi
if [ "$1" != "check" ]; then
for r in 1 2; do for so in sweep_var/*.so; do n=$(basename $so .so)
  for cfg in "rsw 2048 FilteredAB3 2000" "qg2 2048 IFMAB3 2000" "rsw 512 IFMAB3 8000" "ty 512 ETDRK4 2000" \
             "mlqg 512 FilteredRK4 2000" "rsw 4096 FilteredAB3 300" "qg2 8192 IFMRK4 20"; do
    set -- $cfg
    LIBSW_PATH=$PWD/$so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps $4 --warmup 20 --model $1 --grid $2 --stepper $3 > $O/$n.$1$2.$r.json 2> $O/$n.$1$2.$r.err \
      || { echo "$n failed"; exit 3; }
    echo "r$r $n $1$2 $(python -c "import json; d=json.load(open('$O/$n.$1$2.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
fi
