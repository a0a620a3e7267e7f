#!/bin/bash
# On the GPU box (round 6): the software-pipelined wave-local transforms
# (SW_WL_PIPE) against the default build — bitwise state hashes, the 2048/1024
# parity and slab tests on the variant, then interleaved benches (RSW 2048²,
# RSW 1024²).  sweep_var/a_base.so, sweep_var/b_pipe.so.
set -o pipefail
O=gpurun_out/wlpipe; mkdir -p $O
for so in sweep_var/*.so; do n=$(basename $so .so)
  for g in 2048 1024; do
    LIBSW_PATH=$PWD/$so timeout -k 10 120 python tools/state_hash.py 10 $g >> $O/hash.txt 2>> $O/hash.err || exit 1
  done
done
cat $O/hash.txt
LIBSW_PATH=$PWD/sweep_var/b_pipe.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py \
  -x -q --timeout 300 --timeout-method thread -k "2048 or 1024" > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 2; }
tail -1 $O/tests.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  for cfg in "2048" "1024 --nutune 2.5 --cfltune 0.005"; do
    g=${cfg%% *}
    LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
      --no-box-state --steps 2000 --warmup 100 --grid $cfg > $O/$n.$g.$r.json 2> $O/$n.$g.$r.err || { echo "$n failed"; exit 3; }
    echo "r$r $n $g $(python -c "import json; d=json.load(open('$O/$n.$g.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
