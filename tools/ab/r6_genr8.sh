#!/bin/bash
# On the GPU box (round 6): the generic engine's radix plan with radix-8 stages
# (sweep_var/b_r8.so, 384 = 8·8·2·3) against the radix-4 plan (a_r4.so,
# 4·4·4·2·3): the generic GPU tests on the new build, interleaved MattParameters
# 384² benches, TwoLayerSimulation's cadence at 384².
set -o pipefail
O=gpurun_out/genr8; mkdir -p $O
LIBSW_PATH=$PWD/sweep_var/b_r8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_generic.py > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2 3; do for so in sweep_var/*.so; do n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
    --no-box-state --steps 4000 --warmup 200 --model mlqg --grid 384 > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; exit 2; }
  echo "r$r $n $(python -c "import json; d=json.load(open('$O/$n.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
LIBSW_PATH=$PWD/sweep_var/b_r8.so timeout -k 10 300 python tools/driver_cadence.py --only mlqg384 --out $O/cadence.json > $O/cadence.log 2>&1 || exit 3
grep cadence $O/cadence.log
