#!/bin/bash
# On the GPU box: forward-tile shape A/B (SW_TILE_F 2 vs 4) for the half-length
# rows: per variant a state checksum (layouts must not change results), the
# bench line and the row's PMC traffic.  Variants sweep_var/{c,t}{12,13}.so.
mkdir -p gpurun_out/tiles
export TMPDIR=/tmp
for v in c13 t13; do
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 120 python -c "
import hashlib, numpy as np
from juliaraytracingsw_amd import drivers
prob, _ = drivers.qg2_problem(8192, 'IFMRK4')
prob.stepforward(1)
print('$v state sha', hashlib.sha256(prob.sol.tobytes()).hexdigest()[:16])
" || exit 1
done
run() {  # variant model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 \
    --model $2 --grid $3 --stepper $4 --steps $5 --warmup $6 > gpurun_out/tiles/$1_$2.json 2> gpurun_out/tiles/$1_$2.err \
    || { echo "$1 failed"; tail -3 gpurun_out/tiles/$1_$2.err; exit 1; }
  echo "$1 $2 $3 $(python -c "import json; d=json.load(open('gpurun_out/tiles/$1_$2.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  for c in FETCH_SIZE WRITE_SIZE; do
    LIBSW_PATH=$PWD/sweep_var/$1.so timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/tiles/p_$1_$2_$c -o run -- \
      python tools/prof_step.py --model $2 --grid $3 --stepper $4 --steps 4 > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
  done
  python tools/traffic_from_pmc.py $(find gpurun_out/tiles/p_$1_$2_FETCH_SIZE -name '*counter_collection.csv') \
    $(find gpurun_out/tiles/p_$1_$2_WRITE_SIZE -name '*counter_collection.csv') $1_$2 gpurun_out/tiles/tr_$1_$2.json > /dev/null
  rm -rf gpurun_out/tiles/p_$1_$2_*
  python -c "import json; t=json.load(open('gpurun_out/tiles/tr_$1_$2.json')); print('   MB/launch', {k: (round(t['fetch_bytes'].get(k,0)/1e6,1), round(t['write_bytes'].get(k,0)/1e6,1)) for k in t['kernels'] if k in ('row','col_step','col_fwd','col_inv','update')})"
}
for v in c12 t12; do run $v rsw 4096 FilteredAB3 300 30 || exit 1; done
for v in c13 t13; do run $v rsw 8192 FilteredAB3 40 5 || exit 1; done
for v in c13 t13; do run $v qg2 8192 IFMRK4 10 2 || exit 1; done
