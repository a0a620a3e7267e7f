#!/bin/bash
# On the GPU box: 2048-point kernels with the lean register measures
# (sweep_var/{b11,qa,qb,qc}.so), interleaved: 2LQG IFMAB3 (config 3) and the
# RSW FilteredAB3 metric
mkdir -p gpurun_out/lean11
for r in 1 2; do for v in b11 n11; do
  for cfg in "qg2 IFMAB3 2000 200" "rsw FilteredAB3 2000 200"; do set -- $cfg
    SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 \
      --model $1 --grid 2048 --stepper $2 --steps $3 --warmup $4 > gpurun_out/lean11/${v}_$1.json 2> gpurun_out/lean11/${v}_$1.err \
      || { echo "$v $1 failed"; tail -3 gpurun_out/lean11/${v}_$1.err; exit 1; }
    echo "r$r $v $1 $(python -c "import json; d=json.load(open('gpurun_out/lean11/${v}_$1.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
