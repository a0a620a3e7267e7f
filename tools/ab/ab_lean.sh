#!/bin/bash
# On the GPU box: 4096-point column kernels at 4 waves/SIMD (lean twiddles,
# opaque thread index) against the default, interleaved (sweep_var/{b,l}12.so)
mkdir -p gpurun_out/lean
for r in 1 2; do for v in b12 n12 h12; do
  for cfg in "rsw FilteredAB3 400 40" "qg2 IFMAB3 300 30"; do set -- $cfg
    SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 \
      --model $1 --grid 4096 --stepper $2 --steps $3 --warmup $4 > gpurun_out/lean/${v}_$1.json 2> gpurun_out/lean/${v}_$1.err \
      || { echo "$v $1 failed"; tail -3 gpurun_out/lean/${v}_$1.err; exit 1; }
    echo "r$r $v $1 $(python -c "import json; d=json.load(open('gpurun_out/lean/${v}_$1.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
