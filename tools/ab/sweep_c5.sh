#!/bin/bash
# On the GPU box: config 5 (2LQG 8192² IFMRK4) per sweep_var/*.so (--len 13 builds)
mkdir -p gpurun_out/sweep
for so in sweep_var/*.so; do n=$(basename $so .so)
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/$so timeout -k 10 150 python bench.py --no-cpu-baseline --no-config5 --steps 10 --warmup 2 \
    --profile-steps 3 --model qg2 --grid 8192 --stepper IFMRK4 > gpurun_out/sweep/$n.json 2> gpurun_out/sweep/$n.err || exit 1
  echo "$n $(python -c "import json; d=json.load(open('gpurun_out/sweep/$n.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done
