#!/bin/bash
# On the GPU box: per-model bench lines for sweep_var/<name><len>.so builds
# (tools/build_variants.sh --len L).  usage: bash tools/ab/sweep_models.sh
mkdir -p gpurun_out/sweep
run() {  # so model grid stepper
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-config5 \
    --steps 500 --warmup 50 --model $2 --grid $3 --stepper $4 > gpurun_out/sweep/$1_$2.json 2> gpurun_out/sweep/$1_$2.err || return 1
  echo "$1 $2 $3 $4 $(python -c "import json; d=json.load(open('gpurun_out/sweep/$1_$2.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for so in sweep_var/*9.so; do n=$(basename $so .so); run $n ty 512 ETDRK4 || exit 1; run $n mlqg 512 FilteredRK4 || exit 1; done
for so in sweep_var/*11.so; do n=$(basename $so .so); run $n qg2 2048 IFMAB3 || exit 1; run $n rsw 2048 FilteredAB3 || exit 1; done
