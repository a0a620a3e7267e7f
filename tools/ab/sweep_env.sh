#!/bin/bash
# On the GPU box: short bench of every sweep_var/*.so under each value of an
# environment knob.  usage: bash tools/ab/sweep_env.sh [VAR "v1 v2 ..."]
mkdir -p gpurun_out/sweep
VAR=${1:-NONE}; VALS=${2:-0}
for so in sweep_var/*.so; do n=$(basename $so .so); for v in $VALS; do
env $VAR=$v SW_CHECK_NAN=0 LIBSW_PATH=$PWD/$so timeout -k 10 120 python bench.py --no-cpu-baseline --no-config5 --steps 1000 --warmup 100 "${@:3}" > gpurun_out/sweep/$n$v.json 2> gpurun_out/sweep/$n$v.err || exit 1
echo "$n $VAR=$v $(python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$n$v.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
