#!/bin/bash
# On the GPU box: short bench of every build/var/*.so (per-kernel HIP-event times).
# usage: bash tools/sweep.sh [extra bench args]
mkdir -p gpurun_out/sweep
for so in build/var/*.so; do
  n=$(basename $so .so)
  LIBSW_PATH=$PWD/$so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 "$@" \
    > gpurun_out/sweep/$n.json 2> gpurun_out/sweep/$n.err || { echo "$n failed rc=$?"; exit 1; }
  echo "$n $(python -c "import json,sys; d=json.load(open('gpurun_out/sweep/$n.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done
