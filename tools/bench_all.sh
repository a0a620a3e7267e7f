#!/bin/bash
# On the GPU box: bench every model/stepper pair at one size (per-kernel times).
# usage: bash tools/bench_all.sh [N] [tag]    (env passes through, e.g. SW_FUSE_ALL=1)
N=${1:-2048}; TAG=${2:-}
mkdir -p gpurun_out/all
for ms in rsw:FilteredAB3 rsw:IFMAB3 rsw:IFMRK4 qg2:IFMAB3 qg2:IFMRK4 qg2:FilteredAB3; do
  m=${ms%%:*}; st=${ms#*:}
  f=gpurun_out/all/${m}_${st}_$N$TAG
  timeout -k 10 180 python bench.py --no-cpu-baseline --grid $N --model $m --stepper $st --steps 50 --warmup 5 \
    > $f.json 2> $f.err || { echo "$m $st failed"; tail -3 $f.err; exit 1; }
  echo "$TAG $m $st $N $(python -c "import json; d=json.load(open('$f.json')); print(round(d['value'],1), 'steps/s', [(k['name'], round(k['avg_us'],1), k['per_step']) for k in d['kernels']])")"
done
