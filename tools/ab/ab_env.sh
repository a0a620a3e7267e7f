#!/bin/bash
# On the GPU box: interleaved A/B of one environment knob on one bench
# configuration (R rounds, every value once per round).
# usage: bash tools/ab/ab_env.sh TAG "bench args" VAR "v1 v2 ..." [ROUNDS]
# ("-" as a value leaves VAR unset: the library's default)
TAG=$1; ARGS=$2; VAR=$3; VALS=$4; R=${5:-2}
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do for v in $VALS; do
  out=gpurun_out/ab/${TAG}_${v}_$r
  if [ "$v" = "-" ]; then envs=""; else envs="$VAR=$v"; fi
  env $envs timeout -k 10 150 python bench.py --no-cpu-baseline --no-config5 --no-config4 --no-cold-profile \
    --no-box-state $ARGS > $out.json 2> $out.err || exit 1
  echo "$TAG r$r $VAR=$v $(python -c "import json; d=json.load(open('$out.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
