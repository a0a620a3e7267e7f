#!/bin/bash
# On the GPU box: the headline at the driver's short settings vs the default
mkdir -p gpurun_out/short
one() {  # tag args...
  t=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-config5 --no-config4 "$@" > gpurun_out/short/$t.json 2> gpurun_out/short/$t.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/short/$t.json')); print('$t', round(d['value'],1), round(d['ms_per_step'],4), d.get('warmup_extra_steps'))"
}
one k20w5 --steps 20 --warmup 5
one k20w5b --steps 20 --warmup 5
one k20w5_nominwarm --steps 20 --warmup 5 --min-warmup-s 0
one default
