#!/bin/bash
# On the GPU box: A/B of full-build variants (every transform length) over the
# BASELINE configurations, variants interleaved per round so box drift hits
# all alike.  usage: bash tools/ab/ab_cfg.sh R so1 so2 ... [-- CONFIGS]
#   CONFIGS: model:grid:stepper:steps[:nutune:cfltune] (default: configs 2-5 + the metric)
mkdir -p gpurun_out/abc
R=$1; shift
SOS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SOS+=("$1"); shift; done
[ "$1" = "--" ] && shift
CONFIGS=${*:-"rsw:2048:FilteredAB3:2000 qg2:2048:IFMAB3:2000 rsw:1024:FilteredAB3:4000:2.5:0.005 rsw:4096:FilteredAB3:300 qg2:8192:IFMRK4:16"}
for r in $(seq $R); do for c in $CONFIGS; do
  IFS=: read M N S K NU CF <<< "$c"
  X=""; [ -n "$NU" ] && X="--nutune $NU --cfltune $CF"
  W=$(( K / 10 > 2 ? K / 10 : 2 ))
  for so in "${SOS[@]}"; do n=$(basename $so .so)
    o=gpurun_out/abc/$n.$M$N.$r
    LIBSW_PATH=$PWD/$so timeout -k 10 200 python bench.py --model $M --grid $N --stepper $S --steps $K --warmup $W \
      --no-cpu-baseline --no-config5 --no-config4 $X > $o.json 2> $o.err || { echo "$n $M$N failed"; tail -3 $o.err; exit 1; }
    echo "r$r $M$N $S $n $(python -c "import json; d=json.load(open('$o.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done; done
