#!/bin/bash
# MattParameters' grid (384², MLQG FilteredRK4) on the generic engine: the
# bench line (with the oracle's CPU rate at 128²/384²/1024²/2048²) and the
# kernel trace of a warm prof_step run.  usage: bash tools/ab/r6_gen384.sh TAG
set -o pipefail
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model mlqg --grid 384 --stepper FilteredRK4 --steps 1000 --warmup 20 \
  --no-config5 --no-config4 --no-cold-profile > $O/bench_mlqg384_FilteredRK4.json 2> $O/bench_mlqg384.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python tools/prof_step.py --model mlqg --grid 384 --stepper FilteredRK4 --steps 400 > $O/run_mlqg384.json 2> $O/trace.err || exit 2
cp $(find $O/trace -name '*kernel_stats.csv') $O/kernel_stats_mlqg384_FilteredRK4.csv || exit 3
rm -rf $O/trace
python -c "import json; b=json.load(open('$O/bench_mlqg384_FilteredRK4.json')); print(b['value'], b['kernels'], b['cpu_baseline']['by_grid'])"
