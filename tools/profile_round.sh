#!/bin/bash
# Round profile on the GPU box, every configuration warm (bench.py's steady
# state: tools/prof_step.py warms for >= 0.2 s of stepping before its timed
# steps).  Per configuration: the untimed-overhead-free bench line, the
# kernel trace of a warm prof_step run (tools/trace_summary.py: per-kernel
# averages over the timed steps only, their sum per step against the bench's
# ms/step), and the PMC traffic (FETCH_SIZE and WRITE_SIZE in separate passes).
# Then SQ counters for the headline configuration.
# Usage (via gpurun): bash tools/profile_round.sh TAG [CONFIGS]
set -o pipefail
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
# model:grid:stepper:prof_steps:bench_steps[:nutune:cfltune] (RSW FilteredAB3 below
# 2048² is linearly unstable at the driver's νtune: DESIGN §4; the kernels'
# work does not depend on the parameters)
CONFIGS=${2:-"rsw:2048:FilteredAB3:400:2000 rsw:1024:FilteredAB3:800:4000:2.5:0.005 qg2:2048:IFMAB3:400:2000 rsw:4096:FilteredAB3:100:400 qg2:8192:IFMRK4:12:30"}
for c in $CONFIGS; do
  IFS=: read M N S K B NU CF <<< "$c"
  tag=${M}${N}_${S}
  X=""; [ -n "$NU" ] && X="--nutune $NU --cfltune $CF"
  timeout -k 10 300 python bench.py --model $M --grid $N --stepper $S --steps $B --warmup 50 --no-cpu-baseline \
    --no-config5 --no-config4 $X > $O/bench_$tag.json 2> $O/bench_$tag.err || exit 1
  P="python tools/prof_step.py --model $M --grid $N --stepper $S --steps $K $X"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$tag -o run -- $P > $O/run_$tag.json 2> $O/trace_$tag.err || exit 2
  cp $(find $O/trace_$tag -name '*kernel_stats.csv') $O/kernel_stats_$tag.csv || exit 3
  python tools/trace_summary.py $(find $O/trace_$tag -name '*kernel_trace.csv') $O/run_$tag.json $O/warm_$tag.json > /dev/null || exit 4
  rm -rf $O/trace_$tag
  Q="python tools/prof_step.py --model $M --grid $N --stepper $S --steps $(( K / 4 > 4 ? K / 4 : 4 )) $X"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$tag -o run -- $Q > $O/pmcf_$tag.log 2>&1 || exit 5
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$tag -o run -- $Q > $O/pmcw_$tag.log 2>&1 || exit 6
  python tools/traffic_from_pmc.py $(find $O/pmcf_$tag -name '*counter_collection.csv') \
    $(find $O/pmcw_$tag -name '*counter_collection.csv') $tag $O/traffic_$tag.json > /dev/null || exit 7
  rm -rf $O/pmcf_$tag $O/pmcw_$tag
  echo "$tag done: $(python -c "import json; b=json.load(open('$O/bench_$tag.json')); w=json.load(open('$O/warm_$tag.json')); print(round(b['value'],1), 'steps/s', round(1e3/b['value'],4), 'ms/step; warm kernel sum', round(w['kernel_sum_us_per_step'],1), 'us/step', round(w['kernel_sum_us_per_step']*b['value']/1e6,3))")"
done
P="python tools/prof_step.py --steps 100"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_sq -o run -- $P > $O/pmc_sq.log 2>&1 || exit 8
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_inst -o run -- $P > $O/pmc_inst.log 2>&1 || exit 9
python tools/pmc_summary.py $(find $O/pmc_sq $O/pmc_inst -name '*counter_collection.csv') > $O/pmc_sq_inst_summary.txt || exit 10
rm -rf $O/pmc_sq $O/pmc_inst
echo done
