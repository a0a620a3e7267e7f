#!/bin/bash
# Round profile on the GPU box: the bench line, then per configuration the
# rocprofv3 kernel stats and the PMC traffic (FETCH_SIZE and WRITE_SIZE in
# separate passes), SQ counters for the headline configuration, summaries.
# Usage (via gpurun): bash tools/profile_round.sh TAG
set -o pipefail
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo "bench done"
# the bench command itself under the kernel tracer: its col_step/row averages
# must agree with the HIP-event averages bench.py reports (roofline)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bench -o run -- python bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || exit 10
cp $(find $O/trace_bench -name '*kernel_stats.csv') $O/kernel_stats_bench.csv || exit 11
echo "traced bench done"
# model grid stepper steps
CONFIGS="rsw:2048:FilteredAB3:20 rsw:1024:FilteredAB3:20 qg2:2048:IFMAB3:20 rsw:4096:FilteredAB3:10 qg2:8192:IFMRK4:4"
for c in $CONFIGS; do
  IFS=: read M N S K <<< "$c"
  tag=${M}${N}_${S}
  P="python tools/prof_step.py --model $M --grid $N --stepper $S --steps $K --warmup 2"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$tag -o run -- $P > $O/trace_$tag.log 2>&1 || exit 2
  cp $(find $O/trace_$tag -name '*kernel_stats.csv') $O/kernel_stats_$tag.csv || exit 3
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$tag -o run -- $P > $O/pmcf_$tag.log 2>&1 || exit 4
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$tag -o run -- $P > $O/pmcw_$tag.log 2>&1 || exit 5
  python tools/traffic_from_pmc.py $(find $O/pmcf_$tag -name '*counter_collection.csv') \
    $(find $O/pmcw_$tag -name '*counter_collection.csv') $tag $O/traffic_$tag.json > /dev/null || exit 6
  echo "$tag done"
done
P="python tools/prof_step.py --steps 20 --warmup 5"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_sq -o run -- $P > $O/pmc_sq.log 2>&1 || exit 7
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_inst -o run -- $P > $O/pmc_inst.log 2>&1 || exit 8
python tools/pmc_summary.py $(find $O/pmc_sq $O/pmc_inst -name '*counter_collection.csv') > $O/pmc_sq_inst_summary.txt || exit 9
echo done
