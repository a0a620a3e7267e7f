#!/bin/bash
# Round profile on the GPU box: bench line, rocprofv3 kernel stats, PMC traffic
# (FETCH_SIZE and WRITE_SIZE in separate passes) and SQ counters, then the
# summaries.  Usage (via gpurun): bash tools/profile_round.sh TAG
set -o pipefail
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
P="python tools/prof_step.py --steps 20 --warmup 5"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/prof_step.py --steps 200 > $O/trace.log 2>&1 || exit 2
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $P > $O/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $P > $O/pmc_write.log 2>&1 || exit 4
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_sq -o run -- $P > $O/pmc_sq.log 2>&1 || exit 5
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_inst -o run -- $P > $O/pmc_inst.log 2>&1 || exit 6
python tools/traffic_from_pmc.py $(find $O/pmc_fetch -name '*counter_collection.csv') $(find $O/pmc_write -name '*counter_collection.csv') rsw2048_FilteredAB3 $O/traffic_rsw2048_fab3.json > /dev/null || exit 7
python tools/pmc_summary.py $(find $O/pmc_sq $O/pmc_inst -name '*counter_collection.csv') > $O/pmc_sq_inst_summary.txt || exit 8
cp $(find $O/trace -name '*kernel_stats.csv') $O/kernel_stats_rsw2048_fab3.csv || exit 9
echo done
