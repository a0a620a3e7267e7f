#!/bin/bash
# SQ counters (issue / wait / instruction mix) per kernel for the headline,
# config 4 and config 5 rows, two rocprofv3 --pmc passes each
# (8 SQ counters per pass), summarised by tools/pmc_summary.py.
# usage: bash tools/ab/r6_sq.sh TAG ["model:grid:stepper:steps ..."]   (env passes through, e.g. SW_ROW_SP=1)
set -o pipefail
TAG=$1; O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
CONFIGS=${2:-"rsw:2048:FilteredAB3:100 rsw:4096:FilteredAB3:20 qg2:8192:IFMRK4:3"}
for c in $CONFIGS; do
  IFS=: read M N S K <<< "$c"
  tag=${M}${N}_${S}
  P="python tools/prof_step.py --model $M --grid $N --stepper $S --steps $K"
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/sqa_$tag -o run -- $P > $O/sqa_$tag.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/sqb_$tag -o run -- $P > $O/sqb_$tag.log 2>&1 || exit 2
  python tools/pmc_summary.py $(find $O/sqa_$tag $O/sqb_$tag -name '*counter_collection.csv') > $O/pmc_sq_$tag.txt || exit 3
  rm -rf $O/sqa_$tag $O/sqb_$tag
  echo "$tag done"
done
