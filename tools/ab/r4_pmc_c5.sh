#!/bin/bash
# Round 4: SQ counters of the config-5 kernels (2LQG 8192² IFMRK4) and of
# config 4 (RSW 4096² FilteredAB3), two passes each.
export TMPDIR=/tmp
O=gpurun_out/pmc5; mkdir -p $O
for c in "qg2 IFMRK4 8192 4" "rsw FilteredAB3 4096 20"; do
  set -- $c
  P="python tools/prof_step.py --model $1 --stepper $2 --grid $3 --steps $4"
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/sq_$1$3 -o run -- $P > $O/sq_$1$3.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/in_$1$3 -o run -- $P > $O/in_$1$3.log 2>&1 || exit 2
  python tools/pmc_summary.py $(find $O/sq_$1$3 $O/in_$1$3 -name '*counter_collection.csv') > $O/pmc_sq_inst_$1$3.txt || exit 3
  rm -rf $O/sq_$1$3 $O/in_$1$3
done
