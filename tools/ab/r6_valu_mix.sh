#!/bin/bash
# On the GPU box (round 6): the dynamic VALU instruction mix per kernel (fp64
# add/mul/fma against int32/int64/cvt), one rocprofv3 --pmc pass per
# configuration, summarised by tools/pmc_summary.py.
set -o pipefail
O=gpurun_out/valu_mix; mkdir -p $O
export TMPDIR=/tmp
for c in "qg2:8192:IFMRK4:3" "rsw:2048:FilteredAB3:50"; do
  IFS=: read M N S K <<< "$c"
  tag=${M}${N}_${S}
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/p_$tag -o run -- python tools/prof_step.py --model $M --grid $N --stepper $S --steps $K > $O/p_$tag.log 2>&1 || { tail -5 $O/p_$tag.log; exit 1; }
  python tools/pmc_summary.py $(find $O/p_$tag -name '*counter_collection.csv') > $O/valu_mix_$tag.txt || exit 2
  rm -rf $O/p_$tag
  echo "$tag done"
done
