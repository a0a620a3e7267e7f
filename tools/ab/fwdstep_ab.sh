#!/bin/bash
# A/B of the fused forward+update column pass (SW_FWD_STEP=1, default) against
# separate col_fwd + update kernels (SW_FWD_STEP=0) on the coupled-update pairs;
# SW_FWD_STEP=2: the variant with N parked in LDS. FS="0 2" picks the modes.
# Usage (via gpurun): bash tools/ab/fwdstep_ab.sh [OUTDIR]
set -o pipefail
O=${1:-gpurun_out/fwdstep}
mkdir -p $O
for c in ${CONFIGS:-qg2:2048:IFMAB3:1000 rsw:2048:IFMAB3:1000 qg2:2048:FilteredAB3:1000 qg2:1024:IFMAB3:2000 rsw:2048:IFMRK4:300 qg2:4096:IFMAB3:200 qg2:8192:IFMRK4:10}; do
  IFS=: read M N S K <<< "$c"
  for F in ${FS:-0 1 2}; do
    SW_FWD_STEP=$F timeout -k 10 240 python bench.py --model $M --grid $N --stepper $S --steps $K --warmup 20 \
      --no-cpu-baseline --no-config5 > $O/${M}${N}_${S}_fs$F.json 2> $O/${M}${N}_${S}_fs$F.err || exit 1
    python -c "import json,sys; d=json.load(open('$O/${M}${N}_${S}_fs$F.json')); print('$c fs=$F', d['value'], d['ms_per_step'])"
  done
done
