#!/bin/bash
# Round profile: GPU tests, bench line, rocprofv3 kernel stats and PMC traffic.
# Usage (on the GPU box via gpurun): bash tools/profile_round.sh TAG
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
P="python tools/prof_step.py --steps 20 --warmup 5"
timeout -k 10 240 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/trace -o run -- python tools/prof_step.py --steps 200 > gpurun_out/$TAG/trace.log 2>&1 || exit 2
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$TAG/pmc_fetch -o run -- $P > gpurun_out/$TAG/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$TAG/pmc_write -o run -- $P > gpurun_out/$TAG/pmc_write.log 2>&1 || exit 4
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/$TAG/pmc_sq -o run -- $P > gpurun_out/$TAG/pmc_sq.log 2>&1 || exit 5
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$TAG/pmc_inst -o run -- $P > gpurun_out/$TAG/pmc_inst.log 2>&1 || exit 6
echo done
