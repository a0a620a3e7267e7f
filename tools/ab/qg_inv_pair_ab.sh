#!/bin/bash
# A/B of the XCD-paired 2LQG col_inv grid (SW_QG_INV_PAIR) on variant builds
# (tools/build_variants.sh --len 11 pair0:-DSW_QG_INV_PAIR=0 pair1:-DSW_QG_INV_PAIR=2; --len 13 pair0_13/pair1_13),
# after the 2LQG GPU parity tests.  Usage (via gpurun): bash tools/ab/qg_inv_pair_ab.sh
set -o pipefail
r() { n=$1; shift; LIBSW_PATH=$PWD/sweep_var/$n.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-config5 --model qg2 "$@" > gpurun_out/pair/$n.json 2> gpurun_out/pair/$n.err && python -c "import json; d=json.load(open('gpurun_out/pair/$n.json')); print('$n', round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])"; }
mkdir -p gpurun_out/pair
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slabs.py tests/test_gpu_large.py -m gpu -x -q -k "qg2" --timeout 200 --timeout-method thread > gpurun_out/pair/tests.log 2>&1 || { tail -20 gpurun_out/pair/tests.log; exit 1; }
tail -1 gpurun_out/pair/tests.log
r pair0 --stepper IFMAB3 --steps 1000 --warmup 20 && r pair1 --stepper IFMAB3 --steps 1000 --warmup 20 && r pair0 --stepper IFMAB3 --steps 1000 --warmup 20 && r pair1 --stepper IFMAB3 --steps 1000 --warmup 20 && r pair0_13 --grid 8192 --stepper IFMRK4 --steps 10 --warmup 2 && r pair1_13 --grid 8192 --stepper IFMRK4 --steps 10 --warmup 2
