#!/bin/bash
# Round 4 GPU batch 17: 2LQG column inverse at 2048 with both layers of a
# column in one 512-thread block (q exchanged through LDS; lp4: 128 VGPRs,
# 28 spilled; lp3: 168-VGPR cap, one block per CU) against k_col_inv's layer
# blocks (lpoff).  Parity first on the tree (lp4): the 2LQG tests.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "qg2 or invariants or mlqg" \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4l.txt 2>&1; rc=$?
echo "tree 2LQG tests rc=$rc: $(tail -1 gpurun_out/gpu_tests_r4l.txt)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/gpu_tests_r4l.txt; exit $rc; }
run() {  # tag so model grid stepper steps warmup [bench args]
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 "${@:8}" \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do
  run lp4 lp4 qg2 2048 IFMAB3 2000 200 || exit 2
  run lp3 lp3 qg2 2048 IFMAB3 2000 200 || exit 2
  run lpoff lpoff qg2 2048 IFMAB3 2000 200 || exit 2
done
