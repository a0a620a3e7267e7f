#!/bin/bash
# Round 4 GPU batch 5: GPU suite on the default build (2LQG/MultiLayerQG
# columns decimated from 2048), the 8192 2LQG-row variants' parity
# (8192-length tests against sweep_var/q13w16*.so), then their A/B on config 5.
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4d.txt 2>&1; rc=$?
tail -6 gpurun_out/gpu_tests_r4d.txt
case $rc in 0|1) ;; *) exit $rc;; esac
for v in q13w16 q13w16tf4; do
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "config5 or (qg2_line_closed_form and 8192)" \
    --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$v.txt 2>&1; r=$?
  echo "$v parity rc=$r: $(tail -1 gpurun_out/gpu_tests_$v.txt)"
  case $r in 0|1|5) ;; *) exit $r;; esac
done
run() {  # variant
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model qg2 --grid 8192 --stepper IFMRK4 --steps 12 --warmup 3 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do for v in q13base q13tf4 q13w16 q13w16tf4; do run $v || exit 3; done; done
exit $rc
