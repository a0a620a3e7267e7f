#!/bin/bash
# Round 4 GPU batch 11: persistent 2LQG col_inv at 8192 with the next
# column's loads ahead of the last stores (SW_QG_INV_PERSIST, SW_QG_INV_PREF
# slots): parity of the 8192² pins/stepped state, then A/B on config 5.
mkdir -p gpurun_out/ab
for v in q13pp0 q13pp2 q13pp4; do
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "config5 or (qg2_line_closed_form and 8192)" \
    --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$v.txt 2>&1; rc=$?
  echo "$v parity rc=$rc: $(tail -1 gpurun_out/gpu_tests_$v.txt)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
run() {  # tag so
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model qg2 --grid 8192 --stepper IFMRK4 --steps 12 --warmup 3 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do for v in q13p0 q13pp0 q13pp2 q13pp4; do run $v $v || exit 1; done; done
