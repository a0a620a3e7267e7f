#!/bin/bash
# Round 4 GPU batch 14: the 2LQG half row at 8192 on the radix-8 decimated
# transforms (q13dec, default now) against Stockham (q13sto); the 4096-point
# decimated columns with per-call twiddle powers (r12new = this tree) against
# HEAD (r12old) on config 4.  Parity first (8192 2LQG tests on q13dec, the
# 4096 tests on this tree).
mkdir -p gpurun_out/ab
LIBSW_PATH=$PWD/sweep_var/q13dec.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "config5 or (qg2_line_closed_form and 8192)" \
  --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_q13dec.txt 2>&1; rc=$?
echo "q13dec parity rc=$rc: $(tail -1 gpurun_out/gpu_tests_q13dec.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "8192 or 4096" --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4i.txt 2>&1; r=$?
echo "tree 4096/8192 rc=$r: $(tail -1 gpurun_out/gpu_tests_r4i.txt)"
case $r in 0|1) ;; *) exit $r;; esac
run() {  # tag so model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do
  run h_dec q13dec qg2 8192 IFMRK4 12 3 || exit 2
  run h_sto q13sto qg2 8192 IFMRK4 12 3 || exit 2
  run c4_new r12new rsw 4096 FilteredAB3 200 40 || exit 2
  run c4_old r12old rsw 4096 FilteredAB3 200 40 || exit 2
done
exit $(( rc > r ? rc : r ))
