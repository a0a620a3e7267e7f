#!/bin/bash
# Round 4 GPU batch 8: the RSW row through one line buffer at 3 waves per
# SIMD (sweep_var/m11b3.so, -DSW_RSW_ROW_1B=3): parity at 2048, then A/B
# against m11base on the metric.
mkdir -p gpurun_out/ab
LIBSW_PATH=$PWD/sweep_var/m11b3.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "2048" \
  --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_m11b3.txt 2>&1; rc=$?
echo "m11b3 parity rc=$rc: $(tail -1 gpurun_out/gpu_tests_m11b3.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
run() {  # tag so
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model rsw --grid 2048 --stepper FilteredAB3 --steps 2000 --warmup 200 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do run b_base m11base || exit 2; run b_b3 m11b3 || exit 2; done
exit $rc
