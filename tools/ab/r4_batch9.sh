#!/bin/bash
# Round 4 GPU batch 9: twiddle table in LDS for the decimated 4096/8192
# column transforms (SW_COL_TWLDS): GPU suite on the default build, then A/B
# on config 5 (q13tl1/q13tl0) and config 4 (r12tl1/r12tl0).
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4f.txt 2>&1; rc=$?
tail -4 gpurun_out/gpu_tests_r4f.txt
case $rc in 0|1) ;; *) exit $rc;; esac
run() {  # tag so model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do
  for v in q13tl1 q13tl0; do run $v $v qg2 8192 IFMRK4 12 3 || exit 2; done
  for v in r12tl1 r12tl0; do run $v $v rsw 4096 FilteredAB3 200 40 || exit 2; done
done
exit $rc
