#!/bin/bash
# Round 4 GPU batch 6: 8192-length and MultiLayerQG tests on the default build
# (4x2 forward tiles for the 2LQG rows at 8192), the lean RSW row's parity at
# 2048 (sweep_var/m11lean.so), then A/B: m11base/m11lean on the metric,
# q13fa2/q13fa1 on config 5.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "8192 or mlqg or MLQG or config5" --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4e.txt 2>&1; rc=$?
echo "default 8192/mlqg rc=$rc: $(tail -1 gpurun_out/gpu_tests_r4e.txt)"
case $rc in 0|1) ;; *) exit $rc;; esac
LIBSW_PATH=$PWD/sweep_var/m11lean.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "2048 and (rsw or RSW)" \
  --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_m11lean.txt 2>&1; r=$?
echo "m11lean parity rc=$r: $(tail -1 gpurun_out/gpu_tests_m11lean.txt)"
case $r in 0|1) ;; *) exit $r;; esac
run() {  # variant tag model grid stepper steps warmup
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$1.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 \
    > gpurun_out/ab/$1_$2.$r.json 2> gpurun_out/ab/$1_$2.$r.err \
    || { echo "$1 $2 failed"; tail -5 gpurun_out/ab/$1_$2.$r.err; exit 1; }
  echo "r$r $1 $2 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1_$2.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2; do
  for v in m11base m11lean; do run $v m rsw 2048 FilteredAB3 2000 200 || exit 3; done
  for v in q13fa2 q13fa1; do run $v c5 qg2 8192 IFMRK4 12 3 || exit 3; done
done
exit $rc
