#!/bin/bash
# Round 4 GPU batch 18: the RSW row storing (ζu)^ together with P and K after
# the K transform (dzu1, SW_RSW_DEFER_ZU=1) against storing it in the pair
# split (dzu0, the default).  Parity of dzu1 first (RSW invariants at 2048).
mkdir -p gpurun_out/ab
LIBSW_PATH=$PWD/sweep_var/dzu1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
  -k "test_rsw_invariants and 2048-1 or rsw_fab3-2048" --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_dzu1.txt 2>&1; rc=$?
echo "dzu1 tests rc=$rc: $(tail -1 gpurun_out/gpu_tests_dzu1.txt)"
case $rc in 0|5) ;; *) tail -20 gpurun_out/gpu_tests_dzu1.txt; exit $rc;; esac
run() {  # tag so model grid stepper steps warmup [bench args]
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 "${@:8}" \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do
  run dzu1 dzu1 rsw 2048 FilteredAB3 2000 200 || exit 2
  run dzu0 dzu0 rsw 2048 FilteredAB3 2000 200 || exit 2
done
