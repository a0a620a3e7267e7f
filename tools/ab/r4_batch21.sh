#!/bin/bash
# Round 4 GPU batch 21: the RSW row inverse pairs u + iη, v + iζ (ue1, SW_RSW_INV_UE=1, 216
# VGPRs) against u + iv, η + iζ (ue0).  Parity of ue1 first (incl. the invariants).
#
mkdir -p gpurun_out/ab
for v in ue1; do
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "rsw_fab3-2048 or test_rsw_invariants and 2048-1" -s \
    --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$v.txt 2>&1; rc=$?
  echo "$v tests rc=$rc: $(tail -1 gpurun_out/gpu_tests_$v.txt)"
  [ $rc -eq 0 ] || exit $rc
done
run() {  # tag so model grid stepper steps warmup [bench args]
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 "${@:8}" \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do
  run ue1 ue1 rsw 2048 FilteredAB3 2000 200 || exit 2
  run ue0 ue0 rsw 2048 FilteredAB3 2000 200 || exit 2
done
