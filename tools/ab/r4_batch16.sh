#!/bin/bash
# Round 4 GPU batch 16: the paired-K RSW row (k_row_rsw_kp: two rows per
# block, K_A + iK_B as one complex transform) against k_row (kpoff), 2048
# only.  Parity first on the tree (RSW tests at 2048, slabs, invariants).
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "rsw or invariants or slabs or determinism or boundary" \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4k.txt 2>&1; rc=$?
echo "tree RSW tests rc=$rc: $(tail -1 gpurun_out/gpu_tests_r4k.txt)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/gpu_tests_r4k.txt; exit $rc; }
run() {  # tag so model grid stepper steps warmup [bench args]
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 "${@:8}" \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do
  run kp_on kpon rsw 2048 FilteredAB3 2000 200 || exit 2
  run kp_off kpoff rsw 2048 FilteredAB3 2000 200 || exit 2
done
