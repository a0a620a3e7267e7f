# On the GPU box: half-length rows with (b) and without (a) the decimated
# transforms (SW_ROWH_W), 4096 (--len 12 builds) and 8192 (--len 13)
set -o pipefail
mkdir -p gpurun_out/rowhw
for v in b12 b13; do
  L=${v#b}; K=$([ $L = 12 ] && echo 4096 || echo 8192)
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_pins.py -x -q --timeout 300 --timeout-method thread -k "$K and not rectangular" > gpurun_out/rowhw/$v.test.log 2>&1 || { echo "$v TESTS FAILED"; tail -5 gpurun_out/rowhw/$v.test.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/rowhw/$v.test.log)"
done
for r in 1 2; do
  for v in a12 b12; do for m in "rsw FilteredAB3 300" "qg2 IFMAB3 300"; do set -- $m
    LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 200 python bench.py --model $1 --stepper $2 --grid 4096 --steps $3 --warmup 30 --no-cpu-baseline --no-config5 --no-config4 > gpurun_out/rowhw/$v.$1.$r.json 2>/dev/null || exit 1
    echo "r$r $1 4096 $v $(python -c "import json; d=json.load(open('gpurun_out/rowhw/$v.$1.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done; done
  for v in a13 b13; do
    LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 200 python bench.py --model qg2 --grid 8192 --stepper IFMRK4 --steps 16 --warmup 3 --no-cpu-baseline --no-config5 --no-config4 > gpurun_out/rowhw/$v.c5.$r.json 2>/dev/null || exit 1
    echo "r$r c5 $v $(python -c "import json; d=json.load(open('gpurun_out/rowhw/$v.c5.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
  done
done
