# round 5 A/B on the GPU box: the RSW-row tests on the default build, then
# interleaved benches of sweep_var/<so> under SW_ROW_DMA=<d> for every
# "so:d" in $AB (R rounds)
set -o pipefail
O=gpurun_out/r05/ab; mkdir -p $O
R=${R:-3}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_invariants.py tests/test_gpu_slabs.py tests/test_gpu_aliased.py tests/test_gpu_large.py \
  -k "${TESTS:-rsw or row_dma or large or determinism or checkpoint or config5}" > $O/tests.txt 2>&1 \
  || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in $(seq $R); do for c in $AB; do so=${c%%:*}; d=${c#*:}
  LIBSW_PATH=$PWD/sweep_var/$so.so SW_ROW_DMA=$d timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-box-state --steps 2000 --warmup 200 > $O/$so.$d.$r.json 2> $O/$so.$d.$r.err \
    || { echo "bench $c failed"; tail $O/$so.$d.$r.err; exit 2; }
  echo "r$r $so dma=$d $(python -c "import json; d=json.load(open('$O/$so.$d.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
