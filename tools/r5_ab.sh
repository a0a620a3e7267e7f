# round 5 A/B on the GPU box: GPU tests on the default build (TESTS: a -k
# expression), then R interleaved rounds of bench.py for every
# sweep_var/<name>.so in $AB, with BARGS (default: the headline)
set -o pipefail
O=gpurun_out/r05/ab; mkdir -p $O
R=${R:-3}
BARGS=${BARGS:---steps 2000 --warmup 200}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/ -m gpu \
    -k "$TESTS" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
  tail -1 $O/tests.txt
fi
for r in $(seq $R); do for so in $AB; do
  LIBSW_PATH=$PWD/sweep_var/$so.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-box-state $BARGS > $O/$so.$r.json 2> $O/$so.$r.err \
    || { echo "bench $so failed"; tail $O/$so.$r.err; exit 2; }
  echo "r$r $so $(python -c "import json; d=json.load(open('$O/$so.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
