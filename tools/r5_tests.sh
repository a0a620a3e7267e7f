# round 5: selected GPU tests (a -k expression) on the default build
set -o pipefail
O=gpurun_out/r05/tests; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "$1" -s \
  > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "PASSED|FAILED|eta floor|passed|failed" $O/tests.txt | tail -15
