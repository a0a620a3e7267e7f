# GPU check at HEAD (one box): the whole GPU suite, smoke(), the default bench
# line (with the box record).  usage: bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 2; }
tail -2 $O/smoke.txt
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 3; }
python -c "import json; b=json.load(open('$O/bench_default.json')); print(b['value'], b['roofline']['frac'], b['config5']['value'], b['config4']['value'])"
