# round-5 quick GPU check: the driver replays, then one default bench line
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_driver_replay.py > gpurun_out/r05/replay.txt 2>&1 || { tail -30 gpurun_out/r05/replay.txt; exit 1; }
tail -3 gpurun_out/r05/replay.txt
timeout -k 10 400 python bench.py > gpurun_out/r05/bench_box.json 2> gpurun_out/r05/bench_box.err || { tail -20 gpurun_out/r05/bench_box.err; exit 2; }
python -c "import json; b=json.load(open('gpurun_out/r05/bench_box.json')); print(b['value'], b['roofline']['frac'], b['roofline']['traffic_source']); print(json.dumps(b['box'])[:3000])"
