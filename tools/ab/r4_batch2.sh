#!/bin/bash
# Round 4 GPU batch 2: warm profiles of every BASELINE configuration
# (tools/profile_round.sh r04: bench, rocprof kernel trace, PMC traffic, SQ
# counters), then the default bench line and the smoke test.
set -o pipefail
timeout -k 10 1500 bash tools/profile_round.sh r04 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r04/bench_default.json 2> gpurun_out/r04/bench_default.err || exit 2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.txt 2>&1 || exit 3
cat gpurun_out/r04/bench_default.json
