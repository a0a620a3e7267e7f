#!/bin/bash
# On the GPU box: FETCH/WRITE traffic per kernel launch (separate PMC passes)
# and per-kernel times for one libsw build at one size.
# usage: bash tools/traffic_at.sh SO TAG MODEL STEPPER N STEPS
SO=$1; TAG=$2; M=$3; ST=$4; N=$5; K=$6
export TMPDIR=/tmp
O=gpurun_out/tr/$TAG; mkdir -p $O
P="python tools/prof_step.py --model $M --stepper $ST --grid $N --steps $K --warmup 2"
LIBSW_PATH=$SO timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- $P > $O/f.log 2>&1 || exit 1
LIBSW_PATH=$SO timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- $P > $O/w.log 2>&1 || exit 2
python tools/traffic_from_pmc.py $(find $O/f -name '*counter_collection.csv') $(find $O/w -name '*counter_collection.csv') ${M}${N}_$ST $O/t.json > /dev/null || exit 3
LIBSW_PATH=$SO timeout -k 10 200 python bench.py --no-cpu-baseline --model $M --stepper $ST --grid $N --steps $K --warmup 2 --profile-steps 3 > $O/b.json 2> $O/b.err || exit 4
python - $O <<'PY'
import json, sys
o = sys.argv[1]
t = json.load(open(o + "/t.json")); b = json.load(open(o + "/b.json"))
print(o, round(b["value"], 1), "steps/s")
for k in b["kernels"]:
    tr = t["kernels"].get(k["name"])
    print(f"  {k['name']:>9s} {k['avg_us']:9.1f} us  alg {k['alg_bytes']/1e6:8.1f} MB  traffic {tr/1e6 if tr else float('nan'):8.1f} MB")
PY
