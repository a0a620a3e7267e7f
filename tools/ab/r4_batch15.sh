#!/bin/bash
# Round 4 GPU batch 15: the RSW row's magnitude-matched forward pairs
# (ζu + iζv, uη + ivη, K alone; this tree = rownew) against HEAD's
# (K + iζv, ζu + iuη, vη alone; rowold).  The GPU suite first, on the tree.
mkdir -p gpurun_out/ab
if [ -z "$SKIP_SUITE" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_r4j.txt 2>&1; rc=$?
  echo "tree GPU suite rc=$rc: $(tail -1 gpurun_out/gpu_tests_r4j.txt)"
  [ $rc -eq 0 ] || exit $rc
fi
run() {  # tag so model grid stepper steps warmup [bench args]
  SW_CHECK_NAN=0 LIBSW_PATH=$PWD/sweep_var/$2.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-config5 \
    --no-config4 --no-cold-profile --model $3 --grid $4 --stepper $5 --steps $6 --warmup $7 "${@:8}" \
    > gpurun_out/ab/$1.$r.json 2> gpurun_out/ab/$1.$r.err || { echo "$1 failed"; tail -5 gpurun_out/ab/$1.$r.err; exit 1; }
  echo "r$r $1 $(python -c "import json; d=json.load(open('gpurun_out/ab/$1.$r.json')); print(round(d['value'],2), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
}
for r in 1 2 3; do
  run m_new rownew rsw 2048 FilteredAB3 2000 200 || exit 2
  run m_old rowold rsw 2048 FilteredAB3 2000 200 || exit 2
  run c2_new rownew rsw 1024 FilteredAB3 4000 400 --nutune 2.5 --cfltune 0.005 || exit 2
  run c2_old rowold rsw 1024 FilteredAB3 4000 400 --nutune 2.5 --cfltune 0.005 || exit 2
done
