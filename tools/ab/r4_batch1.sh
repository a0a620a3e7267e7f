#!/bin/bash
# Round 4 GPU batch: 2048 row pruning A/B (b11*), half-row A/B (q13*, r12*),
# then the GPU suite on the default build.
mkdir -p gpurun_out/ab
for r in 1 2; do for v in b11a b11b; do
  LIBSW_PATH=$PWD/sweep_var/$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --no-config5 --no-config4 \
    > gpurun_out/ab/$v.$r.json 2> gpurun_out/ab/$v.$r.err || { echo "$v failed"; tail -5 gpurun_out/ab/$v.$r.err; exit 1; }
  echo "r$r $v $(python -c "import json; d=json.load(open('gpurun_out/ab/$v.$r.json')); print(round(d['value'],1), [(k['name'], round(k['avg_us'],1)) for k in d['kernels']])")"
done; done
bash tools/ab/ab_r4_rowh.sh 2 || exit 2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4a.txt 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests_r4a.txt
exit $rc
