#!/bin/bash
# Round 4 GPU batch 3: GPU suite on the default build (decimated columns
# from 4096), then the column-decimation A/B (tools/ab/ab_r4_coldec.sh) and the
# half-row layout A/B (q13*/r12* builds).
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4b.txt 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests_r4b.txt
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/ab/ab_r4_coldec.sh 2 || exit 2

exit $rc
