#!/bin/bash
# Round 4 GPU batch 4: the two tests fixed after batch 3, then the half-row
# layout A/B (tools/ab/ab_r4_rowh.sh: q13base/q13nb2/q13tf4, r12base/r12nb2)
# with PMC traffic per variant.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_driver_replay.py tests/test_gpu_parity.py -m gpu -q -k "driver_float32 or golden" \
  --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r4c.txt 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests_r4c.txt
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/ab/ab_r4_rowh.sh 2 || exit 3
exit $rc
