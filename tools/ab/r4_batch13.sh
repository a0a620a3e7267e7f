#!/bin/bash
# Round 4 GPU batch 13: aliased-state tracking on one slab per process (the
# multiprocess and aliased tests first), then the whole GPU suite.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_multiprocess.py tests/test_gpu_aliased.py -m gpu -q \
  --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_r4g.txt 2>&1; rc=$?
tail -25 gpurun_out/gpu_tests_r4g.txt
case $rc in 0) ;; 1) exit 1;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_r4h.txt 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests_r4h.txt
exit $rc
