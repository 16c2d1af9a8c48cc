#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_full.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/wgfull_tests.log 2>&1 || { tail -40 gpurun_out/wgfull_tests.log; exit 1; }
tail -3 gpurun_out/wgfull_tests.log
bash scripts/ab.sh default wg_full=16385 default wg_full=16385 default wg_full=16385 && cat gpurun_out/ab.txt
