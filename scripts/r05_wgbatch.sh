#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_batch.py tests/test_gpu_bn_pair.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/wgbatch_tests.log 2>&1 || { tail -40 gpurun_out/wgbatch_tests.log; exit 1; }
tail -3 gpurun_out/wgbatch_tests.log
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default wg_batch=0 default wg_batch=0 && cat gpurun_out/ab.txt
