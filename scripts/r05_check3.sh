#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_full.py tests/test_gpu_dropin_graph.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/wgfull_tests.log 2>&1 || { tail -40 gpurun_out/wgfull_tests.log; exit 1; }
tail -3 gpurun_out/wgfull_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 \
  || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
bash scripts/ab.sh default wg_full=16385 default wg_full=16385 default wg_full=16385 && cat gpurun_out/ab.txt
