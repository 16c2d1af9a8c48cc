#!/bin/bash
# GPU box: ring-kernel parity tests, then the ring vs tiled micro-benchmark
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ring.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/ring_tests.log 2>&1; rc=$?
tail -25 gpurun_out/ring_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ring_bench.py > gpurun_out/ring_bench.log 2>&1; rc=$?
cat gpurun_out/ring_bench.log
exit $rc
