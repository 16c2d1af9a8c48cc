#!/bin/bash
# round 5: weight-gradient slab reduction with every wave working (< 64 slabs: 4 column chunks
# per workgroup): bitwise test, then same-box A/B on hourglass_compare and the primary
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_twin.py -k "finish_multi or bitwise" > gpurun_out/reduce_tests.log 2>&1
tail -3 gpurun_out/reduce_tests.log
BENCH_ARGS="--preset hourglass_compare" ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/reduce_ab_hgc.txt
ROUNDS=2 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/reduce_ab_primary.txt
