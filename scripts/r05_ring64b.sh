#!/bin/bash
# round 5: 64-channel ring launches, plain / statistics-only variants (hourglass_compare): tests,
# per-shape timing, same-box A/B on hourglass_compare and the primary
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ring64.py > gpurun_out/ring64b_tests.log 2>&1 || { tail -40 gpurun_out/ring64b_tests.log; exit 1; }
tail -2 gpurun_out/ring64b_tests.log
timeout -k 10 200 python scripts/ring64_bench.py > gpurun_out/ring64b_bench.txt 2>&1
tail -5 gpurun_out/ring64b_bench.txt
BENCH_ARGS="--preset hourglass_compare" ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/ring64b_ab_hgc.txt
