#!/bin/bash
# round 5: batched weight-gradient jobs grouped by tile shape, longest workgroups first: bitwise
# tests, same-box A/B (hourglass_compare, primary), the hourglass_compare step table
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_wgrad_batch.py > gpurun_out/wgsort_tests.log 2>&1
tail -2 gpurun_out/wgsort_tests.log
BENCH_ARGS="--preset hourglass_compare" ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/wgsort_ab_hgc.txt
ROUNDS=2 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/wgsort_ab_primary.txt
bash scripts/r05_stepdump.sh hourglass_compare
grep -E "wgrad_batch|launches" gpurun_out/sd_hourglass_compare/top.txt
