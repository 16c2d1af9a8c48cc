#!/bin/bash
# round 5: ring 1x1 kernel for the 64-channel launches: tests, same-box A/B (primary, then
# try_with_aspp), step table of the primary on the new build
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ring64.py tests/test_gpu_ring.py tests/test_gpu_conv_bf16.py tests/test_gpu_parity.py > gpurun_out/ring64_tests.log 2>&1 || { tail -40 gpurun_out/ring64_tests.log; exit 1; }
tail -2 gpurun_out/ring64_tests.log
ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/ring64_ab_primary.txt
BENCH_ARGS="--preset try_with_aspp" ROUNDS=2 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/ring64_ab_aspp.txt
timeout -k 10 200 python scripts/ring64_bench.py > gpurun_out/ring64_bench.txt 2>&1
cat gpurun_out/ring64_bench.txt
