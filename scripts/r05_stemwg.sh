#!/bin/bash
# round 5: 128-wide k tiles for the stem's weight gradient: tests, same-box A/B (primary)
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_stem.py tests/test_gpu_parity.py tests/test_gpu_conv_bf16.py > gpurun_out/stemwg_tests.log 2>&1 || { tail -30 gpurun_out/stemwg_tests.log; exit 1; }
tail -2 gpurun_out/stemwg_tests.log
ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/stemwg_ab.txt
