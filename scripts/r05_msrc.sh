#!/bin/bash
# round 5: up to 40 sources per multi-use weight-gradient launch: tests, same-box A/B (primary)
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_twin.py tests/test_gpu_parity.py tests/test_gpu_wgrad_batch.py > gpurun_out/msrc_tests.log 2>&1 || { tail -30 gpurun_out/msrc_tests.log; exit 1; }
tail -2 gpurun_out/msrc_tests.log
ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/msrc_ab.txt
