#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_img.py tests/test_gpu_ring.py tests/test_gpu_row3.py tests/test_gpu_conv_bf16.py > gpurun_out/tighttol_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/tighttol_tests.log | grep -v PASSED | head -40
tail -3 gpurun_out/tighttol_tests.log
exit $rc
