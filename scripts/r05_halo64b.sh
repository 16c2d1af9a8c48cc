#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_halo_bn64.py tests/test_abi.py > gpurun_out/halo64_tests.log 2>&1 || { tail -40 gpurun_out/halo64_tests.log; exit 1; }
tail -2 gpurun_out/halo64_tests.log
bash scripts/ab.sh default halo_bn64=6 halo_bn64=0 default halo_bn64=6 halo_bn64=0 && cp gpurun_out/ab.txt gpurun_out/halo64b_ab.txt && cat gpurun_out/halo64b_ab.txt
