#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_halo_bn64.py tests/test_abi.py > gpurun_out/halo64_tests.log 2>&1 || { tail -40 gpurun_out/halo64_tests.log; exit 1; }
tail -2 gpurun_out/halo64_tests.log
timeout -k 10 200 python -u scripts/halo16_bench.py > gpurun_out/halo16_bench.txt 2>&1 || { cat gpurun_out/halo16_bench.txt; exit 1; }
cat gpurun_out/halo16_bench.txt
bash scripts/ab.sh default halo_bn64=1 halo_bn64=2 default halo_bn64=1 halo_bn64=2 && cp gpurun_out/ab.txt gpurun_out/halo64_ab.txt && cat gpurun_out/halo64_ab.txt
