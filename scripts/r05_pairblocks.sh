#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fin_batch.py tests/test_gpu_halo_bn64.py tests/test_gpu_presets.py > gpurun_out/pairblocks_tests.log 2>&1 || { tail -40 gpurun_out/pairblocks_tests.log; exit 1; }
tail -2 gpurun_out/pairblocks_tests.log
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default pair_blocks=0 default pair_blocks=0 && cp gpurun_out/ab.txt gpurun_out/pairblocks_ab.txt && cat gpurun_out/pairblocks_ab.txt
bash scripts/ab.sh default halo_bn64=6 halo_bn64=0 default halo_bn64=6 halo_bn64=0 && cp gpurun_out/ab.txt gpurun_out/halo64b_ab.txt && cat gpurun_out/halo64b_ab.txt
