#!/bin/bash
# round 5: LDS-DMA halo weight gradient — bitwise tests, per-launch bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wgrad_dma.py > gpurun_out/wgdma_tests.log 2>&1 || { tail -40 gpurun_out/wgdma_tests.log; exit 1; }
tail -3 gpurun_out/wgdma_tests.log
cd scripts && timeout -k 10 300 python -u wgrad_dma_bench.py > ../gpurun_out/wgdma_bench.txt 2>&1; rc=$?; cd ..; cat gpurun_out/wgdma_bench.txt; exit $rc
