#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bn_pair.py > gpurun_out/pairapply_tests.log 2>&1 || { tail -40 gpurun_out/pairapply_tests.log; exit 1; }
tail -2 gpurun_out/pairapply_tests.log
timeout -k 10 200 python scripts/bn_pair_bench.py 2>&1 | grep -v amdgpu.ids
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default pair_apply=1 default pair_apply=1 && cp gpurun_out/ab.txt gpurun_out/pairapply_ab.txt && cat gpurun_out/pairapply_ab.txt
