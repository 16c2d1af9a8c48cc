#!/bin/bash
# round 5: batch-planned weight-gradient splits (route wg_batch_target): tests + hgc / aspp A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wgrad_batch.py > gpurun_out/wgbt_tests.log 2>&1 || { tail -40 gpurun_out/wgbt_tests.log; exit 1; }
tail -3 gpurun_out/wgbt_tests.log
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default wg_batch_target=512 wg_batch_target=1024 wg_batch_target=2048 default wg_batch_target=512 wg_batch_target=1024 wg_batch_target=2048 && cp gpurun_out/ab.txt gpurun_out/wgbt_ab_hgc.txt && cat gpurun_out/wgbt_ab_hgc.txt
