#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wgrad_batch.py tests/test_gpu_presets.py tests/test_gpu_fin_batch.py > gpurun_out/slab2_tests.log 2>&1 || { tail -40 gpurun_out/slab2_tests.log; exit 1; }
tail -2 gpurun_out/slab2_tests.log
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default wg_batch_slab_x10=20 wg_batch_slab_x10=3 default wg_batch_slab_x10=20 wg_batch_slab_x10=3 && cp gpurun_out/ab.txt gpurun_out/slab2_ab_hgc.txt && cat gpurun_out/slab2_ab_hgc.txt
