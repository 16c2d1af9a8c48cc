#!/bin/bash
# round 5: batched BN finalizes (route fin_batch): bitwise tests, then hgc / primary A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fin_batch.py tests/test_gpu_bn_pair.py tests/test_gpu_fold_apply.py tests/test_gpu_dropin_graph.py tests/test_gpu_row3.py > gpurun_out/finbatch_tests.log 2>&1 || { tail -40 gpurun_out/finbatch_tests.log; exit 1; }
tail -3 gpurun_out/finbatch_tests.log
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default fin_batch=0 default fin_batch=0 && cp gpurun_out/ab.txt gpurun_out/finbatch_ab_hgc.txt && cat gpurun_out/finbatch_ab_hgc.txt
bash scripts/ab.sh default fin_batch=0 default fin_batch=0 && cp gpurun_out/ab.txt gpurun_out/finbatch_ab_primary.txt && cat gpurun_out/finbatch_ab_primary.txt
