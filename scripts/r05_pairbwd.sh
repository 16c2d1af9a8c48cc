#!/bin/bash
# round 5: paired BN backward (hgk_bn_bwd_pair) bitwise tests + hourglass_compare A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bn_pair.py tests/test_abi.py > gpurun_out/pairbwd_tests.log 2>&1 || { tail -30 gpurun_out/pairbwd_tests.log; exit 1; }
tail -3 gpurun_out/pairbwd_tests.log
timeout -k 10 600 python -u -m pytest -x -v -rxX --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k 8stack > gpurun_out/cfg8_tests.log 2>&1 || { tail -40 gpurun_out/cfg8_tests.log; exit 1; }
grep -E "eval-mode|N=16|PASS|XFAIL|FAIL|passed|failed" gpurun_out/cfg8_tests.log | tail -30
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default bn_pair_bwd=0 default bn_pair_bwd=0 && cp gpurun_out/ab.txt gpurun_out/pairbwd_ab.txt && cat gpurun_out/pairbwd_ab.txt
