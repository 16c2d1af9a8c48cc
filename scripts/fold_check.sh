#!/bin/bash
# GPU check of the folded BN-backward apply: its tests, the twin / parity suites, then a same-box
# A/B (fold_apply=0/1 alternating). usage: bash scripts/fold_check.sh
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fold_apply.py tests/test_gpu_twin.py tests/test_gpu_ring.py -x -v --timeout 120 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || { tail -40 gpurun_out/fold_tests.log; exit 1; }
tail -3 gpurun_out/fold_tests.log
bash scripts/ab.sh "fold_apply=0" "fold_apply=1" "fold_apply=0" "fold_apply=1" "fold_apply=0" "fold_apply=1" && cat gpurun_out/ab.txt
