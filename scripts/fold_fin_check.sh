#!/bin/bash
# GPU check of the folded BN finalize: its tests, the full GPU suite, then a same-box A/B
# (fold_fin=0/1 alternating). usage: bash scripts/fold_fin_check.sh
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold_fin.py -x -v --timeout 120 --timeout-method thread > gpurun_out/foldfin_tests.log 2>&1 || { tail -40 gpurun_out/foldfin_tests.log; exit 1; }
tail -3 gpurun_out/foldfin_tests.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
bash scripts/ab.sh "fold_fin=0" "fold_fin=1" "fold_fin=0" "fold_fin=1" "fold_fin=0" "fold_fin=1" && cat gpurun_out/ab.txt
