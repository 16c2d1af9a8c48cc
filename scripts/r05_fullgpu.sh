#!/bin/bash
# round 5: the whole GPU suite, then the configs[4] N=16 gradient gates' printed numbers, then smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rxX --timeout 300 --timeout-method thread > gpurun_out/r05_gputests.log 2>&1 || { tail -60 gpurun_out/r05_gputests.log; exit 1; }
tail -8 gpurun_out/r05_gputests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -q -s -k "8stack and (eval or batch_fp32)" --timeout 300 --timeout-method thread > gpurun_out/r05_cfg8_numbers.log 2>&1 || { tail -30 gpurun_out/r05_cfg8_numbers.log; exit 1; }
grep -E "engine|draw|eval|loss" gpurun_out/r05_cfg8_numbers.log | head -60
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || { tail -20 gpurun_out/r05_smoke.log; exit 1; }
tail -5 gpurun_out/r05_smoke.log
