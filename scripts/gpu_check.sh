#!/bin/bash
# GPU-box check: the gpu test suite, then one bench line (each step under its own time limit).
# usage: bash scripts/gpu_check.sh
mkdir -p gpurun_out

timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 \
  || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
