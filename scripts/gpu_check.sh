#!/bin/bash
# GPU-box check: the gpu test suite, then one bench line (each step under its own time limit).
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 \
  || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['ms_per_step'])"
