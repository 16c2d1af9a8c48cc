#!/bin/bash
# round-5 GPU check: grid-barrier microbenchmark, the GPU test suite (-s: gate values logged), one
# bench line. Each GPU step under its own time limit, chained.
mkdir -p gpurun_out
timeout -k 10 240 ./scripts/bin/grid_barrier_bench > gpurun_out/grid_barrier.csv 2>&1 \
  || { cat gpurun_out/grid_barrier.csv; exit 1; }
cat gpurun_out/grid_barrier.csv
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1 || { tail -60 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 \
  || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
