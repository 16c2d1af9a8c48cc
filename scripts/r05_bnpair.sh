#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_pair.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/bnpair_tests.log 2>&1 || { tail -40 gpurun_out/bnpair_tests.log; exit 1; }
tail -3 gpurun_out/bnpair_tests.log
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default bn_add=0 default bn_add=0 && cat gpurun_out/ab.txt
timeout -k 10 240 ./scripts/bin/grid_barrier_bench > gpurun_out/grid_barrier_v2.csv 2>&1 || { cat gpurun_out/grid_barrier_v2.csv; exit 1; }
timeout -k 10 240 python scripts/launch_census.py > gpurun_out/census_primary.txt 2>&1 || { tail -30 gpurun_out/census_primary.txt; exit 1; }
timeout -k 10 240 python scripts/launch_census.py --preset hourglass_compare > gpurun_out/census_hgc.txt 2>&1 || { tail -30 gpurun_out/census_hgc.txt; exit 1; }
