#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 240 ./scripts/bin/grid_barrier_bench > gpurun_out/grid_barrier_v2.csv 2>&1 || { cat gpurun_out/grid_barrier_v2.csv; exit 1; }
cat gpurun_out/grid_barrier_v2.csv
timeout -k 10 240 python scripts/launch_census.py > gpurun_out/census_primary.txt 2>&1 || { tail -30 gpurun_out/census_primary.txt; exit 1; }
timeout -k 10 240 python scripts/launch_census.py --preset hourglass_compare > gpurun_out/census_hgc.txt 2>&1 || { tail -30 gpurun_out/census_hgc.txt; exit 1; }
wc -l gpurun_out/census_*.txt
