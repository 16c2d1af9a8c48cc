#!/bin/bash
# One parametrised GPU-box recipe (replaces round 5's one-off r05_*.sh files). Every step has its
# own time limit and the first failure ends the run (no GPU step after a failed one).
#   TAG=name                     output prefix under gpurun_out/ (default: recipe)
#   TESTS="tests/x.py -k y"      pytest selection, run first
#   PRE="python -u scripts/z.py" a measurement command after the tests (stdout -> <TAG>_pre.txt)
#   PROF=1                       a rocprofv3 kernel trace of a 20-step bench run -> per-step kernel
#                                table (scripts/db_stats.py: <TAG>_prof/top.txt, by-grid CSV)
#   AB="default k=v default k=v" alternating same-box bench.py --route configurations (scripts/ab.sh;
#                                BENCH_ARGS is passed on, e.g. "--preset hourglass_compare")
# example: TAG=halo64 TESTS="tests/test_gpu_halo_bn64.py" PRE="python -u scripts/halo16_bench.py" \
#          AB="default halo_bn64=1 halo_bn64=2 default halo_bn64=1 halo_bn64=2" bash scripts/gpu_recipe.sh
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-recipe}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread $TESTS \
    > "gpurun_out/${TAG}_tests.log" 2>&1 || { tail -40 "gpurun_out/${TAG}_tests.log"; exit 1; }
  tail -2 "gpurun_out/${TAG}_tests.log"
fi
if [ -n "$PRE" ]; then
  timeout -k 10 300 $PRE > "gpurun_out/${TAG}_pre.txt" 2>&1 || { tail -20 "gpurun_out/${TAG}_pre.txt"; exit 1; }
  tail -30 "gpurun_out/${TAG}_pre.txt"
fi
if [ -n "$PROF" ]; then
  O="gpurun_out/${TAG}_prof"; mkdir -p "$O"
  TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py $BENCH_ARGS --steps 20 \
    --warmup 5 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 > "$O/prof_bench.txt" 2>&1 || { tail -20 "$O/prof_bench.txt"; exit 1; }
  db=$(find "$O/prof" -name "run_results.db" | head -1)
  python3 scripts/db_stats.py "$db" --steps 10 --csv "$O/step_kernel_stats.csv" \
    --by-grid "$O/step_kernel_stats_by_grid.csv" --top 40 > "$O/top.txt" && rm -rf "$O/prof"
  head -25 "$O/top.txt"
fi
if [ -n "$AB" ]; then
  bash scripts/ab.sh $AB || { cat gpurun_out/ab.txt; exit 1; }
  cp gpurun_out/ab.txt "gpurun_out/${TAG}_ab.txt"
  cat "gpurun_out/${TAG}_ab.txt"
fi
