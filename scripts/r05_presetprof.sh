#!/bin/bash
# round 5: kernel trace per preset -> per-step kernel tables (by grid)
set -eo pipefail
export TMPDIR=/tmp
R=$(pwd)
for p in "$@"; do
  O=$R/gpurun_out/pp_$p
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --preset $p --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 > $O/prof_bench.txt 2>&1
  grep '^{' $O/prof_bench.txt | head -1 | cut -c1-200
  db=$(find $O/prof -name "run_results.db" | head -1)
  python3 scripts/db_stats.py $db --steps 10 --csv $O/step_kernel_stats.csv --by-grid $O/step_kernel_stats_by_grid.csv --top 30 --gaps 15 > $O/top.txt
  rm -rf $O/prof
done
