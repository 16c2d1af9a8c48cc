#!/bin/bash
# round 5: kernel trace of the default bench per preset -> ordered launch list of one step + tables
set -eo pipefail
export TMPDIR=/tmp
R=$(pwd)
for p in "$@"; do
  O=$R/gpurun_out/sd_$p
  mkdir -p $O
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 $R/bench.py --preset $p --steps 12 --warmup 3 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 > $O/prof_bench.txt 2>&1
  db=$(find $O/prof -name "run_results.db" | head -1)
  python3 scripts/step_dump.py $db > $O/step.txt
  python3 scripts/db_stats.py $db --steps 8 --csv $O/step_kernel_stats.csv --by-grid $O/step_kernel_stats_by_grid.csv --top 40 > $O/top.txt
  rm -rf $O/prof
done
