#!/bin/bash
# Per-step kernel tables of bench.py for two libhgk builds on one box (rocprofv3 kernel trace).
# usage: bash scripts/trace_ab.sh ab/a.so ab/b.so
export TMPDIR=/tmp
R=$(pwd)
for lib in "$@"; do
  t=$(basename $lib .so)
  O=$R/gpurun_out/trace_$t
  rm -rf $O; mkdir -p $O
  HGK_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 $R/bench.py --steps 12 --warmup 3 --no-cpu-baseline --dropin-steps 0 > $O/bench.txt 2>&1 || exit 1
  db=$(find $O/prof -name "run_results.db" | head -1)
  python3 scripts/db_stats.py $db --steps 10 --csv $O/step_kernel_stats.csv --top 30 > $O/table.txt || exit 1
  head -40 $O/table.txt
done
