#!/bin/bash
# Per-step kernel tables of bench.py under two route settings on one box (rocprofv3 kernel
# trace). usage: bash scripts/trace_env_ab.sh "route=a" "default"   (bench.py --route)
export TMPDIR=/tmp
R=$(pwd)
i=0
for cfg in "$@"; do
  i=$((i + 1))
  O=$R/gpurun_out/trace_env$i
  rm -rf $O; mkdir -p $O
  echo "== $cfg" > $O/table.txt
  r=$cfg; [ "$r" = default ] && r=""
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run -- python3 $R/bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 --route "$r" > $O/bench.txt 2>&1 || exit 1
  db=$(find $O/prof -name "run_results.db" | head -1)
  python3 scripts/db_stats.py $db --steps 10 --csv $O/step_kernel_stats.csv --top 40 >> $O/table.txt || exit 1
  rm -rf $O/prof
  head -45 $O/table.txt
done
