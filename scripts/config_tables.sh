#!/bin/bash
# rocprofv3 per-step kernel tables of the non-headline single-GPU configurations
# (configs[3] try_with_aspp bs16 bf16, configs[4] 8-stack 384 bs16 fp32). usage: bash scripts/config_tables.sh <tag>
set -eo pipefail
tag=${1:-r03}
R=$(pwd)
O=$R/gpurun_out/tables_$tag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/aspp -o run -- python3 $R/bench.py --preset try_with_aspp --steps 12 --warmup 3 --no-cpu-baseline --dropin-steps 0 > $O/aspp.txt 2>&1
python3 scripts/db_stats.py $(find $O/aspp -name "run_results.db" | head -1) --steps 10 --csv $O/aspp_step_kernel_stats.csv --top 15
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stress -o run -- python3 $R/bench.py --stacks 8 --res 384 --batch 16 --dtype fp32 --steps 8 --warmup 2 --no-cpu-baseline --dropin-steps 0 > $O/stress.txt 2>&1
python3 scripts/db_stats.py $(find $O/stress -name "run_results.db" | head -1) --steps 6 --csv $O/stress_step_kernel_stats.csv --top 15
