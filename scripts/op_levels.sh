#!/bin/bash
set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ops
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ops -o run -- python3 scripts/op_profile.py --log gpurun_out/ops/calls.txt > gpurun_out/ops/run.log 2>&1
csv=$(find gpurun_out/ops -name "run_kernel_trace.csv" | head -1)
python3 scripts/op_profile.py --parse $csv --log gpurun_out/ops/calls.txt --top 120 > gpurun_out/ops/ops.txt
python3 scripts/level_breakdown.py gpurun_out/ops/ops.txt > gpurun_out/ops/levels.txt
rm -f $csv
