#!/bin/bash
# Bench lines of every single-GPU BASELINE configuration (each under its own time limit):
#   configs[1] default line (+ fp32 leg, CPU baseline), configs[3] try_with_aspp bs16, configs[4]
#   8-stack 384 bs16 fp32.  usage: bash scripts/bench_configs.sh <tag>
set -eo pipefail
tag=${1:-r03}
O=gpurun_out/bench_$tag
mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/default.txt 2>&1
grep '^{' $O/default.txt
timeout -k 10 300 python -u bench.py --preset try_with_aspp --no-cpu-baseline > $O/aspp.txt 2>&1
grep '^{' $O/aspp.txt
timeout -k 10 300 python -u bench.py --stacks 8 --res 384 --batch 16 --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline --dropin-steps 0 > $O/stress.txt 2>&1
grep '^{' $O/stress.txt
