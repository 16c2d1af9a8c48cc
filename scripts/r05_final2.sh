#!/bin/bash
# round 5 final build: default bench line, then hourglass_compare / try_with_aspp lines (30 steps)
set -eo pipefail
mkdir -p gpurun_out/final2
timeout -k 10 400 python -u bench.py > gpurun_out/final2/bench_default.txt 2>&1
grep '^{' gpurun_out/final2/bench_default.txt | head -1 | cut -c1-160
for p in hourglass_compare try_with_aspp; do
  timeout -k 10 240 python bench.py --preset $p --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 > gpurun_out/final2/$p.txt 2>&1
  grep '^{' gpurun_out/final2/$p.txt | head -1 | cut -c1-120
done
