#!/bin/bash
# usage: ab.sh "ENV1=a ENV2=b" "ENV3=c" ...   (runs bench per config, on the GPU box)
mkdir -p gpurun_out; : > gpurun_out/ab.txt
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/ab.txt
  env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 > gpurun_out/ab_one.log 2>&1 || { echo FAIL >> gpurun_out/ab.txt; tail -5 gpurun_out/ab_one.log >> gpurun_out/ab.txt; exit 1; }
  python -c "import json,sys; l=[x for x in open('gpurun_out/ab_one.log') if x.startswith('{')][-1]; d=json.loads(l); print(d['value'], d['ms_per_step'])" >> gpurun_out/ab.txt
done
