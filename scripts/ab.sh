#!/bin/bash
# usage: ab.sh "route1=a,route2=b" "route3=c" ...   (bench.py --route per config, on the GPU box;
# "default" = the compiled routes; BENCH_ARGS: extra bench.py arguments, e.g. "--preset try_with_aspp")
mkdir -p gpurun_out; : > gpurun_out/ab.txt
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/ab.txt
  r=$cfg; [ "$r" = default ] && r=""
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 $BENCH_ARGS --route "$r" > gpurun_out/ab_one.log 2>&1 || { echo FAIL >> gpurun_out/ab.txt; tail -5 gpurun_out/ab_one.log >> gpurun_out/ab.txt; exit 1; }
  python -c "import json,sys; l=[x for x in open('gpurun_out/ab_one.log') if x.startswith('{')][-1]; d=json.loads(l); print(d['value'], d['ms_per_step'])" >> gpurun_out/ab.txt
done
