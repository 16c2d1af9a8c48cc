#!/bin/bash
# Same-box A/B of libhgk builds: alternates bench.py runs over the given .so files (HGK_LIB),
# ROUNDS times, so box-to-box spread (~2 %) does not decide. Each run under its own time limit.
# usage (GPU box): ROUNDS=3 bash scripts/ablibs.sh ab/base.so ab/new.so [...]   (BENCH_ARGS: extra bench.py args)
mkdir -p gpurun_out
out=gpurun_out/ablibs.txt
: > $out
rounds=${ROUNDS:-3}
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    HGK_LIB=$lib timeout -k 10 150 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
      --no-fp32-leg --dropin-steps 0 $BENCH_ARGS > gpurun_out/ab_one.log 2>&1 || { echo "FAIL $lib" >> $out; tail -5 gpurun_out/ab_one.log >> $out; exit 1; }
    python -c "import json,sys; l=[x for x in open('gpurun_out/ab_one.log') if x.startswith('{')][-1]; d=json.loads(l); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline_mfma']['avg_us'])" >> $out
  done
done
cat $out
