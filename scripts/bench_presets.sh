#!/bin/bash
# Bench lines of every preset / BASELINE configuration other than the headline, on this build
# (each under its own time limit; 30 timed steps after 5 warm-up steps, steady state per
# profiles/r06_train_step_times.txt). usage (GPU box): bash scripts/bench_presets.sh <tag>
set -eo pipefail
O=gpurun_out/presets_${1:-r06}
mkdir -p $O
for p in try_with_aspp hourglass_compare try_more_layer train; do
  timeout -k 10 300 python -u bench.py --preset $p --steps 30 --warmup 5 --no-cpu-baseline --no-fp32-leg \
    --dropin-steps 0 > $O/$p.txt 2>&1
  grep '^{' $O/$p.txt > $O/$p.json
  python -c "import json; d=json.load(open('$O/$p.json')); print('$p', d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('frac'))"
done
timeout -k 10 400 python -u bench.py --stacks 8 --res 384 --batch 16 --dtype fp32 --steps 10 --warmup 3 \
  --no-cpu-baseline --dropin-steps 0 > $O/stress8x384.txt 2>&1
grep '^{' $O/stress8x384.txt > $O/stress8x384.json
python -c "import json; d=json.load(open('$O/stress8x384.json')); print('configs[4]', d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('frac'))"
