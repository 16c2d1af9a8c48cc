#!/bin/bash
# round-5 bench lines of the other BASELINE configs and presets (each under its own time limit)
mkdir -p gpurun_out/presets
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 "$@" \
    > gpurun_out/presets/$n.log 2>&1 || { echo "FAIL $n"; tail -20 gpurun_out/presets/$n.log; return 1; }
  grep '^{' gpurun_out/presets/$n.log > gpurun_out/presets/$n.json
  python -c "import json; d=json.load(open('gpurun_out/presets/$n.json')); print('$n', d['value'], d['ms_per_step'], (d.get('step_roofline') or {}).get('frac'))"
}
run try_more_layer --preset try_more_layer && run train --preset train && \
run try_with_aspp --preset try_with_aspp && run hourglass_compare --preset hourglass_compare && \
run stress8x384 --stacks 8 --res 384 --batch 16 --dtype fp32
