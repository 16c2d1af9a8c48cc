#!/bin/bash
# ring_bench.py over libhgk ablation builds (HGK_LIB), one box. usage: bash scripts/ring_ablate.sh ablib/*.so
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  HGK_LIB=$lib timeout -k 10 120 python scripts/ring_bench.py --reps 20 || exit 1
done
