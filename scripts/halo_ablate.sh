#!/bin/bash
# 3x3 halo conv micro-benchmark (fwd / input-grad, 64x64 / 32x32 / 16x16) over libhgk builds
for lib in "$@"; do
  echo "== $lib"
  HGK_LIB=$lib timeout -k 10 120 python scripts/conv_bench.py --only "3x3" --modes fwd,dgrad --graph --reps 20 || exit 1
done
