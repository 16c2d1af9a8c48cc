#!/bin/bash
# halo weight-grad micro-benchmark over libhgk builds, then the parity tests of the main build
mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  HGK_LIB=$lib timeout -k 10 120 python scripts/wgrad_bench.py --halo || exit 1
done
