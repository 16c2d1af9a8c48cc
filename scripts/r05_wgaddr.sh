#!/bin/bash
# round 5: halo weight-grad address precompute (+ optional wave priority): bitwise tests, per-launch, same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wgrad_dma.py tests/test_gpu_conv_bf16.py > gpurun_out/wgaddr_tests.log 2>&1 || { tail -40 gpurun_out/wgaddr_tests.log; exit 1; }
tail -2 gpurun_out/wgaddr_tests.log
for l in abx/base.so abx/addr.so abx/prio.so; do
  echo "== $l"; (cd scripts && HGK_LIB=../$l timeout -k 10 200 python -u wgrad_dma_bench.py 2>&1 | grep ",0," | head -4) || exit 1
done
ROUNDS=3 bash scripts/ablibs.sh abx/base.so abx/addr.so abx/prio.so
