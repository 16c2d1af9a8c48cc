#!/bin/bash
# ring kernel: 8-wave (one workgroup per CU) vs 4-wave (two per CU) workgroups, one box.
# parity of the 4-wave build first, then the micro-benchmark alternated twice
mkdir -p gpurun_out
HGK_RING_NW=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ring.py tests/test_gpu_conv_bf16.py tests/test_gpu_fold_apply.py || exit 1
for r in 1 2; do
  for nw in 8 4; do
    echo "== NW $nw (round $r)"
    HGK_RING_NW=$nw timeout -k 10 120 python scripts/ring_bench.py --reps 20 || exit 1
  done
done
