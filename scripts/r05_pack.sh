#!/bin/bash
# round 5: 8-element weight packing: bitwise test, same-box A/B (hourglass_compare, primary),
# then the hourglass_compare step table on the new build
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_pack.py tests/test_gpu_twin.py > gpurun_out/pack_tests.log 2>&1
tail -2 gpurun_out/pack_tests.log
BENCH_ARGS="--preset hourglass_compare" ROUNDS=3 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/pack_ab_hgc.txt
ROUNDS=2 bash scripts/ablibs.sh abx/old.so abx/new.so
cp gpurun_out/ablibs.txt gpurun_out/pack_ab_primary.txt
bash scripts/r05_stepdump.sh hourglass_compare
grep -E "pack_weight|reduce_multi" gpurun_out/sd_hourglass_compare/top.txt
