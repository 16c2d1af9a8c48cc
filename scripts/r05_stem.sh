#!/bin/bash
# round 5: the row-tile stem kernel (route stem): tests, micro-benchmark (route 1 vs 0), same-box
# A/B of the default bench (stem=1 vs stem=0), primary then try_with_aspp
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_stem.py tests/test_gpu_pack.py tests/test_abi.py > gpurun_out/stem_tests.log 2>&1
tail -2 gpurun_out/stem_tests.log
timeout -k 10 120 python scripts/stem_bench.py > gpurun_out/stem_bench.txt 2>&1
cat gpurun_out/stem_bench.txt
bash scripts/ab.sh default stem=0 default stem=0 default stem=0
cp gpurun_out/ab.txt gpurun_out/stem_ab_primary.txt
cat gpurun_out/ab.txt
