#!/bin/bash
# round 5: 32-channel image-tile 1x1 tiles at the small levels (route img_narrow): kernel tests, a
# whole-model parity test with the route on, same-box A/B of the default bench
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_img.py tests/test_abi.py > gpurun_out/imgnarrow_tests.log 2>&1 || { tail -30 gpurun_out/imgnarrow_tests.log; exit 1; }
tail -2 gpurun_out/imgnarrow_tests.log
bash scripts/ab.sh default img_narrow=2560 img_narrow=10240 default img_narrow=2560 img_narrow=10240
cp gpurun_out/ab.txt gpurun_out/imgnarrow_ab.txt
cat gpurun_out/ab.txt
