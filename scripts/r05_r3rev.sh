#!/bin/bash
# round 5: row-streaming 3x3 with alternating row order (L2-shared boundary rows): tests, PMC traffic, A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_row3.py tests/test_gpu_fold_apply.py > gpurun_out/r3rev_tests.log 2>&1 || { tail -40 gpurun_out/r3rev_tests.log; exit 1; }
tail -2 gpurun_out/r3rev_tests.log
for v in norev rev; do
  HGK_LIB=abx/$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3_$v/f -o run -- python3 scripts/roofline_pmc.py run > gpurun_out/r3_$v.flog 2>&1 || exit 1
  HGK_LIB=abx/$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3_$v/w -o run -- python3 scripts/roofline_pmc.py run > gpurun_out/r3_$v.wlog 2>&1 || exit 1
  python3 scripts/roofline_pmc.py parse gpurun_out/r3_$v/f gpurun_out/r3_$v/w > gpurun_out/r3_$v.json && echo "== $v" && cat gpurun_out/r3_$v.json
done
ROUNDS=3 bash scripts/ablibs.sh abx/norev.so abx/rev.so
