#!/bin/bash
# ring tests (4-wave small routes included), then the batch-32 bf16 model test under the ring
# variants (its grad-norm gate is bf16-noise sensitive: compare margins)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py || exit 1
for cfg in "HGK_RING_NW=8" "HGK_RING_NW=4 HGK_RING_SMALL=0" "HGK_RING_NW=4"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u -m pytest -q -s --timeout 150 --timeout-method thread \
    "tests/test_gpu_parity.py::test_model_batch32_bf16_vs_reference_fixture" 2>&1 | grep -E "bf16|passed|failed|Error" 
done
exit 0
