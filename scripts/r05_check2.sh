#!/bin/bash
# GPU suite (minus the configs[4] N=16 fixture test while its reference draws are regenerated),
# one bench line, then the wg_full A/B.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  --deselect "tests/test_gpu_configs.py::test_model_8stack_384_batch_fp32_vs_reference_fixture[16]" \
  > gpurun_out/gputests.log 2>&1 || { tail -60 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 \
  || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
bash scripts/r05_ab1.sh
