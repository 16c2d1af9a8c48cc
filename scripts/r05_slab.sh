#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
BENCH_ARGS="--preset hourglass_compare" bash scripts/ab.sh default wg_slab_x10=10 wg_slab_x10=5 default wg_slab_x10=10 wg_slab_x10=5 && cp gpurun_out/ab.txt gpurun_out/slab_ab_hgc.txt && cat gpurun_out/slab_ab_hgc.txt
bash scripts/ab.sh default wg_slab_x10=10 wg_slab_x10=5 default wg_slab_x10=10 wg_slab_x10=5 && cp gpurun_out/ab.txt gpurun_out/slab_ab_primary.txt && cat gpurun_out/slab_ab_primary.txt
