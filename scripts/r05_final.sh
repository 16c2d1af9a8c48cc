#!/bin/bash
# round 5 final evidence on one box: new-route tests + A/Bs, then the evidence run (default bench,
# rocprof step table, PMC passes), preset bench lines and per-preset step tables
set -o pipefail
mkdir -p gpurun_out
bash scripts/r05_pairblocks.sh || exit 1
BENCH_ARGS="--preset train" bash scripts/ab.sh default pair_blocks=0 default pair_blocks=0 && cp gpurun_out/ab.txt gpurun_out/pairblocks_ab_train.txt && cat gpurun_out/pairblocks_ab_train.txt || exit 1
bash scripts/evidence.sh r05b || exit 1
bash scripts/r05_presets.sh || exit 1
bash scripts/r05_presetprof.sh hourglass_compare try_with_aspp || exit 1
