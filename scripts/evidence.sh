#!/bin/bash
# Round evidence on the GPU box: default bench line, rocprofv3 kernel-trace stats of a bench run,
# and the two PMC passes for bench.py's roofline kernel (each in its own run).
# usage (from the repo root, via gpurun): bash scripts/evidence.sh <tag>
set -eo pipefail
tag=${1:-r01}
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default_$tag.txt 2>&1
tail -1 $O/bench_default_$tag.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench_$tag.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$tag -o run -- python3 $R/scripts/roofline_pmc.py run > $O/pmc_fetch_$tag.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$tag -o run -- python3 $R/scripts/roofline_pmc.py run > $O/pmc_write_$tag.log 2>&1
python3 scripts/roofline_pmc.py parse $O/pmc_fetch_$tag $O/pmc_write_$tag > $O/roofline_pmc_$tag.json
cat $O/roofline_pmc_$tag.json
