#!/bin/bash
# Round evidence on the GPU box (each GPU step under its own time limit, chained with &&):
#   1. the default bench line;
#   2. rocprofv3 kernel trace of a bench run -> per-step kernel table (scripts/db_stats.py);
#   3. three PMC passes over two eager training steps (FETCH_SIZE / WRITE_SIZE / SQ+GRBM) ->
#      per-kernel HBM bytes, MFMA busy and wave-state fractions (scripts/pmc_top.py).
# usage (repo root, via gpurun): bash scripts/evidence.sh <tag> [skip_bench]
set -eo pipefail
tag=${1:-r02}
R=$(pwd)
O=$R/gpurun_out/ev_$tag
mkdir -p $O
export TMPDIR=/tmp
if [ "$2" != "skip_bench" ]; then
  timeout -k 10 400 python -u bench.py > $O/bench_default.txt 2>&1
  grep '^{' $O/bench_default.txt
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-leg --dropin-steps 0 > $O/prof_bench.txt 2>&1
db=$(find $O/prof -name "run_results.db" | head -1)
python3 scripts/db_stats.py $db --steps 10 --csv $O/step_kernel_stats.csv --by-grid $O/step_kernel_stats_by_grid.csv --top 25
# bench.py's roofline launches under the profiler (cold: after the flush; warm: back-to-back runs)
# next to the line the same run printed (its live HIP-event averages)
python3 scripts/rocprof_stats.py $db --csv $O/rocprof_kernel_stats.csv --run 20 > $O/rocprof_roofline_runs.txt
grep '^{' $O/prof_bench.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (d[k] or {}).get('avg_us') for k in ('roofline','roofline_second','roofline_mfma','roofline_wgrad')}, {k: (d[k] or {}).get('warm_us') for k in ('roofline','roofline_second','roofline_mfma','roofline_wgrad')})" >> $O/rocprof_roofline_runs.txt
cat $O/rocprof_roofline_runs.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/scripts/pmc_top.py run > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/scripts/pmc_top.py run > $O/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq -o run -- python3 $R/scripts/pmc_top.py run > $O/pmc_sq.log 2>&1
python3 scripts/pmc_top.py parse $O/pmc_fetch $O/pmc_write $O/pmc_sq $O/step_kernel_stats.csv > $O/pmc_top.json
python3 -c "
import json; d=json.load(open('$O/pmc_top.json'))
for r in d['kernels'][:12]:
    f=lambda v: 'na' if v is None else '%.3f'%v
    print('%8.1f us %6.0f GB/s fabric %s mfma %s wait %s %s' % (r['us_per_step'], r['fabric_GBps'] or 0, f(r['fabric_frac_of_8TBps']), f(r['mfma_busy_frac']), f(r['wave_wait_any_frac']), r['kernel'][:70]))
"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/roof_fetch -o run -- python3 $R/scripts/roofline_pmc.py run > $O/roof_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/roof_write -o run -- python3 $R/scripts/roofline_pmc.py run > $O/roof_write.log 2>&1
python3 scripts/roofline_pmc.py parse $O/roof_fetch $O/roof_write > $O/roofline_pmc.json
cat $O/roofline_pmc.json
