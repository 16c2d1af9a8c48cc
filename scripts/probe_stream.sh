#!/bin/bash
# conv_bench A/B of the streaming 1x1 kernel (HGK_STREAM) on the 64x64 shapes, with and without
# the fused BN transform / statistics epilogue
export TMPDIR=/tmp; mkdir -p gpurun_out/probe
O=gpurun_out/probe
: > $O/cb.txt
for s in 0 1; do
 for extra in "" "--nostats" "--nopre" "--nostats --nopre"; do
  echo "== STREAM=$s $extra" >> $O/cb.txt
  HGK_STREAM=$s timeout -k 10 120 python scripts/conv_bench.py --only "1x1" --modes fwd,dgrad $extra 2>&1 | grep -v "@" >> $O/cb.txt || exit 1
 done
done
cat $O/cb.txt
