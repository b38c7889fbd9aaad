#!/bin/bash
# Write path: ratio and speed over DQ_DEFLATE search settings (chain,lazy,nice,good,fmerge) on the 2M-record stream.
o=gpurun_out/${TAG:-r6w}; mkdir -p $o; export TMPDIR=/tmp
for cfg in ${CFGS:-32,16,32,8,1 24,16,32,8,1 16,16,32,8,1 32,8,32,8,1 32,16,24,8,1 32,16,32,4,1 24,12,24,6,1}; do
  DQ_DEFLATE=$cfg timeout -k 10 120 python3 -u tools/deflate_bench.py --records 2000000 --reps 3 > $o/b_$cfg.log 2>&1 || exit 1
  echo "$cfg $(grep '"ratio"' $o/b_$cfg.log)"
done
