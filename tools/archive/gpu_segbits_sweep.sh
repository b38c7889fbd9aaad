#!/bin/bash
# Inflate sweep of the minimum speculative segment (DQ_SEGBITS: only deflate blocks with fewer than
# 512 x SEGBITS bits, i.e. the small second block of most BGZF blocks, are affected) and of the
# warm-up (DQ_OV), with per-deflate-block phase cycles.  usage: tools/gpu_segbits_sweep.sh TAG
set -eo pipefail
tag=${1:-segbits}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for cfg in "128 96" "64 96" "48 96" "32 96" "96 96" "192 96" "64 64" "48 64"; do
  set -- $cfg
  DQ_SEGBITS=$1 DQ_OV=$2 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_$1_$2.log 2>&1
  DQ_TIMING=1 DQ_SEGBITS=$1 DQ_OV=$2 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$1_$2.log 2>&1
  echo "seg=$1 ov=$2: $(grep 'inflate ms' $out/plain_$1_$2.log | cut -c1-40)"
  grep "first deflate" $out/timing_$1_$2.log
done
