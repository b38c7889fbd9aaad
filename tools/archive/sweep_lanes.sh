#!/bin/bash
# Speculative lanes per deflate block (DQ_NDEC cap, DQ_SEGBITS minimum segment) on the current
# kernel: plain inflate timing on the 2M-record WGS file, two runs each.  usage: TAG "ndec,segbits"...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for cfg in "$@"; do
  nd=${cfg%,*}; sb=${cfg#*,}
  for r in 1 2; do
    DQ_NDEC=$nd DQ_SEGBITS=$sb timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/l_${nd}_${sb}_$r.log 2>&1
  done
  echo "ndec $nd segbits $sb: $(grep -h 'inflate ms' $out/l_${nd}_${sb}_*.log | awk '{print $4}' | tr '\n' ' ')"
done
