#!/bin/bash
# Warm-up bits (DQ_OV) of the speculative segments on the current kernel: plain inflate timing
# on the 2M-record WGS file, two runs per value.  usage: tools/sweep_ov3.sh TAG OV...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for ov in "$@"; do
  for r in 1 2; do
    DQ_OV=$ov timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/ov_${ov}_$r.log 2>&1
  done
  echo "ov $ov: $(grep -h 'inflate ms' $out/ov_${ov}_*.log | awk '{print $4}' | tr '\n' ' ')"
done
