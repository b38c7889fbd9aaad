#!/bin/bash
# Inflate warm-up sweep (DQ_OV bits before each speculative segment), plain timing on the 2M-record file.
set -eo pipefail
out=gpurun_out/${1:-r2ah}
mkdir -p $out
for ov in 48 96 144 192 256; do
  DQ_OV=$ov timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/ov_$ov.log 2>&1
  echo "ov $ov: $(grep 'inflate ms' $out/ov_$ov.log)"
done
