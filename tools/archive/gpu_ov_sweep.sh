#!/bin/bash
# Warm-up bits sweep (DQ_OV), plain timing twice each.  usage: tools/gpu_ov_sweep.sh TAG OV...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do for v in "$@"; do
  DQ_OV=$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/ov${v}_$rep.log 2>&1
done; done
for f in $out/*.log; do echo "$f $(grep -o 'inflate ms [0-9.]*' $f)"; done
