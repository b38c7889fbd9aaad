#!/bin/bash
# Plain inflate timing on the 2M-record WGS file under environment settings, two runs each.
# usage: tools/sweep_env.sh TAG "VAR=value ..." ...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  for r in 1 2; do
    env $cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/c${i}_$r.log 2>&1
  done
  echo "$cfg: $(grep -h 'inflate ms' $out/c${i}_*.log | awk '{print $4}' | tr '\n' ' ')"
done
