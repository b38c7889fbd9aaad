#!/bin/bash
# A/B of runtime settings (environment variables) of the current library: plain inflate timings,
# interleaved, twice, on the WGS file of DQ_N records (default 2M).
# usage: [DQ_N=...] tools/gpu_env_ab.sh TAG "ENV=..." "ENV=..." ...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 120 python3 -u tools/inflate_timing.py ${DQ_N:-2000000} > $out/plain${rep}_$i.log 2>&1
    echo "$e rep$rep: $(grep 'inflate ms' $out/plain${rep}_$i.log)"
  done
done
