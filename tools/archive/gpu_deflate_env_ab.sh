#!/bin/bash
# A/B of DQ_DEFLATE settings on the 2M-record stream (tools/deflate_bench.py): phase cycles and a
# 3-rep bench per setting.  usage: tools/gpu_deflate_env_ab.sh TAG SETTING...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  echo "== DQ_DEFLATE=$v"
  DQ_DEFLATE=$v DQ_DEFLATE_TIMING=1 timeout -k 10 120 python3 -u tools/deflate_bench.py --records 2000000 --reps 1 > $out/timing_$v.log 2>&1
  grep "parse cycles" $out/timing_$v.log | tail -1
  DQ_DEFLATE=$v timeout -k 10 120 python3 -u tools/deflate_bench.py --records 2000000 --reps 3 > $out/bench_$v.log 2>&1
  grep '"ratio"' $out/bench_$v.log
done
