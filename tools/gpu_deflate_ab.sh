#!/bin/bash
# A/B of deflate builds: each argument names a prebuilt library under disq_amd/_build/; for each,
# the write-path tests (first library only), phase cycles and a 3-rep bench of the 2M-record
# stream at DQ_DEFLATE (default setting if unset).  usage: tools/gpu_deflate_ab.sh TAG LIB...
# (list a library twice, alternating, for an interleaved A/B)
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
DQ_GPU_LIB=$PWD/disq_amd/_build/$1 timeout -k 10 300 python3 -u -m pytest tests/test_deflate_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/deflate_tests.log 2>&1 || { tail -30 $out/deflate_tests.log; exit 1; }
tail -1 $out/deflate_tests.log
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== $i $v"
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v DQ_DEFLATE_TIMING=1 timeout -k 10 120 python3 -u tools/deflate_bench.py --records 2000000 --reps 1 > $out/timing_${i}_$v.log 2>&1
  grep "cycles" $out/timing_${i}_$v.log | tail -3
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 120 python3 -u tools/deflate_bench.py --records 2000000 --reps 3 > $out/bench_${i}_$v.log 2>&1
  grep '"ratio"' $out/bench_${i}_$v.log
done
