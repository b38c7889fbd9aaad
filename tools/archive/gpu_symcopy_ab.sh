#!/bin/bash
# GPU suite + inflate A/B of the symbol-copy emit (DQ_SYMCOPY=1 default vs 0: decode again), with
# DQ_TIMING phase cycles of both.  usage: tools/gpu_symcopy_ab.sh TAG
set -eo pipefail
tag=${1:-symcopy}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -30 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
for i in 1 2; do
  for v in 1 0; do
    DQ_SYMCOPY=$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_${v}_$i.log 2>&1
    echo "symcopy=$v: $(grep 'inflate ms' $out/plain_${v}_$i.log)"
  done
done
for v in 1 0; do
  DQ_TIMING=1 DQ_SYMCOPY=$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$v.log 2>&1
  echo "symcopy=$v:"; grep "\[dq\]" $out/timing_$v.log
done
