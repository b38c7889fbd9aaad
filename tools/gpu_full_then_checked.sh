#!/bin/bash
# The whole -m gpu suite on the product library, then the device bounds-checked run.
# usage: tools/gpu_full_then_checked.sh TAG
set -eo pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
tools/gpu_checked_tests.sh $tag
