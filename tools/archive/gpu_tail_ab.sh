#!/bin/bash
# The tail kernel A/B: GPU tests on the current library, then plain + phase timing of the current
# library, the same with DQ_TAIL=0 (no tail kernel) and a reference build.  usage: TAG REFLIB
set -eo pipefail
tag=$1; ref=$2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain${rep}_tail.log 2>&1
  DQ_TAIL=0 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain${rep}_notail.log 2>&1
  DQ_GPU_LIB=$PWD/disq_amd/_build/$ref timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain${rep}_ref.log 2>&1
done
DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_tail.log 2>&1
for f in $out/plain*.log $out/timing*.log; do echo "== $f"; grep -v "^bytes\|amdgpu.ids" $f || true; done
