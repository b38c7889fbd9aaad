#!/bin/bash
# A/B of compile-time kernel variants: each argument names a prebuilt library under
# disq_amd/_build/ (e.g. libdisq_gpu.so libdisq_gpu_b.so); plain + phase timing for each, twice,
# interleaved.  usage: tools/gpu_variant_ab.sh TAG LIB...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain${rep}_$v.log 2>&1
  done
done
for v in "$@"; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$v.log 2>&1
done
for f in $out/*.log; do echo "== $f"; grep -v "^bytes\|amdgpu.ids" $f || true; done
