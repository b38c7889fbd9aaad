#!/bin/bash
# A/B of LLVM scheduling strategies for the library (variants built by tools/build_variant.sh):
# interleaved inflate timing, then the inflate + parity GPU tests under each variant.
# usage: tools/gpu_sched_ab.sh TAG LIB...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
bash tools/gpu_variant_ab.sh $tag libdisq_gpu.so "$@"
for v in "$@"; do
  DQ_GPU_LIB=$PWD/disq_amd/_build/$v timeout -k 10 300 python3 -u -m pytest tests/test_inflate_codes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests_$v.log 2>&1
  echo "$v: $(tail -1 $out/tests_$v.log)"
done
