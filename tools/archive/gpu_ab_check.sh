#!/bin/bash
# Inflate tests on the current library, then an interleaved A/B against prebuilt variants.
# usage: tools/gpu_ab_check.sh TAG LIB...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_inflate_codes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
tail -2 $out/tests.log
bash tools/gpu_variant_ab.sh $tag "$@"
