#!/bin/bash
# Tail-kernel round (r6r): inflate/tail GPU tests under the product and the checked build, then the
# interleaved A/B of the product against the listed variants (tools/gpu_variant_ab.sh: plain and
# DQ_TIMING phase cycles).  usage: tools/gpu_tail_ab.sh TAG VARIANT_LIB...
set -eo pipefail
tag=$1; shift
o=gpurun_out/$tag; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_inflate_codes.py tests/test_tail_handoff.py -m gpu -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_checked.so timeout -k 10 500 python3 -u -m pytest tests/test_inflate_codes.py tests/test_tail_handoff.py -m gpu -q --timeout 300 --timeout-method thread > $o/checked_tests.log 2>&1 || { tail -30 $o/checked_tests.log; exit 1; }
tail -1 $o/checked_tests.log
tools/gpu_variant_ab.sh $tag libdisq_gpu.so "$@" | grep -E "==|inflate ms|tail kernel" 
