#!/bin/bash
# The device bounds-checked build (make -C disq_amd/csrc checked, -DDQ_CHECKED): the inflate,
# parity and adversarial GPU tests under libdisq_gpu_checked.so; the session fails on any failed
# device check (tests/conftest.py).  usage: tools/gpu_checked_tests.sh TAG
set -eo pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp DQ_GPU_LIB=$PWD/disq_amd/_build/libdisq_gpu_checked.so
timeout -k 10 900 python3 -u -m pytest tests/test_inflate_codes.py tests/test_gpu_parity.py \
  tests/test_adversarial.py tests/test_chunk_decode.py tests/test_text_gpu.py tests/test_deflate_gpu.py tests/test_tail_handoff.py \
  -m gpu -v -s --timeout 300 --timeout-method thread > $out/checked_tests.log 2>&1 || { tail -40 $out/checked_tests.log; exit 1; }
grep -h "DQ_CHECKED\|passed\|failed" $out/checked_tests.log | tail -3
