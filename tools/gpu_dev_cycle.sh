#!/bin/bash
# One development cycle on the GPU box: smoke, the inflate/parity GPU tests, then an interleaved
# A/B of prebuilt libraries (tools/gpu_variant_ab.sh).  Stops at the first failure.
# usage: tools/gpu_dev_cycle.sh TAG "pytest -k expr or empty" LIB...
set -eo pipefail
tag=$1; sel=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
if [ -n "$sel" ]; then k=(-k "$sel"); else k=(); fi
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_inflate_codes.py tests/test_tail_handoff.py tests/test_deflate_gpu.py tests/test_arena.py -m gpu -x -v \
  --timeout 120 --timeout-method thread "${k[@]}" > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
if [ $# -gt 0 ]; then tools/gpu_variant_ab.sh $tag "$@"; fi
