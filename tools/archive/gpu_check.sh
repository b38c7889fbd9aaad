#!/bin/bash
# One GPU round trip for a kernel change: inflate phase timing on the 2M-record WGS file, the GPU
# test suite, and a short 12.5 GB bench run.  usage: tools/gpu_check.sh TAG [pytest args]
set -eo pipefail
tag=${1:-check}; shift || true
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain.log 2>&1
DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing.log 2>&1
grep -v "^bytes\|amdgpu.ids" $out/plain.log $out/timing.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --cpu-seconds 8 --e2e 0 --intervals 0 > $out/bench.log 2>&1
grep '"metric"' $out/bench.log > $out/bench.json
grep "step 2" $out/bench.log
