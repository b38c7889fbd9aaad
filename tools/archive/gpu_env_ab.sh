#!/bin/bash
# A/B of one environment switch of the library on the 2M-record WGS file: plain and phase timing
# for each value, then the whole GPU suite under the default environment.
# usage: tools/gpu_env_ab.sh TAG VAR VALUE...   (TESTS=0 skips the suite)
set -eo pipefail
tag=$1; var=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for v in "$@"; do
  env $var=$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_$v.log 2>&1
  env $var=$v DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$v.log 2>&1
  env $var=$v timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain2_$v.log 2>&1
done
for f in $out/*.log; do echo "== $f"; grep -v "^bytes\|amdgpu.ids" $f || true; done
if [ "${TESTS:-1}" != 0 ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
  tail -2 $out/gpu_tests.log
fi
