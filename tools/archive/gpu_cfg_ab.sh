#!/bin/bash
# A/B of inflate tuning configs (DQ_CFG) on the 2M-record WGS file: plain and phase timing for
# each, and the GPU parity suite under the last config.  usage: tools/gpu_cfg_ab.sh TAG CFG...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for cfg in "$@"; do
  DQ_CFG=$cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_$cfg.log 2>&1
  DQ_TIMING=1 DQ_CFG=$cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$cfg.log 2>&1
  DQ_CFG=$cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain2_$cfg.log 2>&1
done
for f in $out/*.log; do echo "== $f"; grep -v "^bytes\|amdgpu.ids" $f; done
DQ_CFG=$cfg timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/parity.log 2>&1
tail -1 $out/parity.log
