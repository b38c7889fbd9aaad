#!/bin/bash
# Inflate phase timing (DQ_TIMING=1) on the 2M-record WGS file, default config.
set -eo pipefail
out=gpurun_out/${1:-r2u}
mkdir -p $out
export TMPDIR=/tmp
for cfg in ${CFGS:-4,1}; do
  DQ_CFG=$cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_$cfg.log 2>&1
  DQ_TIMING=1 DQ_CFG=$cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$cfg.log 2>&1
done
for f in $out/*.log; do echo "== $f"; grep -v "^bytes" $f; done
