#!/bin/bash
# Per-phase inflate cycles (DQ_TIMING=1) and plain inflate ms for a list of environment settings,
# on the 2M-record WGS file.  usage: tools/gpu_phase_sweep.sh TAG "VAR=v VAR2=w" ...
set -eo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_$i.log 2>&1
  env $cfg DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_$i.log 2>&1
  echo "== [$cfg] $(grep -h 'inflate ms' $out/plain_$i.log | awk '{print $4}')"
  grep -h '\[dq\]' $out/timing_$i.log | head -2
done
