#!/bin/bash
# Phase cycles of the inflate kernels at two block workgroups per CU (default) and at one
# (DQ_LDSPAD=80000 pads the dynamic LDS; a -DDQ_TUNING build: DQ_GPU_LIB=.../libdisq_gpu_tune.so): equal per-block cycles mean latency-bound phases.
# usage: tools/gpu_occupancy_probe.sh TAG
set -eo pipefail
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
for pad in 0 80000; do
  DQ_LDSPAD=$pad DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/timing_pad$pad.log 2>&1
  DQ_LDSPAD=$pad timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 > $out/plain_pad$pad.log 2>&1
  echo "== pad $pad"; grep "phase cycles" $out/timing_pad$pad.log | tail -1; grep "inflate ms" $out/plain_pad$pad.log
done
