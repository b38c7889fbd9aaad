#!/bin/bash
# Resolve-phase breakdown and batch-shape sweep of the inflate kernel (2M-record WGS file).
set -eo pipefail
mkdir -p gpurun_out/r2m
for cfg in "4,1" "2,1" "8,1" "2,4"; do
  DQ_CFG=$cfg DQ_TIMING=1 timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 3 > gpurun_out/r2m/timing_$cfg.log 2>&1
  DQ_CFG=$cfg timeout -k 10 120 python3 -u tools/inflate_timing.py 2000000 3 > gpurun_out/r2m/plain_$cfg.log 2>&1
done
