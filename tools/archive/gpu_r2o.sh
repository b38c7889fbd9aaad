#!/bin/bash
# Round-2 final evidence, part 1: the GPU test suite, the rocprof kernel trace of the default
# bench workload (12.5 GB, N = 1), and the inflate kernel's HBM traffic by PMC on that workload.
set -eo pipefail
out=gpurun_out/r2o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u bench.py --steps 3 --warmup 1 --cpu-seconds 1 --e2e 0 --intervals 0 > $out/prof_bench.log 2>&1
grep '"metric"' $out/prof_bench.log | tail -1 | cut -c1-200
bash tools/pmc_traffic.sh $out/traffic $out/traffic.json --e2e 0 --intervals 0 > $out/traffic.log 2>&1
cat $out/traffic.json | head -5
