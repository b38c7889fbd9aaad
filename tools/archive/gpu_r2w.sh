#!/bin/bash
# Round-2 evidence after the pointer-jumping resolve: rocprof kernel trace of the default bench
# workload, the inflate kernel's HBM traffic (FETCH/WRITE passes) and its SQ counters.
set -eo pipefail
out=gpurun_out/${1:-r2w}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u bench.py --steps 3 --warmup 1 --cpu-seconds 1 --e2e 0 --intervals 0 > $out/prof_bench.log 2>&1
grep '"metric"' $out/prof_bench.log | tail -1 | cut -c1-300
bash tools/pmc_traffic.sh $out/traffic $out/traffic.json --e2e 0 --intervals 0 > $out/traffic.log 2>&1
head -c 400 $out/traffic.json; echo
bash tools/pmc_inflate.sh $out/sq 2000000 > $out/sq.log 2>&1
cat $out/sq.log | tail -40
