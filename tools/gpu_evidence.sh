#!/bin/bash
# Evidence for the current inflate kernel: rocprof kernel trace + stats of the default bench
# workload, HBM traffic of the inflate kernel (FETCH/WRITE passes over the same workload) and its
# SQ counters (five passes over the 2M-record file).  usage: tools/gpu_evidence.sh TAG
set -eo pipefail
out=gpurun_out/${1:-evidence}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 -u bench.py --steps 3 --warmup 1 --cpu-seconds 1 --e2e 0 --intervals 0 > $out/prof_bench.log 2>&1
grep '"metric"' $out/prof_bench.log | tail -1 > $out/prof_bench.json
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -6 $out/kernel_stats.csv | cut -c1-200
timeout -k 10 900 bash tools/pmc_traffic.sh $out/traffic $out/traffic.json --e2e 0 --intervals 0 > $out/traffic.log 2>&1
head -c 600 $out/traffic.json; echo
timeout -k 10 600 bash tools/pmc_inflate.sh $out/sq 2000000 > $out/sq.log 2>&1
tail -32 $out/sq.log
